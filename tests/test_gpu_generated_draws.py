"""Generated-draw mode at the variate level: the K <= 32 kernels draw their Philox variates in
place (Z / X normals in the draw kernels, loading normals and psi / ps gammas in k_lambda,
delta gammas in the delta chain) and the wide kernels read k_draws buffers.  Every variate is
addressed by its counter (site, shard, row, index, iteration; csrc/philox.h), so a chain in
generated mode must be BITWISE the chain run in injected mode on the variates dcfm_rng_fill
produces at those counters (row = i / 32, index = i % 32: a fill of rows x 32 is the row's
first 32 indices; dcfm_rng_fill_rows with width K reaches the wide kernels' indices up to 127).
This pins the in-place draws of both paths to the counter scheme the RNG tests check statistically
(tests/test_gpu_rng.py).
"""
import numpy as np
import pytest

from helpers import make_case, state_dict

pytestmark = pytest.mark.gpu

SITE_Z, SITE_X, SITE_LAMBDA, SITE_PSI, SITE_DELTA, SITE_PS = 1, 2, 3, 4, 5, 6


def _rows(dcfm, kind, rows, seed, site, shard, it, K, shape=1.0):
    """rows x K block of variates at (site, shard, row, index < K, it)."""
    if K <= 32:
        x = dcfm.rng_fill(kind, rows * 32, seed=seed, shape=shape, site=site, shard=shard, iteration=it)
        return x.reshape(rows, 32)[:, :K]
    x = dcfm.rng_fill(kind, rows * K, seed=seed, shape=shape, site=site, shard=shard, iteration=it, width=K)
    return x.reshape(rows, K)


def _draws(dcfm, seed, n, P, g, K, first, T, hyper):
    NZ = np.zeros((K, n, g, T)); NX = np.zeros((K, n, T)); NL = np.zeros((K, P, g, T))
    Gpsi = np.zeros((P, K, g, T)); Gdelta = np.zeros((K, g, T)); Gps = np.zeros((P, g, T))
    for t in range(T):
        it = first + t
        NX[:, :, t] = _rows(dcfm, "normal", n, seed, SITE_X, 0, it, K).T
        for m in range(g):
            NZ[:, :, m, t] = _rows(dcfm, "normal", n, seed, SITE_Z, m, it, K).T
            NL[:, :, m, t] = _rows(dcfm, "normal", P, seed, SITE_LAMBDA, m, it, K).T
            Gpsi[:, :, m, t] = _rows(dcfm, "gamma", P, seed, SITE_PSI, m, it, K, shape=hyper.df / 2 + 0.5)
            Gps[:, m, t] = _rows(dcfm, "gamma", P, seed, SITE_PS, m, it, 1, shape=hyper.as_ + n / 2)[:, 0]
        for m in range(g):       # delta: every shard (replicated chain); shapes depend on h (dc:158,163): row 0, index h
            for h in range(K):
                shp = hyper.ad1 + P * K / 2 if h == 0 else hyper.ad2 + P * (K - h) / 2
                Gdelta[h, m, t] = _rows(dcfm, "gamma", 1, seed, SITE_DELTA, m, it, K, shape=shp)[0, h]
    return dict(NZ=NZ, NX=NX, NL=NL, Gpsi=Gpsi, Gdelta=Gdelta, Gps=Gps)


@pytest.mark.parametrize("n,p,g,K", [(40, 60, 4, 5), (50, 96, 8, 30), (36, 64, 2, 32), (44, 80, 4, 20), (30, 52, 4, 13),
                                     (80, 96, 4, 40), (150, 128, 2, 100)])
def test_generated_equals_injected_at_the_counters(dcfm, n, p, g, K):
    seed, burnin, mcmc, thin = 77, 1, 3, 1
    N = burnin + mcmc
    c = make_case(n, p, g, K, seed=9)
    P = c["P"]
    st = {f: v for f, v in state_dict(c["st"]).items() if f != "eta"}
    out = []
    for inject in (False, True):
        smp = dcfm.Sampler(c["n"], P, g, K, c["rho"], burnin, mcmc, thin, seed=seed, inject_draws=inject)
        try:
            smp.set_data(c["Yd"])
            smp.set_state(st)
            if inject:
                smp.set_draws(_draws(dcfm, seed, c["n"], P, g, K, 1, N, dcfm.Hyper()), 1, N)
            smp.run(1, N)
            got = smp.get_state()
            got["Sig"] = smp.get_sigma()
            out.append(got)
        finally:
            smp.close()
    for f in out[0]:
        assert np.array_equal(out[0][f], out[1][f]), f"{f}: generated != injected at the same counters"
