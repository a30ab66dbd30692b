"""Full-size property tests on the GPU (sizes the CPU oracle cannot run).

c5 (BASELINE.json configs[4]): p = 100,096 (P = 391 x g = 256), n = 2,000, K = 30.
Sigmaout is 80 GB of fp64 and stays in HBM; it is read back in column stripes
(dcfm_get_sigma_cols).  With one saved sample, every entry has a closed form in
the sampler's own state (dc:184-192):
    Sigma[a][b] = (coef(a,b) * Lambda_a . Lambda_b + [a == b] omega_a) / effsamp,
    coef = 1 inside a shard block, rho across blocks,
so whole stripes are checked against the state returned by dcfm_get_state — a
size-independent check of the assembly, the tile ownership and the stripe read.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sigma_cols_expected(Lam, omega, P, rho, cols, effsamp):
    """Closed form of Sigmaout(:, cols) from Lambda (P x K x g) and omega (P x g)."""
    g = Lam.shape[2]
    L = np.concatenate([Lam[:, :, m] for m in range(g)], axis=0)      # p x K, permuted order (Q7)
    w = np.concatenate([omega[:, m] for m in range(g)])
    shard = np.arange(L.shape[0]) // P
    out = L @ L[cols].T                                                # p x len(cols)
    coef = np.where(shard[:, None] == shard[cols][None, :], 1.0, rho)
    out *= coef
    out[cols, np.arange(len(cols))] += w[cols]
    return out / effsamp


def _synthetic_state(dcfm, n, P, g, K, rho, seed):
    rng = np.random.default_rng(seed)
    p = P * g
    L0 = rng.standard_normal((p, 8)) * (rng.random((p, 8)) < 0.3)
    Y = rng.standard_normal((n, 8)) @ L0.T
    Y += rng.standard_normal((n, p)) * 0.7
    hyper = dcfm.Hyper()
    Yk, n, pk, P, K_, keep = dcfm.preprocess(Y, g, K * g)
    del Y
    init = dcfm.driver._HostInitDraws(seed, n, pk, g, K, hyper)
    Yd = dcfm.partition_standardize(Yk, g, init.varind)
    del Yk
    return Yd, dcfm.initial_state(n, P, K, g, rho, hyper, init)


@pytest.mark.parametrize("name,n,P,g,K", [
    ("c5", 2000, 391, 256, 30),          # BASELINE configs[4]: 80 GB Sigmaout
    ("c3_stripes", 1000, 312, 64, 30),    # stripe boundaries not aligned to tiles
])
def test_sigma_stripes_closed_form(dcfm, name, n, P, g, K):
    rho = 0.5
    Yd, st = _synthetic_state(dcfm, n, P, g, K, rho, seed=5)
    p = P * g
    burnin, mcmc, thin = 1, 1, 1                  # one saved sample (iteration 2), effsamp = 1
    smp = dcfm.Sampler(n, P, g, K, rho, burnin, mcmc, thin, seed=9)
    try:
        smp.set_data(Yd)
        del Yd
        smp.set_state({f: st[f] for f in dcfm.STATE_FIELDS if f != "eta"})
        smp.run(1, burnin + mcmc)
        got = smp.get_state(("Lambda", "omega"))
        assert np.all(np.isfinite(got["Lambda"])) and np.all(got["omega"] > 0)
        stripes = [(0, 64), (p // 2 - 37, 101), (p - 70, 70)]
        for c0, nc in stripes:
            S = smp.get_sigma_cols(c0, nc)
            cols = np.arange(c0, c0 + nc)
            E = _sigma_cols_expected(got["Lambda"], got["omega"], P, rho, cols, mcmc / thin)
            err = np.max(np.abs(S - E)) / np.max(np.abs(E))
            assert err < 1e-12, f"{name}: stripe {c0}+{nc} rel err {err:.3e}"
            # symmetry across the stripe's own square block
            blk = S[c0:c0 + nc, :]
            assert np.array_equal(blk, blk.T)
    finally:
        smp.close()


def test_full_get_equals_stripes(dcfm):
    """dcfm_get_sigma (internally striped) equals an explicit stripe read."""
    n, P, g, K, rho = 200, 96, 8, 12, 0.5
    Yd, st = _synthetic_state(dcfm, n, P, g, K, rho, seed=3)
    smp = dcfm.Sampler(n, P, g, K, rho, 2, 6, 2, seed=4)
    try:
        smp.set_data(Yd)
        smp.set_state({f: st[f] for f in dcfm.STATE_FIELDS if f != "eta"})
        smp.run(1, 8)
        S = smp.get_sigma()
        p = P * g
        assert np.array_equal(S, S.T)
        for c0, nc in ((0, 33), (100, 77), (p - 5, 5)):
            assert np.array_equal(S[:, c0:c0 + nc], smp.get_sigma_cols(c0, nc))
    finally:
        smp.close()


@pytest.mark.parametrize("name,n,P,g,K", [
    ("c3", 1000, 312, 64, 30),           # BASELINE configs[2] shape on one GPU
    ("c5", 2000, 391, 256, 30),          # BASELINE configs[4]: two 40 GB lower-triangle Sigmas
])
def test_batched_flush_full_size(dcfm, name, n, P, g, K):
    """The driver bench's assembly flush at full size (dc:180-196, Q8): burnin 0, MCMC 20,
    thin 5 in ONE dcfm_run, so the 4 saved samples are accumulated by one k_assemble launch with
    k extent 4K.  A second sampler with the same seed steps one iteration per dcfm_run (its
    sweep is the same chain, bitwise) and records Lambda / omega after every saved iteration;
    the batched chain's Sigmaout stripes must equal the closed form summed over those samples.
    Pins the batched-flush path (asm_batch > 1) at a BASELINE shape, not only at p <= 2,560."""
    rho = 0.5
    Yd, st = _synthetic_state(dcfm, n, P, g, K, rho, seed=7)
    p = P * g
    burnin, mcmc, thin = 0, 20, 5
    init = {f: st[f] for f in dcfm.STATE_FIELDS if f != "eta"}
    batched = dcfm.Sampler(n, P, g, K, rho, burnin, mcmc, thin, seed=21)
    stepped = dcfm.Sampler(n, P, g, K, rho, burnin, mcmc, thin, seed=21)
    try:
        for s in (batched, stepped):
            s.set_data(Yd)
            s.set_state(init)
        del Yd
        batched.run(1, burnin + mcmc)
        samples = []
        for it in range(1, burnin + mcmc + 1):
            stepped.run(it, 1)
            if it > burnin and it % thin == 0:
                samples.append(stepped.get_state(("Lambda", "omega")))
        assert batched.saved_samples() == len(samples) == mcmc // thin
        fin_b = batched.get_state(("Lambda", "ps", "tauh"))
        fin_s = stepped.get_state(("Lambda", "ps", "tauh"))
        for f in fin_b:
            assert np.array_equal(fin_b[f], fin_s[f]), f"{name}: the stepped chain left the batched one at {f}"
        for c0, nc in [(0, 64), (p // 2 - 37, 101), (p - 70, 70)]:
            S = batched.get_sigma_cols(c0, nc)
            cols = np.arange(c0, c0 + nc)
            E = sum(_sigma_cols_expected(sm["Lambda"], sm["omega"], P, rho, cols, mcmc / thin) for sm in samples)
            err = np.max(np.abs(S - E)) / np.max(np.abs(E))
            assert err < 1e-12, f"{name}: batched stripe {c0}+{nc} rel err {err:.3e}"
            # the stepped chain flushed one sample per run: same Sigmaout up to summation order
            S1 = stepped.get_sigma_cols(c0, nc)
            assert np.max(np.abs(S1 - S)) / np.max(np.abs(E)) < 1e-13
    finally:
        batched.close()
        stepped.close()
