"""On-device error of Sigmaout against the synthetic truth (dcfm_sigma_error; SURVEY §8(f)
row 2, north_star check 2).  The device result must equal the host computation on the
read-back matrix (oracle.synth.cov_errors: Frobenius, and the operator norm from a dense
symmetric eigensolve): Frobenius to 1e-10 relative (a different summation order only);
operator norm to 1e-9 relative when Lanczos runs to the full dimension (exact Krylov
space) and to 1e-6 with 60 steps (extremal eigenvalues converged).  The multi-rank case
(loopback ranks, each owning round-robin 128 x 128 tiles of the accumulator) must give
the same numbers on every rank.
"""
import threading

import numpy as np
import pytest

import oracle
from helpers import make_case, stacked_draws, state_dict

pytestmark = pytest.mark.gpu


def _case(n, p, g, K, seed):
    c = make_case(n, p, g, K, seed=seed, k0=4)
    _, _, Lam0, sig2 = oracle.synth.make_data(n, p, k0=4, factors=True)
    return c, Lam0, sig2


def _expected(S, c, Lam0, sig2):
    truth = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
    e = oracle.synth.cov_errors(S, truth)
    e["truth_fro"] = float(np.linalg.norm(truth, "fro"))
    return e


@pytest.mark.parametrize("n,p,g,K", [(120, 200, 4, 4), (80, 333, 3, 6)])
def test_sigma_error_matches_host(dcfm, n, p, g, K):
    c, Lam0, sig2 = _case(n, p, g, K, seed=21)
    burnin, mcmc, thin = 10, 30, 2
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, seed=7)
    try:
        smp.set_data(c["Yd"])
        smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
        smp.run(1, burnin + mcmc)
        S = smp.get_sigma()
        U, s = dcfm.truth_factors(Lam0, sig2, c["Y"], c["keep"], c["init"].varind)
        full = smp.sigma_error(U, s, iters=c["p"])
        short = smp.sigma_error(U, s, iters=60, seed=3)
        norms = smp.sigma_error(U, s, iters=0)
        rng = np.random.default_rng(1)          # a rank-20 truth: the r > 16 kernel variant
        U20, s20 = 0.3 * rng.standard_normal((c["p"], 20)), rng.uniform(0.1, 1.0, c["p"])
        wide = smp.sigma_error(U20, s20, iters=c["p"])
    finally:
        smp.close()
    e = _expected(S, c, Lam0, sig2)
    assert abs(full["fro"] - e["fro"]) <= 1e-10 * e["fro"]
    assert abs(full["truth_fro"] - e["truth_fro"]) <= 1e-10 * e["truth_fro"]
    assert abs(full["op"] - e["op"]) <= 1e-9 * e["op"], (full["op"], e["op"])
    assert abs(short["op"] - e["op"]) <= 1e-6 * e["op"], (short["op"], e["op"])
    assert norms["fro"] == full["fro"] and norms["op"] == 0.0
    e20 = oracle.synth.cov_errors(S, U20 @ U20.T + np.diag(s20))
    assert abs(wide["fro"] - e20["fro"]) <= 1e-10 * e20["fro"]
    assert abs(wide["op"] - e20["op"]) <= 1e-9 * e20["op"]


def test_sigma_error_loopback_ranks(dcfm):
    """2 ranks, p = 320 (3 x 3 assembly tiles split between them): same numbers on both
    ranks, equal to the host computation on the gathered Sigmaout."""
    n_r, g, K = 2, 4, 5
    c, Lam0, sig2 = _case(60, 320, g, K, seed=23)
    burnin, mcmc, thin = 1, 6, 2
    N = burnin + mcmc
    G = g // n_r
    draws = stacked_draws(c["src"], 1, N)
    U, s = dcfm.truth_factors(Lam0, sig2, c["Y"], c["keep"], c["init"].varind)
    smps = [dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True,
                         nranks=n_r, rank=r, device=0) for r in range(n_r)]
    out, errs = [None] * n_r, []
    try:
        dcfm.Sampler.comm_loopback(smps)
        for r, smp in enumerate(smps):
            smp.set_data(c["Yd"][:, :, r * G:(r + 1) * G])
            st = state_dict(c["st"], r * G, G)
            smp.set_state({f: st[f] for f in st if f != "eta"})
            smp.set_draws(draws, 1, N)

        def work(r):
            try:
                smps[r].run(1, N)
                S = smps[r].get_sigma()                                   # collective
                out[r] = (S, smps[r].sigma_error(U, s, iters=c["p"]))      # collective
            except Exception as e:                                        # surfaced below
                errs.append(e)

        ths = [threading.Thread(target=work, args=(r,)) for r in range(n_r)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in ths), "a rank did not finish"
        assert not errs, errs
    finally:
        for smp in smps:
            smp.close()
    assert out[0][1] == out[1][1]
    e = _expected(out[0][0], c, Lam0, sig2)
    got = out[0][1]
    assert abs(got["fro"] - e["fro"]) <= 1e-10 * e["fro"]
    assert abs(got["op"] - e["op"]) <= 1e-9 * e["op"]
