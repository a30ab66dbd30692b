"""Size-independent properties of the HIP path with on-device Philox draws, at
BASELINE sizes (c3) and on a statistical-parity case (north_star check 2)."""
import numpy as np
import pytest

import oracle
from helpers import make_case, state_dict
from oracle import vectorised as V

pytestmark = pytest.mark.gpu


def _c3_sampler(dcfm, n_iter, seed=5, thin=5, asm_batch=16):
    n, g, P, K, rho = 1000, 64, 312, 30, 0.5
    p = g * P
    Y, _ = oracle.synth.make_data(n, p, k0=10)
    hyper = dcfm.Hyper()
    Yk, n, pk, P, K_, keep = dcfm.preprocess(Y, g, K * g)
    init = dcfm.driver._HostInitDraws(seed, n, pk, g, K, hyper)
    Yd = dcfm.partition_standardize(Yk, g, init.varind)
    st = dcfm.initial_state(n, P, K, g, rho, hyper, init)
    smp = dcfm.Sampler(n, P, g, K, rho, 0, n_iter, thin, seed=seed, asm_batch=asm_batch)
    smp.set_data(Yd)
    smp.set_state({k: v for k, v in st.items() if k != "eta"})
    return smp


def test_c3_determinism_symmetry_finiteness(dcfm):
    """Same seed -> bitwise identical state and Sigmaout; Sigmaout symmetric, finite, diag ~ 1."""
    outs = []
    for _ in range(2):
        smp = _c3_sampler(dcfm, 20)
        try:
            smp.run(1, 20)
            st = smp.get_state(("Lambda", "X", "ps", "delta"))
            S = smp.get_sigma()
        finally:
            smp.close()
        outs.append((st, S))
    (s1, S1), (s2, S2) = outs
    for f in s1:
        assert np.array_equal(s1[f], s2[f]), f
        assert np.all(np.isfinite(s1[f])), f
    assert np.array_equal(S1, S2)
    assert np.array_equal(S1, S1.T)
    assert np.all(np.isfinite(S1))
    d = np.diag(S1)
    assert np.all(d > 0.2) and np.all(d < 3.0)


def test_c3_batch_size_invariance(dcfm):
    """Assembly batching is an implementation detail: asm_batch 1 vs 16 agree to rounding."""
    res = []
    for B in (1, 16):
        smp = _c3_sampler(dcfm, 10, thin=1, asm_batch=B)
        try:
            smp.run(1, 10)
            res.append(smp.get_sigma())
        finally:
            smp.close()
    a, b = res
    assert np.max(np.abs(a - b)) / np.max(np.abs(a)) < 1e-12


def test_statistical_parity_with_oracle(dcfm):
    """north_star check 2: posterior-mean covariance error vs the synthetic truth,
    GPU chain (Philox draws) vs oracle chain (NumPy draws), within Monte Carlo error."""
    n, p, g, K = 150, 48, 4, 4
    burnin, mcmc, thin = 100, 300, 2
    errs_gpu, errs_cpu = [], []
    for rep in range(3):
        c = make_case(n, p, g, K, seed=40 + rep, k0=3)
        truth = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
        smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, seed=1000 + rep)
        try:
            smp.set_data(c["Yd"])
            smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
            smp.run(1, burnin + mcmc)
            Sg = smp.get_sigma()
        finally:
            smp.close()
        Sc = V.full(V.run_chain(c["Yd"], c["st"].copy(), c["rho"], c["hyper"], c["src"].iteration, 1,
                                burnin + mcmc, burnin, mcmc, thin))
        errs_gpu.append(oracle.synth.cov_errors(Sg, truth)["fro_rel"])
        errs_cpu.append(oracle.synth.cov_errors(Sc, truth)["fro_rel"])
    eg, ec = np.mean(errs_gpu), np.mean(errs_cpu)
    spread = max(np.std(errs_gpu), np.std(errs_cpu), 0.01)
    assert abs(eg - ec) < 4 * spread + 0.03, (errs_gpu, errs_cpu)


def test_statistical_parity_with_oracle_p960(dcfm):
    """north_star check 2 at a larger shape (p = 960, n = 300, g = 8, K = 10): the GPU chain's
    posterior-mean covariance has the oracle chain's Frobenius AND operator-norm error against
    the synthetic truth, within Monte Carlo error.  Paired design: every replicate runs both
    chains on the same data and initial state with independent draws (Philox vs NumPy), so
    d_r = err_gpu,r - err_cpu,r has mean 0 under parity; the bar is 3 standard errors of the
    mean difference (floored at 1 % of the error itself, the replicates being few)."""
    n, p, g, K = 300, 960, 8, 10
    burnin, mcmc, thin = 100, 300, 3
    R = 4
    diffs = {"fro_rel": [], "op_rel": []}
    base = {"fro_rel": [], "op_rel": []}
    for rep in range(R):
        c = make_case(n, p, g, K, seed=70 + rep, k0=6)
        truth = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
        tnorm = float(np.max(np.abs(np.linalg.eigvalsh(truth))))
        smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, seed=2000 + rep)
        try:
            smp.set_data(c["Yd"])
            smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
            smp.run(1, burnin + mcmc)
            Sg = smp.get_sigma()
        finally:
            smp.close()
        Sc = V.full(V.run_chain(c["Yd"], c["st"].copy(), c["rho"], c["hyper"], c["src"].iteration, 1,
                                burnin + mcmc, burnin, mcmc, thin))
        eg, ec = oracle.synth.cov_errors(Sg, truth), oracle.synth.cov_errors(Sc, truth)
        for key, a, b in (("fro_rel", eg["fro_rel"], ec["fro_rel"]), ("op_rel", eg["op"] / tnorm, ec["op"] / tnorm)):
            diffs[key].append(a - b)
            base[key].append(b)
    for key in diffs:
        d = np.asarray(diffs[key])
        se = max(float(np.std(d, ddof=1)) / np.sqrt(R), 0.01 * float(np.mean(base[key])))
        assert abs(float(np.mean(d))) < 3 * se, (key, diffs[key], base[key])
