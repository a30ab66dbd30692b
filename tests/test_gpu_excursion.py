"""The fused multi-iteration chain in the regime where the reference sampler makes X excursions.

divideconquer.m's Gibbs chain (quirks Q1 / Q2: Omega holds ps, the Z operator is (R R')^-1) makes
occasional long X excursions -- max|X| 1e3-1e7, E = eta'eta and the loading systems Q_j at
cond ~1e11.  There no forward-error bar between two implementations can
hold (two CPU restatements part ways too), so the fused path is pinned here in two exact ways:

* ONE dcfm_run of 6 iterations (the fused chain's cross-iteration hand-offs: iteration t's
  delta / tau chain in the k_cpass of t + 1, its column sums in the next k_wcol, the Z operators
  and loading-row variates handed from one launch to the next, the saved samples' assembly) is
  BITWISE equal to the same library stepped one dcfm_run per iteration;
* every stepped iteration is checked stage-wise against the oracle (tests/helpers.stagewise_errors)
  from the GPU's own state at the iteration's start: the stages before the loading solve (Z, X,
  eta; dc:97-134), psi, delta / tau, Plam (dc:149-165, 174-177) at 1e-10 against the oracle
  update applied to the GPU's own inputs, the loading draw (dc:137-144) by its per-row backward
  error <= 1e-13 against the oracle's systems, ps / omega (dc:168-172) per row at 1e-10 against
  dc:169's direct residual on the GPU's own eta and Lambda.

The start is the state after 200 generated-draw iterations at config c2's shape from Philox seed
11 -- the warm-up that the round-4 multi-iteration test failed from (Lambda 2.03e-5 normwise
against an oracle chain stepped from the same state); tests/test_gpu_parity.py keeps seed 12 as
the stationary case.

The wide path (K > 32) has the same guard on its SS identity (k_lambda_w + k_resid_flagged): a
c4-shape chain of generated draws runs >= 1,000 iterations through excursions without a
non-finite value (DCFM_ERR_NUMERIC would surface from dcfm_run)."""
import numpy as np
import pytest

from helpers import STATE_CMP, make_case, stacked_draws, stagewise_errors, state_dict

pytestmark = pytest.mark.gpu

TOL = 1e-10
BW_TOL = 1e-13


def _warm_state(dcfm, c, g, K, seed, iters):
    warm = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 100000, 0, 1, seed=seed)
    try:
        warm.set_data(c["Yd"])
        warm.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
        warm.run(1, iters)
        return warm.get_state()
    finally:
        warm.close()


def _as_oracle(st):
    from oracle import SamplerState
    return SamplerState(**{f: np.array(v, dtype=np.float64, order="F") for f, v in st.items()})


def test_fused_run_in_x_excursion_regime(dcfm, record_property):
    c = make_case(500, 5000, 8, 20, seed=29, k0=10, dense_truth=False)
    g, K = 8, 20
    st0 = _warm_state(dcfm, c, g, K, seed=11, iters=200)
    xmax0 = float(np.abs(st0["X"]).max())
    N, burnin, thin = 6, 0, 2
    draws = stacked_draws(c["src"], 1, N)
    start = {f: v for f, v in st0.items() if f != "eta"}

    def sampler():
        s = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, N, thin, inject_draws=True, asm_batch=1)
        s.set_data(c["Yd"])
        s.set_state(start)
        s.set_draws(draws, 1, N)
        return s

    fused = sampler()
    try:
        fused.run(1, N)
        got_f, S_f = fused.get_state(), fused.get_sigma()
    finally:
        fused.close()
    stepped = sampler()
    states = [st0]
    try:
        for it in range(1, N + 1):
            stepped.run(it, 1)
            states.append(stepped.get_state())
        S_s = stepped.get_sigma()
    finally:
        stepped.close()
    for f in STATE_CMP:
        assert np.array_equal(got_f[f], states[-1][f]), f"fused vs stepped: {f} not bitwise equal"
    assert np.array_equal(S_f, S_s), "fused vs stepped: Sigmaout not bitwise equal"

    worst = {}
    for it in range(1, N + 1):
        errs, bw, _ = stagewise_errors(_as_oracle(states[it - 1]), states[it], c["Yd"], c["rho"], c["hyper"],
                                       c["src"].iteration(it))
        for f, e in errs.items():
            worst[f] = max(worst.get(f, 0.0), e)
            assert e < TOL, f"iter {it}: stage {f} rel err {e:.3e} (bar {TOL:.0e}); warm-up max|X| {xmax0:.3g}"
        worst["lambda_bw"] = max(worst.get("lambda_bw", 0.0), bw)
        assert bw < BW_TOL, f"iter {it}: loading backward error {bw:.3e} (bar {BW_TOL:.0e})"
    xmax = max(float(np.abs(s["X"]).max()) for s in states)
    record_property("warmup_xmax", xmax0)
    record_property("chain_xmax", xmax)
    for f, e in worst.items():
        record_property(f"worst_{f}", e)
    print("EXCURSION", {"warmup_xmax": xmax0, "chain_xmax": xmax, **{k: f"{v:.2e}" for k, v in worst.items()}})


# c4 shape (p 10,000, n 2,000, g 8, K 100), generated draws.  The Philox seed is one whose chain makes
# X excursions (tools/dev/excursion_probe.py); every dcfm_run raises on a non-finite state.
C4_SEED = 5
C4_ITERS = 1200


def test_c4_generated_chain_through_excursions(dcfm, record_property):
    c = make_case(2000, 10000, 8, 100, seed=29, k0=10, dense_truth=False)
    g, K = 8, 100
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 100000, 0, 1, seed=C4_SEED)
    xmax, psmin = [], []
    try:
        smp.set_data(c["Yd"])
        smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
        step = 100
        for it in range(1, C4_ITERS + 1, step):
            smp.run(it, step)              # raises DCFM_ERR_NUMERIC on a NaN / Inf in the state
            st = smp.get_state(("X", "ps"))
            assert np.all(np.isfinite(st["X"])) and np.all(st["ps"] > 0)
            xmax.append(float(np.abs(st["X"]).max()))
            psmin.append(float(st["ps"].min()))
    finally:
        smp.close()
    record_property("xmax_per_100", xmax)
    print("C4_CHAIN", {"seed": C4_SEED, "xmax": [f"{v:.3g}" for v in xmax], "psmin": f"{min(psmin):.3g}"})
