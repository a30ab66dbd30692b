"""GPU parity at every BASELINE.json shape (configs c1-c4), not only at toy sizes.

The HIP path (through the C ABI) runs 2 iterations with injected draws (burn-in 1, one
saved sample, so the covariance assembly runs too) against the vectorised oracle
(oracle/vectorised.py, itself pinned to the faithful per-row loop in tests/test_oracle.py,
including at c1's shape).  Every state array after every iteration, and Sigmaout
(compared stripe by stripe through dcfm_get_sigma_cols, so the host never holds two
copies of p x p), must match to the north_star bar of 1e-10 normwise relative
(max |gpu - oracle| / max |oracle|).  Reference lines: dc:90-196.

  c1  p = 1,000   n = 100    g = 4   K = 5     (configs[0], the plumbing case)
  c2  p = 5,000   n = 500    g = 8   K = 20    (configs[1])
  c3  p = 19,968  n = 1,000  g = 64  K = 30    (configs[2], north star)
  c4  p = 10,000  n = 2,000  g = 8   K = 100   (configs[3], one chain)

Conditioning.  The reference chain's second iteration is not always well conditioned: with
quirks Q1 (Omega as a variance) and Q2 (the (R R')^-1 operator) the X / Z draws make
excursions (|X| ~ 1e3 at c2), E = eta'eta reaches cond ~1e7 and so does Q_j of the loading
rows (dc:141).  Two restatements of the reference then differ by cond * eps: the faithful
loop and the vectorised oracle differ by 1.3e-9 in Lambda at c2's iteration 2 (8e-12 at c3,
7e-14 at c4).  No implementation can meet 1e-10 there, so where the faithful loop is cheap
enough to run (c1, c2) the bar of iteration 2 is max(1e-10, 10 x the faithful-vs-vectorised
spread of the same conditional updates from the same state); everything upstream of the
loading solve (Z, X, eta) and all of iteration 1 keep the strict 1e-10.  c3 and c4 are
strict throughout (their faithful iterations take 30-80 s; spreads measured 8e-12 / 7e-14).
"""
import numpy as np
import pytest

from helpers import STATE_CMP, make_case, rel_err, sigma_stripe_from_lower, stacked_draws, state_dict
from oracle import dc_oracle as F
from oracle import vectorised as V

pytestmark = pytest.mark.gpu

TOL = 1e-10
CONFIGS = {
    # name: (n, p, g, K, faithful spread check)
    "c1": (100, 1000, 4, 5, True),
    "c2": (500, 5000, 8, 20, True),
    "c3": (1000, 19968, 64, 30, False),
    "c4": (2000, 10000, 8, 100, False),
}
UPSTREAM = ("X", "Z", "eta")   # drawn before the loading solve: always strict


def _sigma_err(smp, SigL, p, w=2048):
    den = float(np.max(np.abs(np.diag(SigL))))        # max |Sigmaout| sits on the diagonal (SPD)
    worst = 0.0
    for c0 in range(0, p, w):
        c1 = min(p, c0 + w)
        S = smp.get_sigma_cols(c0, c1 - c0)
        if c0 == 0:
            assert np.array_equal(S[:c1, :], S[:c1, :].T), "Sigmaout not symmetric"
        worst = max(worst, float(np.max(np.abs(S - sigma_stripe_from_lower(SigL, c0, c1)))) / den)
    return worst


@pytest.mark.parametrize("name", list(CONFIGS))
def test_baseline_shape_parity(dcfm, name):
    n, p, g, K, spread_check = CONFIGS[name]
    burnin, mcmc, thin = 1, 1, 1
    N = burnin + mcmc
    effsamp = mcmc / thin
    c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
    st, Yd = c["st"], c["Yd"]
    D = V.Data(Yd)
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True)
    try:
        smp.set_data(Yd)
        smp.set_state({f: v for f, v in state_dict(st).items() if f != "eta"})
        smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
        ref = st.copy()
        SigL = None
        for it in range(1, N + 1):
            tol = {f: TOL for f in STATE_CMP}
            tol_S = TOL
            if it > 1 and spread_check:
                alt = ref.copy()                                   # same state at the iteration's start
                F.gibbs_iteration(alt, Yd, c["rho"], c["hyper"], c["src"].iteration(it))
            smp.run(it, 1)
            SigL = V.run_chain(D, ref, c["rho"], c["hyper"], c["src"].iteration, it, 1,
                               burnin, mcmc, thin, SigLower=SigL)
            if it > 1 and spread_check:
                for f in STATE_CMP:
                    if f not in UPSTREAM:
                        tol[f] = max(TOL, 10.0 * rel_err(getattr(alt, f), getattr(ref, f)))
                Salt = V.full(V.assemble_lower(np.zeros_like(SigL), alt, c["rho"], effsamp))
                tol_S = max(TOL, 10.0 * rel_err(Salt, V.full(SigL)))
            got = smp.get_state()
            for f in STATE_CMP:
                e = rel_err(got[f], getattr(ref, f))
                assert e < tol[f], f"{name} iter {it}: {f} rel err {e:.3e} (bar {tol[f]:.1e})"
        assert smp.saved_samples() == 1
        e = _sigma_err(smp, SigL, c["p"])
        assert e < tol_S, f"{name}: Sigmaout rel err {e:.3e} (bar {tol_S:.1e})"
    finally:
        smp.close()
