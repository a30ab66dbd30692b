"""Generate the golden fixtures under tests/golden/ from the CPU oracle (faithful loop).

Run from the repo root:  python tests/golden/make_golden.py
Each fixture holds inputs (raw Y, varind, the standardised Yd, the initial
state), the injected standard variates for every iteration, the state after
every iteration and the final Sigmaout.  Cases follow SURVEY.md §4.2:
  (i) K >= 2, g >= 3 (quirk Q4)      (ii) K = 1, g >= 3 (quirk Q5)
  (iii) thin does not divide BURNIN  (iv) zero columns (dc:31-39)   (v) g = 1
These fixtures pin the HIP kernels (and the oracle against regressions); they
do not pin MATLAB — parity against the reference itself is unpinned (no
MATLAB/Octave, no reference fixtures; see oracle/__init__.py).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402
from oracle import dc_oracle as F  # noqa: E402

STATE = ("Lambda", "ps", "omega", "psi", "Plam", "X", "Z", "eta", "delta", "tauh")

CASES = {
    # name: n, p_raw, g, K, burnin, mcmc, thin, zero_cols, seed
    "case_i_K3_g3": (12, 18, 3, 3, 1, 2, 1, 0, 101),
    "case_ii_K1_g3": (12, 18, 3, 1, 1, 2, 1, 0, 102),
    "case_iii_thin2_burnin1": (10, 16, 4, 2, 1, 2, 2, 0, 103),
    "case_iv_zero_cols": (12, 20, 3, 2, 0, 3, 1, 2, 104),
    "case_v_g1": (10, 5, 1, 2, 0, 3, 1, 0, 105),
}


def make(name, n, p_raw, g, K, burnin, mcmc, thin, zero_cols, seed):
    Y, _ = oracle.synth.make_data(n, p_raw, k0=3, seed=seed, zero_cols=zero_cols)
    hyper = F.Hyper()
    rho = 0.5
    Yk, n, p, P, K_, keep = F.preprocess(Y, g, K * g)
    src = oracle.DrawSource(seed, n, p, g, K, hyper)
    init = src.init()
    Yd = F.standardize(F.partition(Yk, g, init.varind))
    st = F.initialise(n, P, K, g, rho, hyper, init)
    N = burnin + mcmc
    out = {"Y": Y, "keep": keep, "varind": init.varind, "Yd": Yd,
           "meta": np.array([n, p, g, K, burnin, mcmc, thin, seed]), "rho": np.array(rho)}
    for f in STATE:
        out[f"init_{f}"] = getattr(st, f).copy()
    draws = [src.iteration(t) for t in range(1, N + 1)]
    for f, a in draws[0].stacked(draws[1:]).items():
        out[f"draw_{f}"] = a
    rec = []
    S = F.run_chain(Yd, st, rho, hyper, lambda t: draws[t - 1], 1, N, burnin, mcmc, thin, record=rec)
    for t, s in enumerate(rec, start=1):
        for f in STATE:
            out[f"it{t}_{f}"] = getattr(s, f)
    out["Sigmaout"] = S
    path = Path(__file__).parent / f"{name}.npz"
    np.savez_compressed(path, **out)
    return path


if __name__ == "__main__":
    for name, args in CASES.items():
        p = make(name, *args)
        print(p.name, p.stat().st_size, "bytes")
