"""Oracle breakdown rate at BASELINE config c4's shape (TEST INFRASTRUCTURE).

At c4 (p 10,000, n 2,000, g 8, K 100) some chains of the reference sampler make an X excursion that
escalates until a loading system Q_j of dc:141 is no longer positive definite: chol(Qlam,'lower')
(dc:142) raises and MATLAB stops.  The GPU library reports the same event as DCFM_ERR_NUMERIC.  This
script measures how often the ORACLE chain ends that way, so tests/test_gpu_c4_breakdown.py can compare
the GPU chains' breakdown fraction with it (two-sided Fisher exact test at 1 %).

Every chain starts from the same data set and initial state (helpers.make_case(2000, 10000, 8, 100,
seed=CASE_SEED, k0=10, dense_truth=False) -- the case of tests/test_gpu_excursion.py) and draws its own
iteration variates (oracle.DrawSource(DRAW_SEED0 + r).iteration, NumPy).  The sweep is
oracle/vectorised.py with dc:169's direct residual (``direct=True``), run stage by stage so a failure
is attributed to the stage where it happens:
  "ZX"      cholcov of Zprec / Xprec (dc:100,118) not positive definite, or a non-finite Z / X / eta
  "Lambda"  chol(Qlam,'lower') of dc:142 raises, or a non-finite Lambda
  "rest"    a non-finite psi / delta / tau / ps / omega / Plam (dc:149-177)
Each chain runs ITERS = BURNIN + MCMC iterations (GPU probes of 33 Philox seeds at this shape broke
down between iterations 150 and 450 or not at all within 1,200; tools/dev/excursion_probe.py) and
records the breakdown iteration and stage, or None, and max|X| every 25 iterations.  A chain that
completes also assembles Sigmaout (dc:180-196; BURNIN 250, MCMC 250, thin 5: 50 saved samples) and
records its Frobenius and operator-norm error against the synthetic truth (make_c3_parity's in-place
lower-triangle errors), so the GPU test can compare the completed chains' posterior error too.

Run from the repo root, one process per chain (about 30 minutes each on one host thread):
  for r in $(seq 0 23); do OMP_NUM_THREADS=1 python3 tests/golden/make_c4_breakdown.py --rep $r; done
  python3 tests/golden/make_c4_breakdown.py --merge
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

import oracle  # noqa: E402
from helpers import make_case  # noqa: E402
from oracle import vectorised as V  # noqa: E402
from make_c3_parity import lower_errors, truth_lowrank  # noqa: E402

PARAMS = dict(n=2000, p=10000, g=8, K=100, k0=10, rho=0.5, burnin=250, mcmc=250, thin=5)
CASE_SEED = 29
DRAW_SEED0 = 4000
R = 24
OUT = ROOT / "tests" / "golden" / "c4_breakdown.json"


def _finite(*arrs):
    return all(bool(np.all(np.isfinite(a))) for a in arrs)


def oracle_chain(c, draws, burnin, mcmc, thin):
    """Runs the vectorised oracle chain; returns (breakdown iteration or None, stage or None, xmax trace,
    lower-triangle Sigmaout accumulator)."""
    iters = burnin + mcmc
    effsamp = mcmc / thin
    T = np.zeros((c["p"], c["p"]), order="F")
    D = V.Data(c["Yd"])
    st = c["st"].copy()
    rho, hyper = c["rho"], c["hyper"]
    xmax = []
    for it in range(1, iters + 1):
        d = draws(it)
        with np.errstate(all="ignore"):
            try:
                V.update_ZX(st, D, rho, d)
                V.update_eta(st, rho)
            except np.linalg.LinAlgError:
                return it, "ZX", xmax, None
            if not _finite(st.Z, st.X, st.eta):
                return it, "ZX", xmax, None
            try:
                V.update_Lambda_psi_delta_ps(st, D, hyper, d, direct=True)
            except np.linalg.LinAlgError:
                return it, "Lambda", xmax, None
            if not _finite(st.Lambda):
                return it, "Lambda", xmax, None
            V.update_Plam(st)
            if not _finite(st.psi, st.delta, st.tauh, st.ps, st.omega, st.Plam):
                return it, "rest", xmax, None
        if it % thin == 0 and it > burnin:                                   # dc:180
            V.assemble_lower(T, st, rho, effsamp)
        if it % 25 == 0:
            xmax.append(float(np.abs(st.X).max()))
    return None, None, xmax, T


def one_rep(r):
    P = PARAMS
    t0 = time.time()
    c = make_case(P["n"], P["p"], P["g"], P["K"], seed=CASE_SEED, k0=P["k0"], rho=P["rho"], dense_truth=False)
    src = oracle.DrawSource(DRAW_SEED0 + r, c["n"], c["p"], P["g"], P["K"], c["hyper"])
    it, stage, xmax, T = oracle_chain(c, src.iteration, P["burnin"], P["mcmc"], P["thin"])
    rec = dict(rep=r, draw_seed=DRAW_SEED0 + r, breakdown_iter=it, stage=stage, xmax_per_25=xmax)
    if T is not None:
        Y, _, L0, sig2 = oracle.synth.make_data(P["n"], P["p"], k0=P["k0"], factors=True, dense_truth=False)
        U, s = truth_lowrank(L0, sig2, Y, c["keep"], c["init"].varind)
        fro, op, tfro, top = lower_errors(T, U, s)
        rec.update(fro_rel=fro / tfro, op_rel=op / top, truth_fro=tfro, truth_op=top)
    rec["seconds"] = round(time.time() - t0, 1)
    (OUT.parent / f"c4_breakdown_rep{r}.json").write_text(json.dumps(rec) + "\n")
    print(json.dumps(rec), flush=True)


def merge():
    reps = [json.loads((OUT.parent / f"c4_breakdown_rep{r}.json").read_text()) for r in range(R)]
    broke = [x for x in reps if x["breakdown_iter"] is not None]
    OUT.write_text(json.dumps(dict(params=PARAMS, case_seed=CASE_SEED, draw_seed0=DRAW_SEED0, direct=True,
                                   chains=R, broke_down=len(broke), replicates=reps), indent=1) + "\n")
    for r in range(R):
        (OUT.parent / f"c4_breakdown_rep{r}.json").unlink()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rep", type=int)
    ap.add_argument("--merge", action="store_true")
    a = ap.parse_args()
    if a.merge:
        merge()
    else:
        one_rep(a.rep)
