"""Oracle leg of north_star check (2) at the north-star config c3 (TEST INFRASTRUCTURE).

c3 = p 19,968 (= 312 x 64), n 1,000, g 64, K 30 (k = 1,920), rho 0.5,
BURNIN 500, MCMC 1,500, thin 5 (300 saved samples).  Same paired design as
make_c2_parity.py: replicate r fixes the synthetic data set (oracle.synth.make_data,
DATA_SEED) and the driver's init / partition draws (oracle.DrawSource(CASE_SEED + r)); the
oracle chain (oracle/vectorised.py, NumPy draws from the same DrawSource; ps from dc:169's
direct residual Yd - eta Lambda', ``direct=True``, the reference's formula as written) runs
BURNIN + MCMC iterations and its posterior-mean Sigmaout is compared with the truth in the reference's
output space (Q7, dc:36-39,50-59).

At p = 19,968 a dense copy of the truth or of the difference would be 3.2 GB each, so the
errors are taken from the lower-triangle accumulator in place: the truth's low-rank form
U U' + diag(s) (the form dcfm_sigma_error takes, <pkg>/driver.truth_factors) is subtracted
column block by column block, the Frobenius norm sums the lower triangle twice minus the
diagonal, and the operator norm is the largest |eigenvalue| of the symmetric difference by
ARPACK (scipy eigsh, tol 1e-10) on the triangle.

Run from the repo root, one process per replicate (about 50 minutes each on 2 host threads):
  for r in 0 1 2 3 4 5; do OMP_NUM_THREADS=2 python3 tests/golden/make_c3_parity.py --rep $r & done; wait
  python3 tests/golden/make_c3_parity.py --merge
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
from scipy.sparse.linalg import LinearOperator, eigsh

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle  # noqa: E402
from helpers import make_case  # noqa: E402
from oracle import vectorised as V  # noqa: E402

PARAMS = dict(n=1000, p=19968, g=64, K=30, k0=10, rho=0.5, burnin=500, mcmc=1500, thin=5)
CASE_SEED = 190
R = 6
OUT = ROOT / "tests" / "golden" / "c3_parity.json"
BLK = 2048


def truth_lowrank(L0, sig2, Y, keep, varind):
    cols = np.asarray(keep)[np.asarray(varind)]
    sd = Y[:, cols].std(axis=0, ddof=1)
    return L0[cols] / sd[:, None], sig2[cols] / (sd * sd)


def lower_errors(T, U, s):
    """T: lower-triangle accumulator (Fortran order, upper triangle untouched zeros) of the
    estimate; overwritten with the lower triangle of (estimate - truth).  Returns the
    Frobenius and operator norms of the symmetric difference and of the truth."""
    p = T.shape[0]
    for c0 in range(0, p, BLK):
        c1 = min(p, c0 + BLK)
        T[c0:, c0:c1] -= U[c0:] @ U[c0:c1].T
        T[np.arange(c0, c1), np.arange(c0, c1)] -= s[c0:c1]
        T[:c0, c0:c1] = 0.0
        blk = T[c0:c1, c0:c1]
        blk[np.triu_indices(c1 - c0, 1)] = 0.0
    dg = np.diag(T).copy()
    fro = float(np.sqrt(2.0 * np.sum(T * T) - np.sum(dg * dg)))

    def mv(x):
        x = np.asarray(x).reshape(-1)
        return T @ x + T.T @ x - dg * x

    op = float(abs(eigsh(LinearOperator((p, p), matvec=mv, dtype=np.float64), k=1, which="LM",
                         tol=1e-10, return_eigenvectors=False)[0]))
    G = U.T @ U
    tfro = float(np.sqrt(np.sum(G * G) + 2.0 * np.sum(s * np.sum(U * U, axis=1)) + np.sum(s * s)))
    top = float(eigsh(LinearOperator((p, p), matvec=lambda x: U @ (U.T @ x.reshape(-1)) + s * x.reshape(-1),
                                     dtype=np.float64), k=1, which="LA", tol=1e-10,
                      return_eigenvectors=False)[0])
    return fro, op, tfro, top


def one_rep(r):
    P = PARAMS
    t0 = time.time()
    Y, _, L0, sig2 = oracle.synth.make_data(P["n"], P["p"], k0=P["k0"], factors=True, dense_truth=False)
    c = make_case(P["n"], P["p"], P["g"], P["K"], seed=CASE_SEED + r, k0=P["k0"], rho=P["rho"],
                  dense_truth=False)
    assert np.array_equal(c["Y"], Y)
    U, s = truth_lowrank(L0, sig2, Y, c["keep"], c["init"].varind)
    N = P["burnin"] + P["mcmc"]
    T = V.run_chain(c["Yd"], c["st"].copy(), c["rho"], c["hyper"], c["src"].iteration, 1, N,
                    P["burnin"], P["mcmc"], P["thin"], direct=True)
    fro, op, tfro, top = lower_errors(T, U, s)
    rec = dict(rep=r, case_seed=CASE_SEED + r, direct=True, fro=fro, op=op, fro_rel=fro / tfro, op_rel=op / top,
               truth_fro=tfro, truth_op=top, seconds=round(time.time() - t0, 1))
    (OUT.parent / f"c3_parity_rep{r}.json").write_text(json.dumps(rec) + "\n")
    print(json.dumps(rec), flush=True)


def merge():
    reps = []
    for r in range(R):
        f = OUT.parent / f"c3_parity_rep{r}.json"
        reps.append(json.loads(f.read_text()))
    OUT.write_text(json.dumps(dict(params=PARAMS, case_seed0=CASE_SEED, direct=True, replicates=reps), indent=1) + "\n")
    for r in range(R):
        (OUT.parent / f"c3_parity_rep{r}.json").unlink()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rep", type=int)
    ap.add_argument("--merge", action="store_true")
    a = ap.parse_args()
    if a.merge:
        merge()
    else:
        one_rep(a.rep)
