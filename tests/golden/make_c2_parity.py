"""Oracle leg of north_star check (2) at BASELINE config c2 (TEST INFRASTRUCTURE).

c2 = p 5,000, n 500, g 8, K 20 (k = 160), rho 0.5, BURNIN 500, MCMC 2,000, thin 5
(SURVEY §8(d) table).  For each replicate r the synthetic data set (oracle.synth.make_data,
data seed DATA_SEED) and the driver's init/partition draws (oracle.DrawSource(CASE_SEED + r))
are fixed; the oracle chain (oracle/vectorised.py, NumPy draws from the same DrawSource; ps from dc:169's
direct residual, ``direct=True``) runs
the full BURNIN + MCMC iterations and its posterior-mean Sigmaout is compared with the truth
in the reference's output space (Q7).  The Frobenius error and the operator-norm error
(exact, eigvalsh) go to tests/golden/c2_parity.json together with everything the GPU leg
(tests/test_gpu_c2_parity.py) needs to rebuild the same data, initial state and truth.

Run from the repo root, one process per replicate (about 6 minutes each on 2 host threads):
  for r in 0 1 2 3 4 5 6 7; do OMP_NUM_THREADS=2 python3 tests/golden/make_c2_parity.py --rep $r; done
  python3 tests/golden/make_c2_parity.py --merge
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

import oracle  # noqa: E402
from helpers import make_case  # noqa: E402
from oracle import vectorised as V  # noqa: E402

PARAMS = dict(n=500, p=5000, g=8, K=20, k0=10, rho=0.5, burnin=500, mcmc=2000, thin=5)
CASE_SEED = 90
R = 8
OUT = ROOT / "tests" / "golden" / "c2_parity.json"


def one_rep(r):
    P = PARAMS
    t0 = time.time()
    c = make_case(P["n"], P["p"], P["g"], P["K"], seed=CASE_SEED + r, k0=P["k0"], rho=P["rho"])
    truth = oracle.synth.truth_in_output_space(c["Sigma0"], c["Y"], c["keep"], c["init"].varind)
    tnorm = float(np.max(np.abs(np.linalg.eigvalsh(truth))))
    N = P["burnin"] + P["mcmc"]
    S = V.full(V.run_chain(c["Yd"], c["st"].copy(), c["rho"], c["hyper"], c["src"].iteration, 1, N,
                           P["burnin"], P["mcmc"], P["thin"], direct=True))
    e = oracle.synth.cov_errors(S, truth)
    rec = dict(rep=r, case_seed=CASE_SEED + r, direct=True, fro=e["fro"], op=e["op"], fro_rel=e["fro_rel"],
               op_rel=e["op"] / tnorm, truth_fro=float(np.linalg.norm(truth, "fro")), truth_op=tnorm,
               seconds=round(time.time() - t0, 1))
    (OUT.parent / f"c2_parity_rep{r}.json").write_text(json.dumps(rec) + "\n")
    print(json.dumps(rec), flush=True)


def merge():
    reps = [json.loads((OUT.parent / f"c2_parity_rep{r}.json").read_text()) for r in range(R)]
    OUT.write_text(json.dumps(dict(params=PARAMS, case_seed0=CASE_SEED, direct=True, replicates=reps),
                              indent=1) + "\n")
    for r in range(R):
        (OUT.parent / f"c2_parity_rep{r}.json").unlink()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rep", type=int)
    ap.add_argument("--merge", action="store_true")
    a = ap.parse_args()
    if a.merge:
        merge()
    else:
        one_rep(a.rep)
