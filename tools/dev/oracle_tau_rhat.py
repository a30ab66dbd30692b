"""Dev evidence (CPU, test infrastructure only): does the REFERENCE's sampler itself mix slowly in
sum(log tau) when K is well above the true factor count?  Runs the vectorised oracle chain
(oracle/vectorised.py, a restatement of divideconquer.m:90-177) at a small shape with
K = 30 > k0 = 10 (as c3) and reports split-R-hat / ESS of the same four chain summaries the
device trace records (dcfm_set_trace: ||Lambda||_F^2, tr Omega, sum log ps, sum log tau) over
the post-burn-in iterations.  Usage: OMP_NUM_THREADS=8 python3 tools/dev/oracle_tau_rhat.py
[n p g K burnin mcmc]"""
import importlib.util
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from helpers import make_case  # noqa: E402
from oracle import vectorised as V  # noqa: E402

spec = importlib.util.spec_from_file_location(
    "diag", ROOT / "a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd" / "diagnostics.py")
diag = importlib.util.module_from_spec(spec)
spec.loader.exec_module(diag)

a = [int(x) for x in sys.argv[1:]] or [300, 960, 8, 30, 1000, 5000]
n, p, g, K, burnin, mcmc = a
c = make_case(n, p, g, K, seed=11, k0=10, rho=0.5)
st, D = c["st"].copy(), V._as_data(c["Yd"])
tr = []
t0 = time.time()
for it in range(1, burnin + mcmc + 1):
    V.gibbs_iteration(st, D, c["rho"], c["hyper"], c["src"].iteration(it))
    if it > burnin:
        tr.append([float(np.sum(st.Lambda ** 2)), float(np.sum(st.omega)), float(np.sum(np.log(st.ps))),
                   float(np.sum(np.log(st.tauh)))])
x = np.asarray(tr)[None]
names = ["lambda_fro2", "tr_omega", "sum_log_ps", "sum_log_tau"]
rh, es = diag.split_rhat(x), diag.ess(x)
out = {"shape": dict(n=n, p=p, g=g, K=K, k0=10, burnin=burnin, mcmc=mcmc), "seconds": round(time.time() - t0, 1),
       "split_rhat": {k: round(float(v), 4) for k, v in zip(names, rh)},
       "ess": {k: round(float(v), 1) for k, v in zip(names, es)},
       "sum_log_tau_first_last_mean": [round(float(x[0, :mcmc // 10, 3].mean()), 2), round(float(x[0, -mcmc // 10:, 3].mean()), 2)]}
print(json.dumps(out))
