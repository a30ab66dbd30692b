"""Per-field relative error vs the oracle after each iteration (dev aid).
Usage: python tools/debug_fields.py CASE   (a tests/test_gpu_parity.py case name)"""
import os, sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from helpers import make_case, state_dict, stacked_draws, rel_err
from oracle import dc_oracle as F
import test_gpu_parity as T
dcfm = ge.load_package()
n, p, g, K, burnin, mcmc, thin = T.CASES[sys.argv[1] if len(sys.argv) > 1 else "basic"]
c = make_case(n, p, g, K)
st, Yd = c["st"], c["Yd"]
N = burnin + mcmc
smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True)
smp.set_data(Yd); smp.set_state(state_dict(st)); smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
ref = st.copy(); Sref = None
for it in range(1, N + 1):
    smp.run(it, 1)
    Sref = F.run_chain(Yd, ref, c["rho"], c["hyper"], c["src"].iteration, it, 1, burnin, mcmc, thin, Sigmaout=Sref)
    got = smp.get_state()
    print(it, " ".join(f"{f}={rel_err(got[f], getattr(ref, f)):.1e}" for f in T.STATE_CMP))
