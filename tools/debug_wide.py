"""Per-field GPU-vs-oracle errors for a few wide-K shapes (debug aid)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np
from helpers import STATE_CMP, make_case, rel_err, stacked_draws, state_dict
from oracle import dc_oracle as F
import __graft_entry__ as ge
dcfm = ge.load_package()
for (n, p, g, K) in [(40, 141, 3, 40), (37, 99, 3, 33), (40, 99, 3, 40), (37, 141, 3, 40), (64, 96, 2, 48)]:
    c = make_case(n, p, g, K)
    N = 3
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 0, N, 1, inject_draws=True)
    smp.set_data(c["Yd"]); smp.set_state(state_dict(c["st"])); smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
    ref = c["st"].copy()
    for it in range(1, N + 1):
        smp.run(it, 1)
        F.run_chain(c["Yd"], ref, c["rho"], c["hyper"], c["src"].iteration, it, 1, 0, N, 1)
        got = smp.get_state()
        print((n, p, g, K), it, " ".join(f"{f}={rel_err(got[f], getattr(ref, f)):.1e}" for f in STATE_CMP), flush=True)
    smp.close()
