"""Dev diagnostic: a c2-shape chain from a stationary state, several iterations, in several
library modes, each compared field by field with the oracle stepped from the same state."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from helpers import make_case, state_dict, stacked_draws, rel_err, STATE_CMP
from oracle import SamplerState
from oracle import vectorised as V

dcfm = ge.load_package()
n, p, g, K = [int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (500, 5000, 8, 20))]
c = make_case(n, p, g, K, seed=29, k0=10, dense_truth=False)
warm = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], 1000, 0, 1, seed=11)
warm.set_data(c["Yd"]); warm.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
warm.run(1, 200); st0 = warm.get_state(); warm.close()
np.savez_compressed("gpurun_out/diag_st0.npz", **st0)
if len(sys.argv) > 5:
    sys.exit(0)
N, burnin, mcmc, thin = 6, 0, 6, 2
D = V.Data(c["Yd"])
refs = []
ref = SamplerState(**{f: np.array(v, dtype=np.float64, order="F") for f, v in st0.items()})
for it in range(1, N + 1):
    V.run_chain(D, ref, c["rho"], c["hyper"], c["src"].iteration, it, 1, burnin, mcmc, thin)
    refs.append(ref.copy())
draws = stacked_draws(c["src"], 1, N)
for name, kw, step in [("run16", {}, False), ("step", {}, True), ("run16_notail", {"asm_tail": -1}, False),
                       ("run16_exact", {"flags": 0x10}, False), ("run16_unfused", {"flags": 0x2}, False),
                       ("step_unfused", {"flags": 0x2}, True)]:
    smp = dcfm.Sampler(c["n"], c["P"], g, K, c["rho"], burnin, mcmc, thin, inject_draws=True, asm_batch=3, **kw)
    smp.set_data(c["Yd"]); smp.set_state({f: v for f, v in st0.items() if f != "eta"}); smp.set_draws(draws, 1, N)
    if step:
        for it in range(1, N + 1):
            smp.run(it, 1)
            got = smp.get_state()
            print(name, it, {f: "%.1e" % rel_err(got[f], getattr(refs[it - 1], f)) for f in ("Lambda", "X", "Z", "ps", "psi", "delta")}, flush=True)
    else:
        smp.run(1, N)
        got = smp.get_state()
        print(name, N, {f: "%.1e" % rel_err(got[f], getattr(refs[-1], f)) for f in ("Lambda", "X", "Z", "ps", "psi", "delta")}, flush=True)
    smp.close()
