"""Dev diagnostic: max|X| along generated (Philox) c2-shape chains for several seeds."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from helpers import make_case, state_dict

dcfm = ge.load_package()
c = make_case(500, 5000, 8, 20, seed=29, k0=10, dense_truth=False)
seeds = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(11, 27))
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for seed in seeds:
    smp = dcfm.Sampler(c["n"], c["P"], 8, 20, c["rho"], 100000, 0, 1, seed=seed, flags=flags)
    smp.set_data(c["Yd"]); smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
    t0, out = 1, []
    try:
        for mk in (10, 50, 100, 200, 400):
            smp.run(t0, mk - t0 + 1); t0 = mk + 1
            out.append("%d:X%.3g" % (mk, float(np.abs(smp.get_state(("X",))["X"]).max())))
    except Exception as e:
        out.append(f"ERROR at <= {mk}: {str(e)[:40]}")
    print(seed, " ".join(out), flush=True)
    smp.close()
