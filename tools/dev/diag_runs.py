"""Dev diagnostic: the same generated c2-shape chain (seed 11) stepped with different dcfm_run
call patterns must give bitwise the same state (counter-based draws)."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from helpers import make_case, state_dict

dcfm = ge.load_package()
c = make_case(500, 5000, 8, 20, seed=29, k0=10, dense_truth=False)
res = {}
for name, pattern in [("1x10", [(1, 10)]), ("steps", [(1, 1), (2, 1), (3, 1), (4, 2), (6, 5)]),
                      ("2x5", [(1, 5), (6, 5)]), ("10x1", [(t, 1) for t in range(1, 11)])]:
    smp = dcfm.Sampler(c["n"], c["P"], 8, 20, c["rho"], 100000, 0, 1, seed=11)
    smp.set_data(c["Yd"]); smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
    try:
        for a, b in pattern:
            smp.run(a, b)
            s = smp.get_state()
            print(name, a + b - 1, "maxX %.4g" % float(np.abs(s["X"]).max()), "maxLam %.4g" % float(np.abs(s["Lambda"]).max()), flush=True)
        res[name] = s
    except Exception as e:
        print(name, "ERROR", e, flush=True)
    smp.close()
names = list(res)
for n2 in names[1:]:
    print(names[0], "vs", n2, {f: bool(np.array_equal(res[names[0]][f], res[n2][f])) for f in ("Lambda", "X", "Z", "ps", "delta")})
