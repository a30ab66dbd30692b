"""Dev aid: the c2 chain iteration by iteration (generated or injected draws), state ranges."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from helpers import make_case, state_dict, stacked_draws
dcfm = ge.load_package()
mode = sys.argv[1]
N = int(sys.argv[2])
c = make_case(500, 5000, 8, 20, seed=90, k0=10, rho=0.5)
smp = dcfm.Sampler(c["n"], c["P"], 8, 20, 0.5, 500, 2000, 5, seed=5000, inject_draws=(mode == "inject"))
smp.set_data(c["Yd"])
smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
if mode == "inject":
    smp.set_draws(stacked_draws(c["src"], 1, N), 1, N)
for it in range(1, N + 1):
    smp.run(it, 1)
    try:
        st = smp.get_state(("Lambda", "ps", "X", "Z", "delta", "tauh", "psi", "Plam", "omega"))
    except Exception as e:
        print(mode, "non-finite after iteration", it, e, flush=True)
        break
    print(mode, it, {k: "%.3g" % float(np.max(np.abs(v))) for k, v in st.items()}, "min ps %.3g" % float(st["ps"].min()),
          "min psi %.3g" % float(st["psi"].min()), flush=True)
