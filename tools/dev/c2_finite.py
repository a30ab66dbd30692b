"""Dev aid: run the c2 chain (tests/test_gpu_c2_parity.py replicate 0) in 50-iteration chunks and
report the state's range after each, to find where a chain turns non-finite.
Usage: python tools/dev/c2_finite.py [n_iter] (DCFM_LIB selects the library)."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
from helpers import make_case, state_dict
dcfm = ge.load_package()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
c = make_case(500, 5000, 8, 20, seed=90, k0=10, rho=0.5)
smp = dcfm.Sampler(c["n"], c["P"], 8, 20, 0.5, 500, 2000, 5, seed=5000)
smp.set_data(c["Yd"])
smp.set_state({k: v for k, v in state_dict(c["st"]).items() if k != "eta"})
it = 1
while it <= N:
    smp.run(it, 50)
    try:
        st = smp.get_state(("Lambda", "ps", "X", "delta", "tauh", "psi", "Plam"))
    except Exception as e:
        print("non-finite after iteration", it + 49, e, flush=True)
        break
    print(it + 49, {k: "%.3g" % float(np.max(np.abs(v))) for k, v in st.items()}, "min ps %.3g" % float(st["ps"].min()),
          "min tau %.3g" % float(st["tauh"].min()), flush=True)
    it += 50
