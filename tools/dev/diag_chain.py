"""Dev diagnostic: a c2-shape chain from the initial state for T iterations, generated (Philox)
and injected (oracle DrawSource(11) draws), printing max|X|, max|Z| every few iterations; the
injected chain is compared with the oracle chain fed the same draws (computed here, vectorised)."""
import sys
sys.path.insert(0, "."); sys.path.insert(0, "tests")
import numpy as np
import __graft_entry__ as ge
import oracle
from helpers import make_case, state_dict, stacked_draws, rel_err
from oracle import vectorised as V

dcfm = ge.load_package()
T = int(sys.argv[1]) if len(sys.argv) > 1 else 200
c = make_case(500, 5000, 8, 20, seed=29, k0=10, dense_truth=False)
src = oracle.DrawSource(11, c["n"], c["p"], 8, 20, c["hyper"])
marks = [1, 2, 3, 5, 10, 20, 50, 100, 150, 200, 300, 400]
for mode in ("generated", "injected"):
    smp = dcfm.Sampler(c["n"], c["P"], 8, 20, c["rho"], 100000, 0, 1, seed=11, inject_draws=(mode == "injected"))
    smp.set_data(c["Yd"]); smp.set_state({f: v for f, v in state_dict(c["st"]).items() if f != "eta"})
    if mode == "injected":
        smp.set_draws(stacked_draws(src, 1, T), 1, T)
    t0 = 1
    out = []
    for mk in [m for m in marks if m <= T]:
        smp.run(t0, mk - t0 + 1); t0 = mk + 1
        s = smp.get_state()
        out.append((mk, float(np.abs(s["X"]).max()), float(np.abs(s["Z"]).max()), float(np.abs(s["tauh"]).max())))
    print(mode, " ".join(f"{a}:X{b:.3g}/Z{c_:.3g}/tau{d:.3g}" for a, b, c_, d in out), flush=True)
    smp.close()
D = V.Data(c["Yd"])
st = c["st"].copy()
t0 = 1
out = []
for mk in [m for m in marks if m <= T]:
    V.run_chain(D, st, c["rho"], c["hyper"], src.iteration, t0, mk - t0 + 1, 100000, 0, 1); t0 = mk + 1
    out.append((mk, float(np.abs(st.X).max()), float(np.abs(st.Z).max()), float(np.abs(st.tauh).max())))
print("oracle  ", " ".join(f"{a}:X{b:.3g}/Z{c_:.3g}/tau{d:.3g}" for a, b, c_, d in out), flush=True)
