"""Dev aid: per-phase shader cycles per block of k_lambda_t at the c4 shape (needs the variant
built from a dev patch (git history: tools/patches/ltphase.py); run with DCFM_LIB=build/libdcfm_ltphase.so)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

dcfm = ge.load_package()
g, P, n, K = 8, 1250, 2000, 100
if len(sys.argv) > 1:
    g, P, n, K = (int(v) for v in sys.argv[1:5])
Y = bench.synth_data(n, g * P)
smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 100000, 100000, seed=1)
smp.set_data_raw(Y, np.arange(g * P))
smp.init_state()
smp.run(1, 5)
smp.synchronize()
lib = smp.lib
lib.dcfm_debug_phases.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(8, dtype=np.uint64)
lib.dcfm_debug_phases(buf.ctypes.data, 1)
iters = 10
smp.run(6, iters)
smp.synchronize()
lib.dcfm_debug_phases(buf.ctypes.data, 0)
per = buf.astype(np.float64) / (g * P * iters)
names = ["loads+Q", "diag0/v", "panel", "trailing", "backsolve", "epilogue"]
tot = per[:6].sum()
for i, nm in enumerate(names):
    print(f"{nm:10s} {per[i]:10.0f} cycles/block  {per[i] / tot:6.1%}")
print(f"{'total':10s} {tot:10.0f}")
print(f"{'slot6':10s} {per[6]:10.0f}   slot7 {per[7]:10.0f}")
