"""Dev aid: phase stamps (s_memrealtime, 100 MHz) of the blocks of the last k_xdraw launch at c3 —
delta blocks [start, end], row blocks [start, sums done, operators staged, X stored]; needs a
variant built with /tmp dev patch xstamps.py; run with DCFM_LIB=build/libdcfm_xst.so."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

dcfm = ge.load_package()
g, P, n, K = 64, 312, 1000, 30
Y = bench.synth_data(n, g * P)
smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 100, 5, seed=1)
smp.set_data_raw(Y, np.arange(g * P))
smp.init_state()
smp.run(1, 26)
smp.synchronize()
lib = smp.lib
lib.dcfm_debug_xstamps.argtypes = [C.c_void_p, C.c_int]
ndel = (g + 15) // 16
nb = ndel + (n + 15) // 16
buf = np.zeros((512, 4), dtype=np.uint64)
lib.dcfm_debug_xstamps(buf.ctypes.data, 512)
b = buf[:nb].astype(np.int64)
t0 = b[:, 0].min()
us = lambda x: (x - t0) / 100.0
print("delta blocks: start", np.round(us(b[:ndel, 0]), 2), "end", np.round(us(b[:ndel, 3]), 2))
r = b[ndel:nb]
for name, col in (("start", 0), ("sums done", 1), ("XM staged", 2), ("X stored", 3)):
    v = us(r[:, col])
    print(f"rows {name:10s} min {v.min():6.2f} med {np.median(v):6.2f} max {v.max():6.2f} us")
