"""Dev aid: per-role block timelines of one k_wcol launch at c3 (needs a variant built with
tools/patches/stamps.py; run with DCFM_LIB=build/libdcfm_stamps.so)."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

dcfm = ge.load_package()
g, P, n, K = 64, 312, 1000, 30
Y = bench.synth_data(n, g * P)
smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 100, 5, seed=1)
smp.set_data_raw(Y, np.arange(g * P))
smp.init_state()
smp.run(1, 20)
smp.synchronize()
lib = smp.lib
lib.dcfm_debug_stamps.argtypes = [C.c_void_p, C.c_int]
G, nxs = 64, 8
nb = G + G + nxs + (1024 // 128) * G
buf = np.zeros((nb, 2), dtype=np.uint64)
smp.run(21, 1)          # one iteration: k_wcol(ops + delta + wpass), then the trailing delta-only launch
smp.synchronize()
lib.dcfm_debug_stamps(buf.ctypes.data, nb)
t0 = buf[:, 0].min()
roles = [("ops", G), ("colsum", G), ("xsum", nxs), ("wpass", nb - 2 * G - nxs)]
o = 0
for name, cnt in roles:
    st = (buf[o:o + cnt, 0] - t0) / 100.0
    en = (buf[o:o + cnt, 1] - t0) / 100.0
    print(f"{name:12s} start {st.min():7.2f}..{st.max():7.2f} us  end {en.min():7.2f}..{np.median(en):7.2f}..{en.max():7.2f} us")
    o += cnt
