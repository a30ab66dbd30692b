"""Dev aid: per-role block timelines of one k_wcol launch at c3, or g shards from argv[1] (needs a variant built with
a dev patch (git history: tools/patches/stamps.py); run with DCFM_LIB=build/libdcfm_stamps.so)."""
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
if len(sys.argv) > 1:
    g = int(sys.argv[1])
Y = bench.synth_data(n, g * P)
smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 100, 5, seed=1)
smp.set_data_raw(Y, np.arange(g * P))
smp.init_state()
smp.run(1, 20)
smp.synchronize()
lib = smp.lib
lib.dcfm_debug_stamps.argtypes = [C.c_void_p, C.c_int]
G = g
chunk = 1                       # xsum_blocks (dcfm_internal.h)
while G // chunk > 8 and (G // chunk) % 2 == 0:
    chunk *= 2
nxs = 1 if G <= 8 else G // chunk
nb = G + G + nxs + (1024 // (128 if (1024 // 128) * G >= 256 else 64)) * G
buf = np.zeros((nb, 2), dtype=np.uint64)
smp.run(21, 6)          # steady state: the last k_wcol with a W pass is iteration 26's
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
if hasattr(lib, "dcfm_debug_xs"):
    xs = np.zeros((64, 8), dtype=np.uint64)
    lib.dcfm_debug_xs.argtypes = [C.c_void_p]
    lib.dcfm_debug_xs(xs.ctypes.data)
    for j in range(nxs):
        print("xsum", j, " ".join(f"{(int(v) - int(t0)) / 100.0:7.2f}" if v else "   -   " for v in xs[j]))
    print("chol_inv32 done", (int(xs[63][5]) - int(t0)) / 100.0)
