"""Dev aid: block stamps (s_memrealtime, 100 MHz) of the last full k_wcol launch at c3, by role
(OPS, colsum, A-sum chunks, W tiles, loading-row variates); needs a variant built with
-DDCFM_WSTAMPS (bash tools/build_variant.sh wst -DDCFM_WSTAMPS); run with DCFM_LIB=build/libdcfm_wst.so."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as ge  # noqa: E402
import bench  # noqa: E402

dcfm = ge.load_package()
g, P, n, K = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (64, 312, 1000, 30)))
Y = bench.synth_data(n, g * P)
smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 100000, 100000, seed=1)
smp.set_data_raw(Y, np.arange(g * P))
smp.init_state()
smp.run(1, 26)
smp.synchronize()
lib = smp.lib
lib.dcfm_debug_wstamps.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros((8192, 2), dtype=np.uint64)
lib.dcfm_debug_wstamps(buf.ctypes.data, 8192)
nb = int(np.max(np.nonzero(buf[:, 0])[0])) + 1
b = buf[:nb].astype(np.int64)
t0 = b[:, 0].min()
st, en = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0
G = g
nxs = 1
while G // nxs > 8 and (G // nxs) % 2 == 0:
    nxs *= 2
NP = (n + 127) // 128 * 128
nw = NP // 128 * G
roles = [("OPS", 0, G), ("colsum", G, 2 * G)]
# the A-sum blocks: whatever lies between colsum and the W tiles
nsum = nb - 2 * G - nw
lamb = 0
# the W tiles are the run of nw blocks after the sums; lam blocks follow
for ns in range(0, 65):
    pass
print(f"blocks with stamps: {nb}")
for name, lo, hi in roles:
    print(f"{name:8s} [{lo},{hi}) start med {np.median(st[lo:hi]):7.2f} max {st[lo:hi].max():7.2f}  end med {np.median(en[lo:hi]):7.2f} max {en[lo:hi].max():7.2f} us")
# print the rest in windows of 64 blocks
for lo in range(2 * G, nb, 64):
    hi = min(nb, lo + 64)
    print(f"blk [{lo},{hi}) start min {st[lo:hi].min():7.2f} med {np.median(st[lo:hi]):7.2f} max {st[lo:hi].max():7.2f}  end min {en[lo:hi].min():7.2f} med {np.median(en[lo:hi]):7.2f} max {en[lo:hi].max():7.2f} us")
print(f"launch span {en.max():.2f} us")
