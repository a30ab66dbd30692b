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
buf = np.zeros((8192, 8), dtype=np.uint64)
lib.dcfm_debug_wstamps(buf.ctypes.data, 8192)
nb = int(np.max(np.nonzero(buf[:, 0])[0])) + 1
b = buf[:nb].astype(np.int64)
t0 = b[:, 0].min()
st, en = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0
s2, s3, s4, s5 = ((b[:, k] - t0) / 100.0 for k in (2, 3, 4, 5))
G = g
nxs = 1 if G <= 8 else G
if G > 8:
    chunk = 1
    while G // chunk > 8 and (G // chunk) % 2 == 0:
        chunk *= 2
    nxs = G // chunk
NP = (n + 127) // 128 * 128
import os
wmode = int(os.environ.get("WMODE", "0")) or (3 if (NP // 32) * G >= 1024 else 4)   # kernels.hip wcol_mode
rows = {1: 128, 2: 64, 3: 32, 4: 16}[wmode]
nw = NP // rows * G
w0 = 2 * G + nxs


def line(name, lo, hi, *cols):
    out = f"{name:10s} [{lo},{hi})"
    for lab, v in cols:
        out += f"  {lab} med {np.median(v[lo:hi]):6.2f} max {v[lo:hi].max():6.2f}"
    print(out)


print(f"blocks with stamps: {nb}  (G {G}, A-sum blocks {nxs}, W tiles {nw} of {rows} rows, mode {wmode})")
line("OPS", 0, G, ("start", st), ("A out", s2), ("U out", s3), ("end", en))
line("colsum", G, 2 * G, ("start", st), ("end", en))
line("A-sum", 2 * G, w0, ("start", st), ("end", en))
line("W tiles", w0, w0 + nw, ("start", st), ("pass", s2), ("ops in", s3), ("staged", s4), ("draw 1", s5), ("end", en))
tail = en[w0:w0 + nw] - s5[w0:w0 + nw]
print(f"W tiles end - draw: med {np.median(tail):.2f} max {tail.max():.2f} us; end percentiles 50/90/99/100: "
      + " ".join(f"{np.percentile(en[w0:w0 + nw], q):.2f}" for q in (50, 90, 99, 100)))
if nb > w0 + nw:
    line("lam gen", w0 + nw, nb, ("start", st), ("end", en))
clk = (b[:, 7] - b[:, 6]) / np.maximum(b[:, 1] - b[:, 0], 1) * 100e6 / 1e9   # GHz
print(f"W tiles shader clock (GHz): med {np.median(clk[w0:w0 + nw]):.3f} min {clk[w0:w0 + nw].min():.3f} max {clk[w0:w0 + nw].max():.3f}")
print(f"launch span {en.max():.2f} us")
