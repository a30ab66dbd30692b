"""Per-phase shader-clock cycles of k_lambda (dev aid; needs build/libdcfm_phase.so)."""
import ctypes as C, os, sys
os.environ["DCFM_LIB"] = os.path.abspath("build/libdcfm_phase.so")
sys.path.insert(0, ".")
import numpy as np
import __graft_entry__ as ge
import bench
dcfm = ge.load_package()
g, P, n, K = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (64, 312, 1000, 30)))
p = g * P
Y = bench.synth_data(n, p)
hyper = dcfm.Hyper()
Yk, n, pk, P, K_, keep = dcfm.preprocess(Y, g, K * g)
init = dcfm.driver._HostInitDraws(1, n, pk, g, K, hyper)
Yd = dcfm.partition_standardize(Yk, g, init.varind)
state = dcfm.initial_state(n, P, K, g, 0.5, hyper, init)
smp = dcfm.Sampler(n, P, g, K, 0.5, 0, 100, 1000, seed=1)
smp.set_data(Yd); smp.set_state(dcfm.local_state(state, 0, g))
lib = smp.lib
lib.dcfm_debug_phases.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * 32)()
smp.run(1, 10); smp.synchronize(); lib.dcfm_debug_phases(buf)
T = 20
smp.run(11, T); smp.synchronize(); lib.dcfm_debug_phases(buf)
waves = ((P + 3) // 4) * g if K <= 32 else P * g * 3
tot = sum(buf[:8])
for k in range(8):
    if buf[k]:
        print(f"phase {k}: {buf[k] / waves / T:10.0f} cycles/wave  ({100 * buf[k] / tot:.1f}%)")
