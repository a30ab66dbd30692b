"""Role completion stamps of one k_wprep / k_zxchol launch at c3 (dev aid; needs
build/libdcfm_phase.so from tools/build_variant.sh phase -DDCFM_PHASE_TIMING)."""
import ctypes as C, os, sys
os.environ["DCFM_LIB"] = os.path.abspath("build/libdcfm_phase.so")
sys.path.insert(0, ".")
import __graft_entry__ as ge
import bench
dcfm = ge.load_package()
g, P, n, K = 64, 312, 1000, 30
Y = bench.synth_data(n, g * P)
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
for it in range(11, 16):
    smp.run(it, 1); smp.synchronize(); lib.dcfm_debug_phases(buf)
    t0 = (~buf[24]) & 0xFFFFFFFFFFFFFFFF
    t1 = (~buf[28]) & 0xFFFFFFFFFFFFFFFF
    f = lambda v, t: (v - t) if v else -1
    print(f"k_wprep: prep end {f(buf[25], t0)}  tree end {f(buf[26], t0)}  W tiles end {f(buf[27], t0)} x10ns | "
          f"k_zxchol: Z tiles end {f(buf[29], t1)}  X ops end {f(buf[30], t1)} x10ns")
