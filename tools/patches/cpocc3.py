"""A/B: k_cpass with __launch_bounds__(256, 3) (<= 168 VGPRs: 3 waves per SIMD)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "__global__ __launch_bounds__(256) void k_cpass(Dims d,"
assert old in s
s = s.replace(old, "__global__ __launch_bounds__(256, 3) void k_cpass(Dims d,")
open(f, "w").write(s)
