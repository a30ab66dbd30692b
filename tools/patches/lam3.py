"""A/B: k_lambda limited to 3 waves per SIMD worth of registers."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "__global__ __launch_bounds__(64) void k_lambda("
assert old in s
s = s.replace(old, "__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k_lambda(")
open(f, "w").write(s)
