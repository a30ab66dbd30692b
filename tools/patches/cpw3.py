"""Dev A/B: k_cpass held to 3 waves per SIMD (<= 168 registers) so the c3 grid fits one round."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "__global__ __launch_bounds__(64 * cp_waves<KW>()) void k_cpass("
assert old in s
s = s.replace(old, "__global__ __launch_bounds__(64 * cp_waves<KW>()) __attribute__((amdgpu_waves_per_eu(3))) void k_cpass(")
open(f, "w").write(s)
