"""A/B: k_lambda_t diagonal factorisation on wave (J + blockIdx.x) & 3 instead of wave 0
(spreads the serial chol_inv16 chains of co-resident rows over the CU's four SIMDs)."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels_wide.hip"
s = p.read_text()
old = "        __syncthreads();\n        if (wave == 0) {\n            chol_inv16_p<LD>(Sd, 0, Ud, lds_l, lds_u, lane);"
assert s.count(old) == 1
s = s.replace(old, "        __syncthreads();\n        if (wave == ((J + (int)blockIdx.x) & 3)) {\n            chol_inv16_p<LD>(Sd, 0, Ud, lds_l, lds_u, lane);")
p.write_text(s)
