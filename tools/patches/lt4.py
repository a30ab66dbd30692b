"""A/B: k_lambda_t at 4 waves/SIMD (launch bound min 4 blocks: 128 VGPRs, some spills)."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels_wide.hip"
s = p.read_text()
assert s.count("#define DCFM_LT_MINW 3") == 1
p.write_text(s.replace("#define DCFM_LT_MINW 3", "#define DCFM_LT_MINW 4"))
