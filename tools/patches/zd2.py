"""A/B: wide k_zdraw with 2 row tiles per block."""
import sys, pathlib
p = pathlib.Path(sys.argv[1]) / "kernels_wide.hip"
s = p.read_text()
assert s.count("#define DCFM_ZD_RT 1") == 1
p.write_text(s.replace("#define DCFM_ZD_RT 1", "#define DCFM_ZD_RT 2"))
