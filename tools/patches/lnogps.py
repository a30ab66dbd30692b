"""A/B: k_lambda with the ps gamma (shape as + n/2, Marsaglia-Tsang) replaced by a constant."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "        Gps = (valid && l == 0) ? rng.gamma(d.as_ + 0.5 * d.n, SITE_PS, mg32, j32, 0u, it32) : 0.0;\n    }\n    // ---- Q_j rows"
assert old in s
s = s.replace(old, "        Gps = (valid && l == 0) ? 500.0 : 0.0;\n    }\n    // ---- Q_j rows")
open(f, "w").write(s)
