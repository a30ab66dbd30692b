"""A/B: k_lambda with its in-place draws replaced by constants (cost of the draw code)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
a = s.index("        const Rng rng(d.seed);\n        const uint32_t it32 = (uint32_t)iter, mg32 = (uint32_t)mg, j32 = (uint32_t)jj;\n        // lane l draws normal pairs l and l + 8")
b = s.index("    // ---- Q_j rows r_b, columns <= 8b + 7")
body = s[a:b]
end = body.rindex("    }\n")
s = s[:a] + "        for (int b = 0; b < 4; ++b) { z[b] = rv[b] ? 0.01 * (l + b) : 0.0; G[b] = rv[b] ? 1.0 : 0.0; }\n        Gps = (valid && l == 0) ? 500.0 : 0.0;\n" + body[end:] + s[b:]
open(f, "w").write(s)
