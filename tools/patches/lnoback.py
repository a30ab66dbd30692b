"""A/B: k_lambda without the back solve (x = 0; cost of the back solve)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
a = s.index("    static_for<KP / 2>([&](auto JC) {\n        constexpr int c = KP - 1 - 2 * decltype(JC)::value;     // odd; c and c-1 in block cb")
b = s.index("#pragma unroll\n    for (int b = 0; b < 4; ++b)\n        if (!rv[b]) x[b] = 0.0;")
s = s[:a] + "    for (int b = 0; b < 4; ++b) { x[b] = q3[b] + z[b]; ww += q2[b]; wv += q1[b]; }\n" + s[b:]
open(f, "w").write(s)
