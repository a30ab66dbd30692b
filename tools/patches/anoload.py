"""A/B (timing only, wrong results): k_assemble cross tiles start from zero (no Sigma read)."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "                for (int g = 0; g < 4; ++g) acc[u][v][g] = St[(wa + 16 * u + q + 4 * g) * ASM_TILE + wb + 16 * v + r];"
assert old in s
s = s.replace(old, "                for (int g = 0; g < 4; ++g) acc[u][v][g] = 0.0;")
open(f, "w").write(s)
