"""A/B (timing only, wrong results): k_assemble cross tiles skip their stores."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "                for (int g = 0; g < 4; ++g) St[(wa + 16 * u + q + 4 * g) * ASM_TILE + wb + 16 * v + r] = acc[u][v][g];\n        return;"
assert old in s
s = s.replace(old, "                for (int g = 0; g < 4; ++g) if (acc[u][v][g] == 1.2345e300) St[(wa + 16 * u + q + 4 * g) * ASM_TILE + wb + 16 * v + r] = acc[u][v][g];\n        return;")
open(f, "w").write(s)
