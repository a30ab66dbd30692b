"""A/B: k_lambda trailing update without the per-chunk scheduling barriers."""
import sys
f = sys.argv[1] + "/kernels.hip"
s = open(f).read()
old = "            __builtin_amdgcn_sched_barrier(0);\n        });\n    });"
assert old in s
s = s.replace(old, "        });\n    });")
open(f, "w").write(s)
