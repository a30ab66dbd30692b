"""A/B timing only (wrong numbers): k_wcol without the operator roles."""
import sys
f = sys.argv[1] + "/dcfm.hip"
s = open(f).read()
old = "if (int rc = wcol(true, delta_pending, true, it)) return rc;"
assert old in s
s = s.replace(old, "if (int rc = wcol(false, delta_pending, true, it)) return rc;")
open(f, "w").write(s)
