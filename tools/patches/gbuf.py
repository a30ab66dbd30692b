"""A/B timing only: the delta chain reads the draw buffer instead of drawing its gammas."""
import sys
f = sys.argv[1] + "/linalg.h"
s = open(f).read()
old = "    if (d.inject) return dr.Gdelta["
assert old in s
s = s.replace(old, "    if (true) return dr.Gdelta[")
open(f, "w").write(s)
