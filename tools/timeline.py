"""Per-iteration kernel timeline from a rocprofv3 kernel trace (dev aid).
Usage: python tools/timeline.py gpurun_out/prof_TAG [anchor_kernel]"""
import csv, glob, re, sys
from collections import defaultdict
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
anchor = sys.argv[2] if len(sys.argv) > 2 else None
ev = []
for r in rows:
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    k = m.group(1) if m else r["Kernel_Name"][:20]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r["Queue_Id"]))
ev.sort()
if anchor is None:
    anchor = "k_wprep" if any(e[2] == "k_wprep" for e in ev) else "k_wpass"
w = [e[0] for e in ev if e[2] == anchor]
t0, t1 = w[-20], w[-10]
win = [e for e in ev if t0 <= e[0] < t1]
tot = defaultdict(float)
for s, e, k, q in win:
    tot[k] += (e - s) / 10 / 1000
print(f"wall per iteration {(t1 - t0) / 10 / 1000:.1f} us")
for k, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {k:14s} {v:7.1f} us/iter")
print("one iteration:")
for s, e, k, q in [x for x in ev if w[-12] <= x[0] < w[-11]]:
    print(f"  {(s - w[-12]) / 1000:8.1f} {(e - w[-12]) / 1000:8.1f}  {k:12s} q{q}")
