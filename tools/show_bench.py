"""Compact view of bench.py JSON lines (dev aid).  Usage: python tools/show_bench.py FILE..."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    print(f, d["value"], "it/s", d["ms_per_step"], "ms/it", "roof", r.get("kernel"), r.get("frac"))
    print("   " + "  ".join(f"{k}={v['avg_us']:.1f}" for k, v in d["kernels"].items()))
