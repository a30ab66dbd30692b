"""dev: print one kernel's trace stats and per-wave PMC figures (tools/kprof.sh output)."""
import csv
import glob
import sys
from collections import defaultdict

base, kern = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{base}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Name"]:
            print(f"  trace: calls {r['Calls']} avg {float(r['AverageNs']) / 1000:.1f} us  min {float(r['MinNs']) / 1000:.1f}  max {float(r['MaxNs']) / 1000:.1f}")
def pmc(suffix):
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(f"{base}{suffix}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"].split("(")[0]:
                acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


acc = pmc("_w")
if acc:
    n = len(acc)
    m = {c: sum(d[c] for d in acc.values()) / n for c in next(iter(acc.values()))}
    w = m.get("SQ_WAVES", 1)
    print(f"  pmc ({n} dispatches): waves {w:.0f}  valu/wave {m['SQ_INSTS_VALU'] / w:.0f}  lds/wave {m['SQ_INSTS_LDS'] / w:.0f}  "
          f"salu/wave {m['SQ_INSTS_SALU'] / w:.0f}  wave_cycles/wave {m['SQ_WAVE_CYCLES'] / w:.0f}  "
          f"active_valu/wave {m['SQ_ACTIVE_INST_VALU'] / w:.0f}  wait_inst/wave {m['SQ_WAIT_INST_ANY'] / w:.0f}  busy {m['SQ_BUSY_CYCLES']:.0f}")
acc = pmc("_w2")
if acc:
    n = len(acc)
    m = {c: sum(d[c] for d in acc.values()) / n for c in next(iter(acc.values()))}
    w = m.get("SQ_WAVES", 1)
    print("  per wave (quad-cycles): " + "  ".join(f"{c[3:]} {m[c] / w:.0f}" for c in m if c != "SQ_WAVES"))
