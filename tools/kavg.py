"""Median / mean duration per kernel name from rocprofv3 kernel traces (dev aid).
Usage: python tools/kavg.py gpurun_out/prof_A [gpurun_out/prof_B ...]"""
import collections
import csv
import glob
import gzip
import statistics
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*kernel_trace.csv*", recursive=True):
        fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dcfm::", "")
            agg[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(d)
    for k, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:12]:
        print(f"   {k:40s} n={len(v):5d} median={statistics.median(v):9.1f} us  mean={sum(v) / len(v):9.1f} us")
