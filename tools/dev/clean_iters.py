"""Dev aid: start-to-start spacing of the loading-row kernel in rocprofv3 kernel traces, over the
iterations with no chain-trace / save / assembly launch in them ("clean" sweep iterations).
Usage: python tools/dev/clean_iters.py gpurun_out/abprof_TAG_V [...]"""
import csv
import glob
import gzip
import statistics
import sys

for d in sys.argv[1:]:
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv*", recursive=True):
        for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    lam = [i for i, r in enumerate(rows) if "k_lambda" in r[1]]
    cl = [(rows[b][0] - rows[a][0]) / 1000 for a, b in zip(lam, lam[1:])
          if not any(k in r[1] for r in rows[a:b] for k in ("trace", "assemble", "save"))]
    if cl:
        print(f"{d}: clean iterations {len(cl)}, median {statistics.median(cl):.1f} us")
