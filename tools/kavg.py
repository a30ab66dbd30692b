"""Average duration per kernel name from rocprofv3 kernel traces (dev aid).
Usage: python tools/kavg.py gpurun_out/vp_A [gpurun_out/vp_B ...]"""
import csv, glob, sys, collections
for d in sys.argv[1:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dcfm::", "")
            agg[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(d, " ".join(f"{k}={sum(v)/len(v):.0f}" for k, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:6]))
