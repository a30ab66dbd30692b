import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, d["value"], "it/s", d["ms_per_step"], "ms/it")
    print("   " + "  ".join(f"{k}={v['avg_us']:.0f}" for k, v in d["kernels"].items()))
