#!/bin/bash
# Alternating A/B benches (product build vs build/libdcfm_V.so), R rounds each, to separate a
# change from box drift.  Usage: bash tools/gpu_abab.sh TAG V R   (BENCH_ARGS as gpu_ab.sh)
TAG=$1; V=$2; R=${3:-3}
ARGS=${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
mkdir -p gpurun_out
for i in $(seq $R); do
  timeout -k 10 200 python3 -u bench.py $ARGS --no-cpu-baseline > gpurun_out/abab_${TAG}_base_$i.json 2>/dev/null || { echo "base bench failed"; exit 1; }
  DCFM_LIB=build/libdcfm_$V.so timeout -k 10 200 python3 -u bench.py $ARGS --no-cpu-baseline > gpurun_out/abab_${TAG}_${V}_$i.json 2>/dev/null || { echo "$V bench failed"; exit 1; }
done
python3 - "$TAG" "$V" "$R" <<'PY'
import json, sys
tag, v, r = sys.argv[1], sys.argv[2], int(sys.argv[3])
for name in ("base", v):
    vals = [json.load(open(f"gpurun_out/abab_{tag}_{name}_{i}.json"))["value"] for i in range(1, r + 1)]
    print(f"{name:8s} " + " ".join(f"{x:9.1f}" for x in vals) + f"   mean {sum(vals) / len(vals):9.1f}")
PY
