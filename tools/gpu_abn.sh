#!/bin/bash
# Alternating benches of several library builds (dev aid, run on the GPU box): "main" = the
# in-tree libdcfm.so, any other name = build/libdcfm_NAME.so.  R rounds, each build once per
# round, to separate a change from box drift.  Prints it/s and the per-kernel averages.
# Usage: BENCH_ARGS="..." bash tools/gpu_abn.sh TAG R NAME...
TAG=$1; R=$2; shift 2
ARGS=${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
mkdir -p gpurun_out
for i in $(seq $R); do
  for V in "$@"; do
    LIB=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd/libdcfm.so
    [ "$V" != main ] && LIB=build/libdcfm_$V.so
    DCFM_LIB=$LIB timeout -k 10 200 python3 -u bench.py $ARGS --no-cpu-baseline > gpurun_out/abn_${TAG}_${V}_$i.json 2> gpurun_out/abn_${TAG}_${V}_$i.err || { echo "$V bench failed"; tail -5 gpurun_out/abn_${TAG}_${V}_$i.err; exit 1; }
  done
done
python3 - "$TAG" "$R" "$@" <<'PY'
import json, sys
tag, r, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for v in names:
    runs = [json.loads(open(f"gpurun_out/abn_{tag}_{v}_{i}.json").read().strip().splitlines()[-1]) for i in range(1, r + 1)]
    vals = [d["value"] for d in runs]
    ks = {}
    for d in runs:
        for k, x in d["kernels"].items():
            ks.setdefault(k, []).append(x["avg_us"])
    print(f"{v:10s} " + " ".join(f"{x:9.1f}" for x in vals) + f"   mean {sum(vals) / len(vals):9.1f}")
    print("           " + "  ".join(f"{k}={sum(x) / len(x):.1f}" for k, x in ks.items()))
PY
