#!/bin/bash
# A/B benches: the product build and each named variant (build/libdcfm_NAME.so) on the
# driver's c3 command (or on BENCH_ARGS, e.g. the c4 shape).  Usage: bash tools/gpu_ab.sh TAG [variant...]
TAG=$1; shift
ARGS=${BENCH_ARGS:---gpus 1 --steps 20 --warmup 5}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab_${TAG}_base.json 2> gpurun_out/ab_${TAG}_base.err || { echo "base bench failed"; tail gpurun_out/ab_${TAG}_base.err; exit 1; }
for V in "$@"; do
  DCFM_LIB=build/libdcfm_$V.so timeout -k 10 200 python3 -u bench.py $ARGS --no-cpu-baseline > gpurun_out/ab_${TAG}_$V.json 2> gpurun_out/ab_${TAG}_$V.err || { echo "$V bench failed"; tail gpurun_out/ab_${TAG}_$V.err; exit 1; }
done
python3 tools/show_bench.py gpurun_out/ab_${TAG}_*.json
