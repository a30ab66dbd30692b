#!/bin/bash
# A/B of library builds on the box: build/ab/libdcfm_<V>.so for each variant V, the driver's
# bench command interleaved R times, then one rocprofv3 kernel trace per variant.
# Usage: bash tools/gpu_ab.sh TAG R V1 V2 ...      (restores the in-tree build at the end)
TAG=$1; R=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
mkdir -p gpurun_out; export TMPDIR=/tmp
cp $PKG/libdcfm.so /tmp/libdcfm_intree.so
trap 'cp /tmp/libdcfm_intree.so "$ROOT/$PKG/libdcfm.so"' EXIT   # the product build comes back on any exit
BENCH="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 $BENCH_EXTRA"
for r in $(seq 1 $R); do
  for V in "$@"; do
    cp build/ab/libdcfm_$V.so $PKG/libdcfm.so
    timeout -k 10 200 python3 -u $BENCH > gpurun_out/ab_${TAG}_${V}_$r.json 2> gpurun_out/ab_${TAG}_${V}_$r.err || { echo "bench $V failed"; tail -5 gpurun_out/ab_${TAG}_${V}_$r.err; cp /tmp/libdcfm_intree.so $PKG/libdcfm.so; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})" gpurun_out/ab_${TAG}_${V}_$r.json $V
  done
done
for V in "$@"; do
  cp build/ab/libdcfm_$V.so $PKG/libdcfm.so
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/abprof_${TAG}_$V -o run -- python3 $ROOT/$BENCH > $ROOT/gpurun_out/abprof_${TAG}_$V.log 2>&1) || { echo "trace $V failed"; cp /tmp/libdcfm_intree.so $PKG/libdcfm.so; exit 1; }
  python3 tools/kavg.py gpurun_out/abprof_${TAG}_$V
  find gpurun_out -path "*abprof_${TAG}_$V*" -name "*.csv" -size +512k -exec gzip -9 {} \;
done
cp /tmp/libdcfm_intree.so $PKG/libdcfm.so
echo ab done
