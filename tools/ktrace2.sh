#!/bin/bash
# Kernel traces (no counters) of the driver's c3 command and of the g = 8 share (run on the GPU
# box); per-kernel stats + the iteration's inter-kernel gap share from the trace (timeline.py),
# big CSVs gzipped so gpurun_out stays small.  Usage: bash tools/ktrace2.sh TAG
set -o pipefail
TAG=$1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
run() {   # name, bench args
  local N=$1; shift
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${TAG}_$N -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline "$@" > $OUT/kt_${TAG}_$N.log 2>&1 ) || { echo "trace $N failed"; return 1; }
  python3 tools/timeline.py $OUT/kt_${TAG}_$N k_wcol > $OUT/kt_${TAG}_$N.timeline 2>&1 || true
  find $OUT/kt_${TAG}_$N -name "*.csv" -size +512k -exec gzip -9 {} \;
  echo "trace $N ok"
}
run c3 --gpus 1 --steps 20 --warmup 5 --converged-mcmc 0 || exit 1
run g8 --g 8 --thin 100000 --steps 2000 --warmup 100 --no-profile --converged-mcmc 0 || exit 1
du -sh $OUT
