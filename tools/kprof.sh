#!/bin/bash
# dev: kernel-trace stats + one wave-state PMC pass of the driver's bench for a named kernel,
# under each given environment setting.  Usage: bash tools/kprof.sh TAG KERNEL "ENV=.." ["ENV=.."...]
set -o pipefail
TAG=$1; K=$2; shift 2
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
BENCH="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --gpus 1 --steps 20 --warmup 5"
i=0
for E in "$@"; do
  cd /tmp
  env $E timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kp_${TAG}_$i -o run -- $BENCH > $OUT/kp_${TAG}_$i.log 2>&1 || { echo "trace $E failed"; exit 1; }
  if [ -z "$KPROF_TRACE_ONLY" ]; then
  env $E timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/kp_${TAG}_${i}_w -o run -- $BENCH > $OUT/kp_${TAG}_${i}_w.log 2>&1 || { echo "pmc $E failed"; exit 1; }
  env $E timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $OUT/kp_${TAG}_${i}_w2 -o run -- $BENCH > $OUT/kp_${TAG}_${i}_w2.log 2>&1 || { echo "pmc2 $E failed"; exit 1; }
  fi
  cd $GRAFT_REPO_ROOT
  echo "== $E"
  python3 tools/kprof_show.py $OUT/kp_${TAG}_$i $K
  i=$((i+1))
done
