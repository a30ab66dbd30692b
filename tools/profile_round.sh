#!/bin/bash
# rocprofv3 evidence for one bench configuration (run on the GPU box):
#   1. --kernel-trace --stats       per-kernel durations
#   2-4. separate --pmc passes       FETCH_SIZE | WRITE_SIZE | fp64 MFMA ops + busy cycles
# Usage: bash tools/profile_round.sh TAG [bench args...]     (outputs under gpurun_out/prof_TAG*)
set -o pipefail
TAG=$1; shift
ARGS="$@"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
BENCH="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 40 --warmup 5 $ARGS"
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG} -o run -- $BENCH > $OUT/prof_${TAG}.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_${TAG}_fetch -o run -- $BENCH > $OUT/prof_${TAG}_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_${TAG}_write -o run -- $BENCH > $OUT/prof_${TAG}_write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_${TAG}_mfma -o run -- $BENCH > $OUT/prof_${TAG}_mfma.log 2>&1 || { echo "mfma pass failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/prof_${TAG}_waves -o run -- $BENCH > $OUT/prof_${TAG}_waves.log 2>&1 || { echo "waves pass failed"; exit 1; }
echo "profile $TAG ok"
