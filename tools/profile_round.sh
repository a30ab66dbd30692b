#!/bin/bash
# rocprofv3 evidence for one bench configuration (run on the GPU box):
#   1. --kernel-trace --stats       per-kernel durations
#   2-5. separate --pmc passes       FETCH_SIZE | WRITE_SIZE | fp64 MFMA ops + busy cycles | wave states
# Default bench arguments = the driver's command (bench.py --gpus 1 --steps 20 --warmup 5), so
# the PMC summary's config key matches the driver's bench line (bench.py pmc_traffic).
# Usage: bash tools/profile_round.sh TAG [bench args...]     (outputs under gpurun_out/prof_TAG*)
set -o pipefail
TAG=$1; shift
ARGS="$@"
[ -z "$ARGS" ] && ARGS="--gpus 1 --steps 20 --warmup 5"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out
BENCH="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --converged-mcmc 0 $ARGS"   # no converged leg: the summary takes the timed region as the last dispatches
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG} -o run -- $BENCH > $OUT/prof_${TAG}.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_${TAG}_fetch -o run -- $BENCH > $OUT/prof_${TAG}_fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_${TAG}_write -o run -- $BENCH > $OUT/prof_${TAG}_write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_${TAG}_mfma -o run -- $BENCH > $OUT/prof_${TAG}_mfma.log 2>&1 || { echo "mfma pass failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/prof_${TAG}_waves -o run -- $BENCH > $OUT/prof_${TAG}_waves.log 2>&1 || { echo "waves pass failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py gpurun_out/prof_${TAG} > gpurun_out/prof_${TAG}_pmc.json || { echo "summary failed"; exit 1; }
find $OUT -path "*prof_${TAG}*" -name "*.csv" -size +512k -exec gzip -9 {} \;   # keep gpurun_out small
echo "profile $TAG ok"
