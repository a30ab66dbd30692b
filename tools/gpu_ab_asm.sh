#!/bin/bash
# A/B of the product build against named variants on the assembly-heavy shapes: the driver's
# c3 command (one 4-sample flush) and 480 c3 steps (96-sample flushes).  Usage: bash tools/gpu_ab_asm.sh TAG [variant...]
TAG=$1; shift
mkdir -p gpurun_out
declare -A CFG
CFG[c3]="--gpus 1 --steps 20 --warmup 5 --converged-mcmc 0"
CFG[c3l]="--steps 480 --warmup 20 --converged-mcmc 0"
for S in c3 c3l; do
  for V in base "$@"; do
    if [ "$V" = base ]; then unset DCFM_LIB; else export DCFM_LIB=build/libdcfm_$V.so; fi
    timeout -k 10 200 python3 -u bench.py ${CFG[$S]} --no-cpu-baseline > gpurun_out/ab_${TAG}_${S}_$V.json 2> gpurun_out/ab_${TAG}_${S}_$V.err || { echo "$S $V bench failed"; tail gpurun_out/ab_${TAG}_${S}_$V.err; exit 1; }
  done
done
python3 tools/show_bench.py gpurun_out/ab_${TAG}_*.json
