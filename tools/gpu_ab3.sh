#!/bin/bash
# A/B of the product build against named variants (build/libdcfm_NAME.so) on three shapes:
# the driver's c3 command, the g = 8 share, and the c4 shape.  Usage: bash tools/gpu_ab3.sh TAG [variant...]
TAG=$1; shift
mkdir -p gpurun_out
declare -A CFG
CFG[c3]="--gpus 1 --steps 20 --warmup 5 --converged-mcmc 0 --err-iters 0"
CFG[g8]="--g 8 --thin 100000 --steps 2000 --warmup 100 --no-profile --converged-mcmc 0"
CFG[c4]="--g 8 --P 1250 --n 2000 --K 100 --steps 50 --warmup 5 --converged-mcmc 0"
for S in ${SHAPES:-c3 g8 c4}; do
  for V in base "$@"; do
    if [ "$V" = base ]; then unset DCFM_LIB; else export DCFM_LIB=build/libdcfm_$V.so; fi
    timeout -k 10 200 python3 -u bench.py ${CFG[$S]} --no-cpu-baseline > gpurun_out/ab_${TAG}_${S}_$V.json 2> gpurun_out/ab_${TAG}_${S}_$V.err || { echo "$S $V bench failed"; tail gpurun_out/ab_${TAG}_${S}_$V.err; exit 1; }
  done
done
python3 tools/show_bench.py gpurun_out/ab_${TAG}_*.json
