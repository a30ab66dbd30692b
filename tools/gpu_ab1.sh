#!/bin/bash
# A/B on the driver's c3 command only (per-kernel event table), product build vs variants;
# a variant whose chain fails is reported and skipped.  Usage: bash tools/gpu_ab1.sh TAG [variant...]
TAG=$1; shift
mkdir -p gpurun_out
for V in base "$@"; do
  if [ "$V" = base ]; then unset DCFM_LIB; else export DCFM_LIB=build/libdcfm_$V.so; fi
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --converged-mcmc 0 --err-iters 0 --no-cpu-baseline > gpurun_out/ab_${TAG}_$V.json 2> gpurun_out/ab_${TAG}_$V.err
  rc=$?
  [ $rc -ge 124 ] && { echo "$V: timeout/kill rc=$rc"; exit 1; }
  [ $rc -ne 0 ] && { echo "$V failed rc=$rc"; tail -3 gpurun_out/ab_${TAG}_$V.err; rm -f gpurun_out/ab_${TAG}_$V.json; }
done
python3 tools/show_bench.py gpurun_out/ab_${TAG}_*.json
