#!/bin/bash
TAG=${1:-r4h}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
bash tools/gpu_ab.sh ${TAG}c3 2 base g1 g1nog || exit 1
BENCH_EXTRA="--g 8 --P 1250 --n 2000 --K 100 --steps 50 --warmup 5" bash tools/gpu_ab.sh ${TAG}c4 2 cpw_old g1 || exit 1
echo all done
