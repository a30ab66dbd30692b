#!/bin/bash
# round 4: GPU tests on the in-tree build, then A/B of build variants
TAG=${1:-r4b}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
bash tools/gpu_ab.sh $TAG 2 "$@"
