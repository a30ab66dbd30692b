#!/bin/bash
# One GPU round on the box: GPU tests, smoke, bench (+ optional rocprof). Each step time-limited;
# stops at the first failing step.  Usage: bash tools/gpu_round.sh TAG [prof]
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed $?"; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; exit 1; }
echo "bench ok"
if [ "$2" == "prof" ]; then
  export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-profile > gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; exit 1; }
  echo "prof ok"
fi
