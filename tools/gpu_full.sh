#!/bin/bash
# Full GPU round on the box: all GPU tests, smoke, the driver's bench command, then the
# rocprofv3 kernel trace + PMC passes of that same command.  Each step time-limited; stops at
# the first failing step.  Usage: bash tools/gpu_full.sh TAG [noprof]
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
echo "bench ok"
if [ "$2" != "noprof" ]; then
  bash tools/profile_round.sh $TAG || exit 1
fi
