#!/bin/bash
# One development iteration on the box: all GPU tests, smoke, the driver's bench command, and
# the kernel-trace timelines of c3 and the g = 8 share (tools/ktrace2.sh).  Stops at the first
# failing step.  Usage: bash tools/gpu_iter.sh TAG [pytest args...]
TAG=$1; shift
T=${@:-tests}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed $?"; grep -E "FAIL|Error|assert|rel" gpurun_out/t_$TAG.log | head -30; tail -15 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_$TAG.json
bash tools/ktrace2.sh $TAG || exit 1
head -8 gpurun_out/kt_${TAG}_c3.timeline
head -8 gpurun_out/kt_${TAG}_g8.timeline
