#!/bin/bash
# GPU tests + smoke + the driver's bench + the g = 8 share bench (no profiling); stops at the
# first failing step.  Usage: bash tools/gpu_quick3.sh TAG
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed $?"; grep -E "FAIL|Error|assert" gpurun_out/t_$TAG.log | head -20; tail -30 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --g 8 --thin 100000 --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/bench_${TAG}_g8.json 2> gpurun_out/bench_${TAG}_g8.err || { echo "g8 bench failed"; tail gpurun_out/bench_${TAG}_g8.err; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_$TAG.json gpurun_out/bench_${TAG}_g8.json
# kernel trace of the g = 8 share (strong-scaling floor): per-kernel durations vs the iteration
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_g8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --g 8 --thin 100000 --steps 2000 --warmup 100 --no-cpu-baseline --no-profile --converged-mcmc 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}_g8.log 2>&1 ) || { echo "g8 trace failed"; exit 1; }
echo "g8 trace ok"
