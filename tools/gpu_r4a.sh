#!/bin/bash
# round 4 iteration: every GPU test, the driver's bench with and without the exact residual, and
# a rocprofv3 kernel trace of the driver's command.  Usage: bash tools/gpu_r4a.sh TAG [quick]
TAG=${1:-r4a}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$2" != "notest" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_$TAG.log | tail -1
fi
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > gpurun_out/bench_drv_$TAG.json 2> gpurun_out/bench_drv_$TAG.err || { echo "driver bench failed"; tail gpurun_out/bench_drv_$TAG.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --exact-residual > gpurun_out/bench_ex_$TAG.json 2> gpurun_out/bench_ex_$TAG.err || { echo "exact bench failed"; tail gpurun_out/bench_ex_$TAG.err; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_drv_$TAG.json gpurun_out/bench_ex_$TAG.json
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --converged-mcmc 0 --gpus 1 --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1 || { echo "trace failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/kavg.py gpurun_out/prof_$TAG 2>/dev/null | head -30
find gpurun_out -path "*prof_${TAG}*" -name "*.csv" -size +512k -exec gzip -9 {} \;
echo done
for AB in 1 2; do
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --asm-batch $AB > gpurun_out/bench_ab${AB}_$TAG.json 2> gpurun_out/bench_ab${AB}_$TAG.err || { echo "ab bench failed"; exit 1; }
done
python3 tools/show_bench.py gpurun_out/bench_ab1_$TAG.json gpurun_out/bench_ab2_$TAG.json
