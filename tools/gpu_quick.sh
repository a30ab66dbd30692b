#!/bin/bash
# quick GPU check: parity tests, then c3 and c4 benches (no CPU baseline). Usage: bash tools/gpu_quick.sh TAG
TAG=${1:-q}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || { echo "c3 bench failed"; tail gpurun_out/bench_c3_$TAG.err; exit 1; }
timeout -k 10 200 python -u bench.py --g 8 --P 1250 --n 2000 --K 100 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || { echo "c4 bench failed"; tail gpurun_out/bench_c4_$TAG.err; exit 1; }
echo done
