#!/bin/bash
# quick GPU check: parity + loopback tests, then the driver's c3 bench, a long c3 bench and a
# c4-shape bench (no CPU legs).  Usage: bash tools/gpu_quick.sh TAG [pytest files...]
TAG=${1:-q}; shift
TESTS=${@:-tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_golden.py}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_drv_$TAG.json 2> gpurun_out/bench_drv_$TAG.err || { echo "c3 driver bench failed"; tail gpurun_out/bench_drv_$TAG.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --steps 480 --warmup 20 --no-cpu-baseline > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || { echo "c3 bench failed"; tail gpurun_out/bench_c3_$TAG.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --g 8 --P 1250 --n 2000 --K 100 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || { echo "c4 bench failed"; tail gpurun_out/bench_c4_$TAG.err; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_drv_$TAG.json gpurun_out/bench_c3_$TAG.json gpurun_out/bench_c4_$TAG.json
