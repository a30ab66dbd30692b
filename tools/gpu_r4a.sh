#!/bin/bash
# round 4: changed GPU tests, then the driver's bench with and without the exact residual
TAG=${1:-r4a}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py tests/test_gpu_rccl.py tests/test_gpu_alt_paths.py tests/test_gpu_loopback.py -x -v --timeout 240 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -3 gpurun_out/t_$TAG.log
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > gpurun_out/bench_drv_$TAG.json 2> gpurun_out/bench_drv_$TAG.err || { echo "driver bench failed"; tail gpurun_out/bench_drv_$TAG.err; exit 1; }
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --exact-residual > gpurun_out/bench_ex_$TAG.json 2> gpurun_out/bench_ex_$TAG.err || { echo "exact bench failed"; tail gpurun_out/bench_ex_$TAG.err; exit 1; }
python3 tools/show_bench.py gpurun_out/bench_drv_$TAG.json gpurun_out/bench_ex_$TAG.json
