set -o pipefail
timeout -k 10 200 python -u tools/dev/nan_hunt.py --shape c2 --seed 11 > gpurun_out/nan_c2.log 2>&1
timeout -k 10 120 python -u tools/dev/nan_hunt.py --shape c2 --seed 11 --flags 16 >> gpurun_out/nan_c2.log 2>&1
timeout -k 10 200 python -u tools/dev/nan_hunt.py --shape c4 --seed 7 > gpurun_out/nan_c4.log 2>&1
timeout -k 10 200 python -u tools/dev/nan_hunt.py --shape c4 --seed 7 --flags 16 >> gpurun_out/nan_c4.log 2>&1
cat gpurun_out/nan_c2.log gpurun_out/nan_c4.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "exact or 16" > gpurun_out/t_r5b.log 2>&1 && tail -2 gpurun_out/t_r5b.log && \
timeout -k 10 200 python -u bench.py --exact-residual --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > gpurun_out/b_exact.json 2> gpurun_out/b_exact.err && python tools/show_bench.py gpurun_out/b_exact.json && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > gpurun_out/b_def.json 2> gpurun_out/b_def.err && python tools/show_bench.py gpurun_out/b_def.json
