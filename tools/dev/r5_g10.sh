# round 5 (dev): Z normals drawn one iteration ahead in k_lambda's tail — bitwise / parity checks, then A/B
timeout -k 10 600 python -u -m pytest tests/test_gpu_generated_draws.py tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_gpu_chains.py tests/test_gpu_init.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r5j.log 2>&1; tail -2 gpurun_out/t_r5j.log
bash tools/gpu_ab.sh r5l 3 head zpre > gpurun_out/ab_r5l.log 2>&1; grep -E "^(head|zpre) " gpurun_out/ab_r5l.log; grep -A5 "abprof" gpurun_out/ab_r5l.log | grep -E "abprof|k_wcol|k_lambda"
