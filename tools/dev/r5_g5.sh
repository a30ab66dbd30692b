# round 5 (dev): parity with the permlane row exchanges, then A/B against the previous build at c4 and c3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py tests/test_gpu_loopback.py tests/test_gpu_excursion.py tests/test_gpu_generated_draws.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r5e.log 2>&1; tail -3 gpurun_out/t_r5e.log
BENCH_EXTRA="--g 8 --P 1250 --n 2000 --K 100 --steps 100 --warmup 10" bash tools/gpu_ab.sh r5f 2 head perm > gpurun_out/ab_r5f.log 2>&1; grep -E "^(head|perm) " gpurun_out/ab_r5f.log; grep -A3 "abprof" gpurun_out/ab_r5f.log | grep -E "abprof|lambda_w"
bash tools/gpu_ab.sh r5g 2 head perm > gpurun_out/ab_r5g.log 2>&1; grep -E "^(head|perm) " gpurun_out/ab_r5g.log
