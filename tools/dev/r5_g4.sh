# round 5 (dev): parity of the paired-pivot chol_inv16, then A/B pair vs single pivots at c4 and c3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_configs.py tests/test_gpu_loopback.py tests/test_gpu_excursion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r5d.log 2>&1; tail -3 gpurun_out/t_r5d.log
BENCH_EXTRA="--g 8 --P 1250 --n 2000 --K 100 --steps 100 --warmup 10" bash tools/gpu_ab.sh r5d 2 pair chol1 > gpurun_out/ab_r5d.log 2>&1; grep -E "^(pair|chol1) " gpurun_out/ab_r5d.log; grep -A6 "abprof" gpurun_out/ab_r5d.log | grep -E "abprof|lambda_w|k_prep|k_xchol|k_wpass|k_cpass"
bash tools/gpu_ab.sh r5e 2 pair chol1 > gpurun_out/ab_r5e.log 2>&1; grep -E "^(pair|chol1) " gpurun_out/ab_r5e.log
