# round 5 (dev): k_resid64 with 16-byte Y loads (paired column tiles) — exact-mode parity, then A/B
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "exact or 16" > gpurun_out/t_r5g.log 2>&1; tail -2 gpurun_out/t_r5g.log
BENCH_EXTRA="--exact-residual --timed-samples 0" bash tools/gpu_ab.sh r5k 2 cur p16 > gpurun_out/ab_r5k.log 2>&1; grep -E "^(cur|p16) " gpurun_out/ab_r5k.log | sed 's/.k_wpass.*k_resid/ k_resid/'; grep -A4 "abprof" gpurun_out/ab_r5k.log | grep -E "abprof|k_resid"
