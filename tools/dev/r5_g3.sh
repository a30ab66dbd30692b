# round 5 (dev): seed scans for X excursions, then A/B of timing variants
timeout -k 10 240 python -u tools/dev/excursion_probe.py --shape c4 --seeds 8-40 --iters 1200 --step 50 > gpurun_out/probe_c4b.log 2>&1
timeout -k 10 120 python -u tools/dev/excursion_probe.py --shape c2 --seeds 1-40 --iters 1200 --step 50 > gpurun_out/probe_c2b.log 2>&1
bash tools/gpu_ab.sh r5b 2 base nolg norng ring3 zsplit > gpurun_out/ab_r5b.log 2>&1; grep -v "^ *$" gpurun_out/ab_r5b.log | tail -30
BENCH_EXTRA=--exact-residual bash tools/gpu_ab.sh r5c 2 base rw4 > gpurun_out/ab_r5c.log 2>&1; tail -12 gpurun_out/ab_r5c.log
