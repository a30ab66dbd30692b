# round 5 (dev): W pass with split-K accumulators (8 chains per wave) — A/B at c3, then c4
bash tools/gpu_ab.sh r5h 3 base split splitr3 splitw2 > gpurun_out/ab_r5h.log 2>&1; grep -E "^(base|split|splitr3|splitw2) " gpurun_out/ab_r5h.log; grep -A3 "abprof" gpurun_out/ab_r5h.log | grep -E "abprof|k_wcol"
BENCH_EXTRA="--g 8 --P 1250 --n 2000 --K 100 --steps 100 --warmup 10" bash tools/gpu_ab.sh r5i 1 base splitr3 > gpurun_out/ab_r5i.log 2>&1; grep -E "^(base|splitr3) " gpurun_out/ab_r5i.log
