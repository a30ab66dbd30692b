# round 5 (dev): k_cpass with split accumulators (8 chains per wave), k_lambda pipeline depth
bash tools/gpu_ab.sh r5m 2 base cps cps2 pipe2 pipe6 > gpurun_out/ab_r5m.log 2>&1; grep -E "^(base|cps|cps2|pipe2|pipe6) " gpurun_out/ab_r5m.log; grep -A6 "abprof" gpurun_out/ab_r5m.log | grep -E "abprof|k_cpass|k_lambda"
