# round 5: the gpu_ab A/B of k_wcol timing variants (dev)
bash tools/gpu_ab.sh r5a 2 base nolg nozn norng ring3 zsplit > gpurun_out/ab_r5a.log 2>&1; tail -20 gpurun_out/ab_r5a.log
