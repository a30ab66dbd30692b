bash tools/profile_round.sh a1 > gpurun_out/prof_a1_run.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/prof_a1_run.log; exit 1; }
tail -2 gpurun_out/prof_a1_run.log
bash tools/lambench/run2.sh > gpurun_out/lam6.log 2>&1; cat gpurun_out/lam6.log
