timeout -k 10 200 python3 -u tools/dev/c2_first.py gen 12 > gpurun_out/c2first_gen.log 2>&1; cat gpurun_out/c2first_gen.log | cut -c1-400
timeout -k 10 200 python3 -u tools/dev/c2_first.py inject 12 > gpurun_out/c2first_inj.log 2>&1; cat gpurun_out/c2first_inj.log | cut -c1-400
