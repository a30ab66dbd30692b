PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
timeout -k 10 300 python3 -u tools/dev/diag_chain.py 200 > gpurun_out/diag_chain_new.log 2>&1; cat gpurun_out/diag_chain_new.log | tail -4
cp build/ab/libdcfm_base.so $PKG/libdcfm.so
timeout -k 10 300 python3 -u tools/dev/diag_chain.py 200 > gpurun_out/diag_chain_base.log 2>&1; cat gpurun_out/diag_chain_base.log | tail -4
