PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
timeout -k 10 300 python3 -u tools/dev/diag_runs.py > gpurun_out/diag_runs_new.log 2>&1; tail -30 gpurun_out/diag_runs_new.log
cp build/ab/libdcfm_base.so $PKG/libdcfm.so
echo BASE
timeout -k 10 300 python3 -u tools/dev/diag_runs.py > gpurun_out/diag_runs_base.log 2>&1; tail -30 gpurun_out/diag_runs_base.log
