mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_wide.log 2>&1; rc=$?
tail -25 gpurun_out/t_wide.log; exit $rc
