set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_r4p.log 2>&1 || { tail -30 gpurun_out/t_r4p.log; exit 1; }
tail -2 gpurun_out/t_r4p.log
bash tools/gpu_ab.sh r4p 3 base sfrag > gpurun_out/r4p.log 2>&1
head -6 gpurun_out/r4p.log
grep -A6 "abprof_r4p_" gpurun_out/r4p.log | grep "abprof\|k_assemble"
