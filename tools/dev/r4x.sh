set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_r4x.log 2>&1 || { tail -30 gpurun_out/t_r4x.log; exit 1; }
tail -1 gpurun_out/t_r4x.log
bash tools/gpu_ab.sh r4x 3 base xovl > gpurun_out/r4x.log 2>&1
head -6 gpurun_out/r4x.log
grep -A8 "abprof_r4x_" gpurun_out/r4x.log | grep "abprof\|k_xdraw"
BENCH_EXTRA="--g 8 --thin 100000" bash tools/gpu_ab.sh r4x8 2 base xovl > gpurun_out/r4x8.log 2>&1
head -4 gpurun_out/r4x8.log
grep -A8 "abprof_r4x8_" gpurun_out/r4x8.log | grep "abprof\|k_xdraw"
