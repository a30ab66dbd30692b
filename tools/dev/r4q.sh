set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_r4q.log 2>&1 || { tail -30 gpurun_out/t_r4q.log; exit 1; }
tail -2 gpurun_out/t_r4q.log
bash tools/gpu_ab.sh r4q 3 sfrag extl > gpurun_out/r4q.log 2>&1
head -6 gpurun_out/r4q.log
python3 tools/dev/gaps.py gpurun_out/abprof_r4q_sfrag gpurun_out/abprof_r4q_extl
