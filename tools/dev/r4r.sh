set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh r4r 2 base wtw wtl wtb > gpurun_out/r4r.log 2>&1
head -8 gpurun_out/r4r.log
python3 tools/dev/gaps.py gpurun_out/abprof_r4r_base gpurun_out/abprof_r4r_wtw gpurun_out/abprof_r4r_wtl gpurun_out/abprof_r4r_wtb | grep -v "trace_part\|fillBuffer\|sigma_err"
