set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_ab.sh r4v 1 base noldag nozmma lgnt > gpurun_out/r4v.log 2>&1
head -4 gpurun_out/r4v.log
python3 tools/dev/gaps.py gpurun_out/abprof_r4v_base gpurun_out/abprof_r4v_noldag gpurun_out/abprof_r4v_nozmma gpurun_out/abprof_r4v_lgnt | grep -v "trace_part\|fillBuffer\|sigma_err"
grep -A5 "abprof_r4v_" gpurun_out/r4v.log | grep "abprof\|k_wcol"
