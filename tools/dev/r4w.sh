set -e
export TMPDIR=/tmp
PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
mkdir -p gpurun_out
cp $PKG/libdcfm.so /tmp/libdcfm_intree.so
for V in "$@"; do
  cp build/ab/libdcfm_$V.so $PKG/libdcfm.so
  timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_loopback.py > gpurun_out/t_r4w_$V.log 2>&1 || { tail -30 gpurun_out/t_r4w_$V.log; cp /tmp/libdcfm_intree.so $PKG/libdcfm.so; exit 1; }
  echo "$V: $(tail -1 gpurun_out/t_r4w_$V.log)"
done
cp /tmp/libdcfm_intree.so $PKG/libdcfm.so
bash tools/gpu_ab.sh r4w 3 base "$@" > gpurun_out/r4w.log 2>&1
head -9 gpurun_out/r4w.log
grep -A6 "abprof_r4w_" gpurun_out/r4w.log | grep "abprof\|k_assemble"
