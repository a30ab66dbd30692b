set -e
export TMPDIR=/tmp
PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
mkdir -p gpurun_out
cp $PKG/libdcfm.so /tmp/libdcfm_intree.so
cp build/ab/libdcfm_$1.so $PKG/libdcfm.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_loopback.py > gpurun_out/t_r4j.log 2>&1 || { tail -30 gpurun_out/t_r4j.log; cp /tmp/libdcfm_intree.so $PKG/libdcfm.so; exit 1; }
tail -2 gpurun_out/t_r4j.log
cp /tmp/libdcfm_intree.so $PKG/libdcfm.so
bash tools/gpu_ab.sh r4j 3 base $1
