# k_cpass + k_lambda as one launch (-DDCFM_FUSE_CL=1, build/ab/libdcfm_cl.so): parity, then A/B
set -e
export TMPDIR=/tmp
PKG=a-divide-and-conquer-strategy-for-high-dimensional-bayesian-factor-models_amd
mkdir -p gpurun_out
cp $PKG/libdcfm.so /tmp/libdcfm_intree.so
cp build/ab/libdcfm_cl.so $PKG/libdcfm.so
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_generated_draws.py tests/test_gpu_loopback.py tests/test_gpu_parity_configs.py > gpurun_out/t_r4cl.log 2>&1 || { tail -30 gpurun_out/t_r4cl.log; cp /tmp/libdcfm_intree.so $PKG/libdcfm.so; exit 1; }
tail -1 gpurun_out/t_r4cl.log
cp /tmp/libdcfm_intree.so $PKG/libdcfm.so
bash tools/gpu_ab.sh r4cl 3 base cl > gpurun_out/r4cl.log 2>&1
head -6 gpurun_out/r4cl.log
BENCH_EXTRA="--g 8 --thin 100000" bash tools/gpu_ab.sh r4cl8 2 base cl > gpurun_out/r4cl8.log 2>&1
head -4 gpurun_out/r4cl8.log
