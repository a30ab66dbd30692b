set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hiptr_r4s -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > $GRAFT_REPO_ROOT/gpurun_out/hiptr_r4s.log 2>&1
cd $GRAFT_REPO_ROOT
ls -la gpurun_out/hiptr_r4s/* | head
find gpurun_out/hiptr_r4s -name "*.csv" -size +4M -exec gzip -9 {} \;
ls -la gpurun_out/hiptr_r4s/*
