# rocprofv3 kernel trace of the g = 8 share (the per-rank work of c3 on 8 GPUs) on one GPU
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g8tr -o run -- python3 $GRAFT_REPO_ROOT/bench.py --g 8 --thin 100000 --steps 2000 --warmup 100 --no-cpu-baseline --no-profile --converged-mcmc 0 > $GRAFT_REPO_ROOT/gpurun_out/g8tr.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/kavg.py gpurun_out/g8tr
python3 tools/dev/gaps.py gpurun_out/g8tr
find gpurun_out/g8tr -name "*trace.csv" -size +2M -exec gzip -9 {} \;
