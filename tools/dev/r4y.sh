set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_r4y.log 2>&1 || { tail -30 gpurun_out/t_r4y.log; exit 1; }
tail -1 gpurun_out/t_r4y.log
for r in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > gpurun_out/b_r4y_$r.json 2> gpurun_out/b_r4y_$r.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['avg_us'], r['launches'], r['launches_in_region'], r['frac'])" gpurun_out/b_r4y_$r.json
done
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_r4y -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 > $GRAFT_REPO_ROOT/gpurun_out/tr_r4y.log 2>&1
cd $GRAFT_REPO_ROOT && python3 tools/dev/gaps.py gpurun_out/tr_r4y
