set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity_configs.py tests/test_gpu_parity.py > gpurun_out/t_r4k.log 2>&1 || { tail -30 gpurun_out/t_r4k.log; exit 1; }
tail -2 gpurun_out/t_r4k.log
for r in 1 2; do
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --exact-residual > gpurun_out/b_r4k_exact$r.json 2> gpurun_out/b_r4k_exact.err
python3 -c "import json; d=json.loads(open('gpurun_out/b_r4k_exact$r.json').read().strip().splitlines()[-1]); print('exact', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
done
