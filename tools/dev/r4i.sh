set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --exact-residual > gpurun_out/b_r4i_exact.json 2> gpurun_out/b_r4i_exact.err
python3 -c "import json; d=json.loads(open('gpurun_out/b_r4i_exact.json').read().strip().splitlines()[-1]); print('exact', d['value'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
bash tools/gpu_ab.sh r4i 3 base cps wc2
