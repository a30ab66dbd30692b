# same box, interleaved: the roofline kernel timed on every launch of the region vs on 5
set -e
mkdir -p gpurun_out
for r in 1 2 3 4; do
  for S in 0 5; do
    timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --timed-samples $S > gpurun_out/b_r4z_${S}_$r.json 2> gpurun_out/b_r4z.err
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['avg_us'], r['launches'])" gpurun_out/b_r4z_${S}_$r.json $S
  done
done
