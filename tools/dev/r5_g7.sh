# round 5 (dev): does timing every k_wcol launch with events cost wall-clock time?  Interleaved
# driver-command benches, events on all 20 launches (default) vs on 2 of them
for r in 1 2 3 4; do
  for ts in 0 2; do
    timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --converged-mcmc 0 --timed-samples $ts > gpurun_out/ts_${ts}_$r.json 2> gpurun_out/ts_${ts}_$r.err || { echo "bench failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ts', sys.argv[2], d['value'], d['roofline']['achieved'])" gpurun_out/ts_${ts}_$r.json $ts
  done
done
for r in 1 2; do
  for ts in 0 2; do
    timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 200 --warmup 20 --no-cpu-baseline --converged-mcmc 0 --timed-samples $ts > gpurun_out/ts200_${ts}_$r.json 2> gpurun_out/ts200_${ts}_$r.err || { echo "bench failed"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('ts200', sys.argv[2], d['value'], d['roofline']['achieved'])" gpurun_out/ts200_${ts}_$r.json $ts
  done
done
