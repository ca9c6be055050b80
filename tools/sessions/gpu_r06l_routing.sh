# default routing at 256^2 after the per-op batch thresholds (Gaussian 96, Poisson 192, RL 96): small batches
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd $R
B="python3 bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest --no-extra"
line() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', round(d['value']), d['blocks']['eager_ms_per_step'], {k: round(x['avg_ms'], 4) for k, x in d['kernels'].items()}, d['config']['iteration'])"; }
for N in 1 16 64 128 192 256; do
  timeout -k 10 120 $B --llh Poisson --batch $N --steps 30 --warmup 5 > $O/r06l_p$N.json 2>/dev/null || { echo "fail P $N"; exit 1; }
  line $O/r06l_p$N.json "Poisson N=$N default"
done
for N in 1 64 96 128; do
  timeout -k 10 120 $B --workload rl --n-iters 100 --batch $N --steps 5 --warmup 1 > $O/r06l_rl$N.json 2>/dev/null || { echo "fail RL $N"; exit 1; }
  line $O/r06l_rl$N.json "RL(100) N=$N default"
done
