# small batches at 256^2 for Poisson (two-pass vs three-kernel chain) and Richardson-Lucy (k_rl_reg vs the chunked
# chain), and the Gaussian threshold's neighbourhood with the routing build
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd $R
B="python3 bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest --no-extra"
line() { python3 -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', round(d['value']), d['blocks']['eager_ms_per_step'], {k: round(x['avg_ms'], 4) for k, x in d['kernels'].items()}, d['config']['iteration'])"; }
for N in 1 16 64 128 256; do
  for f in 1 0; do
    timeout -k 10 120 $B --llh Poisson --batch $N --steps 30 --warmup 5 --fused $f --fused-init $f > $O/r06k_p${N}_f$f.json 2>/dev/null || { echo "fail P $N $f"; exit 1; }
    line $O/r06k_p${N}_f$f.json "Poisson N=$N fused=$f"
  done
done
for N in 1 16 64 128 256; do
  for f in 1 0; do
    timeout -k 10 120 $B --workload rl --n-iters 100 --batch $N --steps 5 --warmup 1 --fused-rl $f > $O/r06k_rl${N}_f$f.json 2>/dev/null || { echo "fail RL $N $f"; exit 1; }
    line $O/r06k_rl${N}_f$f.json "RL(100) N=$N fused_rl=$f"
  done
done
for N in 64 80 96 112 128; do
  timeout -k 10 120 $B --batch $N --steps 40 --warmup 5 > $O/r06k_g${N}.json 2>/dev/null || { echo "fail G $N"; exit 1; }
  line $O/r06k_g${N}.json "Gaussian N=$N default routing"
done
