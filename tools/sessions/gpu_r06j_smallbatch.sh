# small-batch routing check at 256^2: the one-workgroup-per-galaxy kernels (fused) against the chained row /
# column kernels (fused 0) for batches below one round of workgroups
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd $R
for N in 1 8 32 64 128 256; do
  for f in 1 0; do
    timeout -k 10 120 python3 bench.py --batch $N --steps 40 --warmup 5 --fused $f --fused-init $f --no-cpu-baseline --no-e2e --no-graph --no-ingest --no-extra > $O/r06j_b${N}_f$f.json 2> $O/r06j_b${N}_f$f.err || { echo "fail $N $f"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/r06j_b${N}_f$f.json').read().strip().splitlines()[-1])
print('N=$N fused=$f', round(d['value']), d['blocks']['eager_ms_per_step'], {k: round(x['avg_ms'], 4) for k, x in d['kernels'].items()})"
  done
done
