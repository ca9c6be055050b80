# Time the Gaussian init variants (gd_set_fused_init 0 / 1 / 2) on the default 256^2 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in $1; do
  timeout -k 10 150 python3 $R/bench.py --steps 5 --warmup 2 --fused-init $v --no-cpu-baseline --no-e2e --no-graph --no-ingest > /tmp/iv.json 2>/dev/null || { echo "fail $v"; break; }
  python3 -c "import json; d=json.loads(open('/tmp/iv.json').read().strip().splitlines()[-1]); print('init $v |', round(d['value']), {k: round(x['avg_ms'],3) for k,x in d['kernels'].items()})"
done
