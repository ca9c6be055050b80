# op_admm_init vs Infinity-Cache chunk size and pipeline streams (fused iteration unaffected)
for cfg in "96 2" "48 2" "48 4" "192 2" "64 3" "32 4" "0 1"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest --chunk-mb $1 --pipe-streams $2 > gpurun_out/si.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/si.json').read().strip().splitlines()[-1]); k=d['kernels']; print('chunk $1 streams $2', round(d['value']), {n: round(v['avg_ms'],3) for n,v in k.items()})"
done
