# Richardson-Lucy(100) at 4096 x 256^2 vs Infinity-Cache chunk size / pipeline streams
for cfg in "96 2" "48 2" "32 2" "24 2" "32 3" "16 4" "64 1"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --workload rl --steps 2 --warmup 1 --no-cpu-baseline --no-graph --no-ingest --chunk-mb $1 --pipe-streams $2 > gpurun_out/srl.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/srl.json').read().strip().splitlines()[-1]); print('chunk $1 streams $2', round(d['value']), round(d['ms_per_step'],1))"
done
