# Quick GPU loop: pytest -m gpu subset (-k expression $1, default all), then the default bench.
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/gpu_check.log 2>&1 || { tail -30 gpurun_out/gpu_check.log; exit 1; }
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_check.log 2>&1 || { tail -30 gpurun_out/gpu_check.log; exit 1; }
fi
tail -3 gpurun_out/gpu_check.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > gpurun_out/bench_check.json 2>gpurun_out/bench_check.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_check.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernels'])"
