# Quick GPU check: Gaussian/ADMM parity subset, bench with the fused and the three-kernel iteration, rocprof trace.
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x -k "admm or fused or full_batch or pipelined" > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --fused 1 > gpurun_out/bench_f1.json 2>gpurun_out/bench_f1.err && \
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --fused 0 > gpurun_out/bench_f0.json 2>gpurun_out/bench_f0.err && \
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_f1 -o f1 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --fused 1 > /dev/null 2>&1
fi
