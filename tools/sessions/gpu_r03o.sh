# Round-3 session o (tag = $1): state check of the restored tree - GPU tests, default bench, Poisson/RL lines,
# rocprofv3 kernel stats of the default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03o}; mkdir -p $O
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline --no-graph --llh Poisson > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 300 python3 bench.py --workload rl --no-e2e --no-ingest --no-graph --no-cpu-baseline > $O/bench_rl_$T.json 2> $O/bench_rl_$T.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 $R/bench.py --no-e2e --no-ingest --no-cpu-baseline --no-graph --steps 3 > $O/benchtr_$T.json 2> $O/benchtr_$T.err
