# Round-3 session h (tag = $1): spill-free Poisson pass A / B and RL, opaque addresses - GPU tests, bench
# lines (Gaussian, Poisson, RL, 48^2), PMC traffic (FETCH / WRITE in separate passes) for every workload,
# rocprofv3 kernel stats of the default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-h}; mkdir -p $O
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest"
cd $R && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-ingest > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 400 $B --llh Poisson > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 500 python3 bench.py --workload rl --no-e2e --no-ingest --no-graph > $O/bench_rl_$T.json 2> $O/bench_rl_$T.err
