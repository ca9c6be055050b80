# Round check on the committed tree (tag = $1): GPU tests, smoke, bench lines (256^2 default, RL(100), Poisson, 48^2).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-rc}
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-e2e --no-ingest > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 500 python3 bench.py --workload rl --no-e2e --no-ingest > $O/bench_rl_$T.json 2> $O/bench_rl_$T.err &&
timeout -k 10 400 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-graph --no-cpu-baseline > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
