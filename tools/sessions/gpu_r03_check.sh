# Round-3 check (tag = $1): GPU tests, smoke, default bench, 48^2 bench, 2-rank self-spawned bench rehearsal.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-rc}; mkdir -p $O
cd $R && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-ingest > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest > $O/bench48_$T.json 2> $O/bench48_$T.err
