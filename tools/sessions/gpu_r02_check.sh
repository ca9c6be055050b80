# Round-2 check pass: GPU tests, smoke, default bench line (tag = $1).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; TAG=${1:-r02a}
cd $R && GD_PARITY_LOG=$O/parity_$TAG.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-e2e --no-ingest > $O/bench_$TAG.json 2> $O/bench_$TAG.err
