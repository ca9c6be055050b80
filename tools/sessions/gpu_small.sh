# 48^2 small-kernel change check (tag = $1): small-size GPU tests, 48^2 bench, 4096 x 48^2 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-sm}
cd $R && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "48 or 32 or 64 or small or configs" > $O/small_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 4096 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench48b_$T.json 2> $O/bench48b_$T.err
