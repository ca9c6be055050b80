# init || SubNet overlap check (tag = $1): Gaussian GPU tests, graph tests, 48^2 and 256^2 bench lines
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-ov}
cd $R && timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "Gaussian or gaussian or 48 or 32 or 64 or graph or full_model or fused or configs or smoke or init" > $O/ov_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err
