# W~1 deferred at every size + Gaussian init concurrent with the SubNet: GPU tests, 48^2 and 256^2 bench
# lines, 48^2 kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03j}
cd $R && mkdir -p $O &&
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline --steps 20 > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof48_$T -o run -- python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline --steps 20 > $O/bench48tr_$T.json 2> $O/bench48tr_$T.err
