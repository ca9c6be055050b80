# Check of the tree with the reworked SubNet convs (tag = $1): GPU tests, smoke, bench lines (256^2 default, 48^2), kernel stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-rc}
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest > $O/bench48_$T.json 2> $O/bench48_$T.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ps_$T -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest --steps 3 --warmup 1 > $O/bench_stats_$T.json 2> $O/stats_$T.err
