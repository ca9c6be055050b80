# Round-4 check (tag = $1): GPU tests, smoke (engine rev + source hash), default bench (clean value + a separate
# profiling pass), 48^2 bench, and the self-spawned 2-rank gloo rehearsal line (rank spread, gather GB/s,
# cpu_baseline on rank 0).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r04a}; mkdir -p $O
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rfs --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-ingest > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --steps 200 --warmup 20 --no-e2e --no-ingest > $O/bench48_$T.json 2> $O/bench48_$T.err &&
GD_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-e2e --no-ingest --no-graph --cpu-seconds 3 --cpu-sample 8 > $O/bench_g2gloo_$T.json 2> $O/bench_g2gloo_$T.err
