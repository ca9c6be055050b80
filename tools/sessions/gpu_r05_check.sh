# GPU tests + smoke + the default bench line (as the driver runs it), tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r05c}; mkdir -p $O
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 &&
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$T.json 2> $O/bench_$T.err
