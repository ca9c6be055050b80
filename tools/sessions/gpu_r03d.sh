# Round-3 session d: symmetric odd-prime stage - pixel parity vs fp64, generic GPU tests, 255^2 / 97x80 rates
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-d}; mkdir -p $O
cd $R && rm -f $O/parity_$T.jsonl
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pixel_parity.py tests/test_gpu_generic.py -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pixpar_$T.log 2>&1
echo "pixel parity exit $?" >> $O/pixpar_$T.log
timeout -k 10 300 python3 bench.py --size 255 --batch 1024 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench255_$T.json 2> $O/bench255_$T.err &&
timeout -k 10 300 python3 bench.py --size 160 --batch 4096 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench160_$T.json 2> $O/bench160_$T.err &&
timeout -k 10 300 python3 bench.py --size 192 --batch 4096 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench192_$T.json 2> $O/bench192_$T.err
