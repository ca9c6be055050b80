# Round-3 session q (tag = $1): non-square UnrolledADMMGaussian + any-shape engine SubNet tests first, then
# the whole GPU suite and the default bench line
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03q}; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_parity.py -m gpu -x -q -rf -k "rect or any_psf" --timeout 120 --timeout-method thread > $O/gpu_new_$T.log 2>&1 &&
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err
