# the 256^2 GPU tests + a short default bench (no e2e)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r05t}; mkdir -p $O
cd $R && timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-extra > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-extra --llh Poisson --no-ingest > $O/benchp_$T.json 2> $O/benchp_$T.err
