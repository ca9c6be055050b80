# 48^2 iteration microbenchmark + phase trace; concurrency test; bench lines 48^2 / 256^2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03k}
cd $R && mkdir -p $O &&
timeout -k 10 60 tools/kbench_small 256 48 400 > $O/ksmall_$T.txt 2>&1 &&
timeout -k 10 60 tools/kbench_smalltr 256 48 100 >> $O/ksmall_$T.txt 2>&1 &&
timeout -k 10 60 tools/kbench_small 4096 48 50 >> $O/ksmall_$T.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "concurrent or configs1 or admm48 or zero_iters or fused_init" > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline --steps 20 > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err
