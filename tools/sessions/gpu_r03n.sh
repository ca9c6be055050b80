# SubNet pointers back as restrict kernel args; z prefetch in k_gal_small: microbenchmarks, GPU tests, bench lines, 48^2 trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03n}
cd $R && mkdir -p $O &&
timeout -k 10 60 tools/kbench_small 256 48 400 > $O/ksmall_$T.txt 2>&1 &&
timeout -k 10 60 tools/kbench_smalltr 256 48 100 >> $O/ksmall_$T.txt 2>&1 &&
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline --steps 20 > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof48_$T -o run -- python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline --steps 20 > $O/bench48tr_$T.json 2> $O/bench48tr_$T.err
