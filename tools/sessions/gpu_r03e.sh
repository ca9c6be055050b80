# Round-3 session e: SubNet one-round kernel at 1024 threads, 16-part MLP - kbench timing + phase trace,
# SubNet / full GPU tests, 48^2 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-e}; mkdir -p $O
cd $R && timeout -k 10 60 tools/kbench_subnet 4096 256 20 > $O/ksn_$T.txt 2>&1 &&
timeout -k 10 60 tools/kbench_subnet_trace 4096 256 5 >> $O/ksn_$T.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 300 python3 -u tools/host_profile.py > $O/hostprof_$T.txt 2>&1
