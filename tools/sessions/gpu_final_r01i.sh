# Round-end evidence for the current engine: GPU tests, smoke, PMC traffic (FETCH / WRITE in separate
# passes), kernel stats, and the default bench line (after the PMC summary so 'traffic' is filled).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp
cd $R && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests_r01i.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r01i.log 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/prof_fetch4 -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /dev/null 2> $O/pmc4.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/prof_write4 -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /dev/null 2>> $O/pmc4.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stats4 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > $O/bench_stats4.json 2>> $O/pmc4.err &&
cd $R && python3 tools/pmc_summary.py $O/prof_fetch4/fetch_counter_collection.csv $O/prof_write4/write_counter_collection.csv $R/profiles/pmc_traffic.json --batch 4096 --size 256 > $O/pmc4_summary.txt 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_r01i.json 2> $O/bench_r01i.err
