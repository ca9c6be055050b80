# Round-6 final check, part 1 (tag = $1): GPU tests + smoke, PMC traffic
# (FETCH_SIZE / WRITE_SIZE in separate passes) for the default / Poisson / RL / 48^2 workloads of the final
# engine rev, rocprofv3 kernel stats of the default bench and the 48^2 line, pmc_summary -> pmc_traffic_*.json.
# Part 2 (gpu_r05_benchfinal.sh) runs the bench lines reading that traffic.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r06final}; mkdir -p $O
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest --no-extra"
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 &&
cd /tmp && timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pf_$T -o fetch --output-format csv -- $B --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2> $O/pmc_$T.err &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pw_$T -o write --output-format csv -- $B --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pfp_$T -o fetch --output-format csv -- $B --llh Poisson --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pwp_$T -o write --output-format csv -- $B --llh Poisson --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pfrl_$T -o fetch --output-format csv -- $B --workload rl --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pwrl_$T -o write --output-format csv -- $B --workload rl --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pf48_$T -o fetch --output-format csv -- $B --size 48 --batch 256 --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pw48_$T -o write --output-format csv -- $B --size 48 --batch 256 --steps 1 --warmup 1 --blocks 1 --settle-s 0 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ps_$T -o run --output-format csv -- $B --steps 3 --warmup 1 --blocks 1 --settle-s 0 > $O/bench_stats_$T.json 2>> $O/pmc_$T.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ps48_$T -o run --output-format csv -- $B --size 48 --batch 256 --steps 20 --warmup 2 --blocks 1 --settle-s 0 > $O/bench48_stats_$T.json 2>> $O/pmc_$T.err &&
cd $R && python3 tools/pmc_summary.py $O/pf_$T/fetch_counter_collection.csv $O/pw_$T/write_counter_collection.csv $O/pmc_traffic_$T.json --batch 4096 --size 256 --n-iters 8 > $O/pmc_summary_$T.txt 2>&1 &&
python3 tools/pmc_summary.py $O/pfp_$T/fetch_counter_collection.csv $O/pwp_$T/write_counter_collection.csv $O/pmc_traffic_poisson_$T.json --batch 4096 --size 256 --n-iters 8 > $O/pmc_summary_poisson_$T.txt 2>&1 &&
python3 tools/pmc_summary.py $O/pfrl_$T/fetch_counter_collection.csv $O/pwrl_$T/write_counter_collection.csv $O/pmc_traffic_rl_$T.json --batch 4096 --size 256 --rl-calls 1 --n-iters 100 > $O/pmc_summary_rl_$T.txt 2>&1 &&
python3 tools/pmc_summary.py $O/pf48_$T/fetch_counter_collection.csv $O/pw48_$T/write_counter_collection.csv $O/pmc_traffic48_$T.json --batch 256 --size 48 --n-iters 8 > $O/pmc_summary48_$T.txt 2>&1
