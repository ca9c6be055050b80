# Round-3 session i (tag = $1): Poisson two-pass with H read once (pass A: conj(H) W and H X; pass B: H X in,
# F(w') out) - GPU tests, Poisson bench, Poisson PMC traffic
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-i}; mkdir -p $O
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest"
cd $R && timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 400 $B --llh Poisson > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 400 $B --llh Poisson > $O/bench_poisson2_$T.json 2> $O/bench_poisson2_$T.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pfp_$T -o fetch --output-format csv -- $B --llh Poisson --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pwp_$T -o write --output-format csv -- $B --llh Poisson --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
cd $R && python3 tools/pmc_summary.py $O/pfp_$T/fetch_counter_collection.csv $O/pwp_$T/write_counter_collection.csv $O/pmc_traffic_poisson_$T.json --batch 4096 --size 256 --n-iters 8 > $O/pmc_summary_poisson_$T.txt 2>&1
