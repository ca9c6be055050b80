# Kernel stats and PMC traffic of the mid-size lines (tag $1): rocprofv3 --kernel-trace --stats of the 160^2 and 80^2
# benches, FETCH_SIZE / WRITE_SIZE passes (separate runs) at 160^2 and 80^2, summarised by tools/pmc_summary.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r04midprof}; mkdir -p $O
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest"
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ps160_$T -o run --output-format csv -- $B --size 160 --steps 3 --warmup 1 > $O/bench160_stats_$T.json 2> $O/prof_$T.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ps80_$T -o run --output-format csv -- $B --size 80 --steps 3 --warmup 1 > $O/bench80_stats_$T.json 2>> $O/prof_$T.err &&
for L in 160 80; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pf${L}_$T -o fetch --output-format csv -- $B --size $L --steps 1 --warmup 1 > /dev/null 2>> $O/prof_$T.err || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pw${L}_$T -o write --output-format csv -- $B --size $L --steps 1 --warmup 1 > /dev/null 2>> $O/prof_$T.err || exit 1
  (cd $R && python3 tools/pmc_summary.py $O/pf${L}_$T/fetch_counter_collection.csv $O/pw${L}_$T/write_counter_collection.csv $O/pmc_traffic${L}_$T.json --batch 4096 --size $L --n-iters 8 > $O/pmc_summary${L}_$T.txt 2>&1) || exit 1
done
