# HBM traffic per launch for every engine kernel of the default bench (fused iteration + fused init):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (MI355X_MICROARCH.md HBM section).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/prof_fetch3 -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /dev/null 2> $O/pmc3.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/prof_write3 -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /dev/null 2>> $O/pmc3.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_stats3 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > $O/bench_stats3.json 2>> $O/pmc3.err
