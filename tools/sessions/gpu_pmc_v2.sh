R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gal" -d $O/prof_fetch2 -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest --fused 2 > /dev/null 2> $O/pmc2.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_gal" -d $O/prof_write2 -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest --fused 2 > /dev/null 2>> $O/pmc2.err
