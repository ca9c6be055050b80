# Round-6 final check, part 2 (tag = $1): the default bench line as the driver runs it (with its configs[1] /
# configs[4] sub-lines) and the Poisson line, reading profiles/pmc_traffic*.json from part 1.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r06final}; mkdir -p $O
cd $R && timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-graph --no-extra > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err
