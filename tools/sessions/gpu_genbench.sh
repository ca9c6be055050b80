# Bench lines of the runtime-planned path next to the compile-time one (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-gb}
cd $R && timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --size 80 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench80_$T.json 2> $O/bench80_$T.err &&
timeout -k 10 300 python3 bench.py --size 96 --no-e2e --no-ingest --no-cpu-baseline --no-graph --fused 0 > $O/bench96c_$T.json 2> $O/bench96c_$T.err &&
timeout -k 10 300 python3 bench.py --size 255 --batch 1024 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench255_$T.json 2> $O/bench255_$T.err &&
timeout -k 10 300 python3 bench.py --size 256 --batch 1024 --fused 0 --fused-init 0 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench256c_$T.json 2> $O/bench256c_$T.err
