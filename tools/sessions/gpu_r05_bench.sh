# the default bench line (as the driver runs it), tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r05c}; mkdir -p $O
cd $R && timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$T.json 2> $O/bench_$T.err
