# 160^2 bench diagnosis (tag $1): the r04z session's `bench.py --size 160` died with SIGSEGV and no output.
# Small batch without the graph, full batch without the graph, then small batch with the graph; Python's
# faulthandler prints the stack of a native crash.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04dbg}; mkdir -p $O
B="python3 -X faulthandler $R/bench.py --size 160 --steps 2 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline"
cd $R && timeout -k 10 200 $B --batch 64 --no-graph > $O/b160a_$T.json 2> $O/b160a_$T.err &&
timeout -k 10 200 $B --batch 4096 --no-graph > $O/b160b_$T.json 2> $O/b160b_$T.err &&
timeout -k 10 200 $B --batch 64 > $O/b160c_$T.json 2> $O/b160c_$T.err
