# 160^2 bench diagnosis, part 2 (tag $1): the crash needs the full batch AND the graph (r04dbg: 64 + graph,
# 4096 without graph both fine).  Full batch with the graph under Python's faulthandler.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04dbg2}; mkdir -p $O
B="python3 -X faulthandler $R/bench.py --size 160 --steps 2 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline"
cd $R && timeout -k 10 200 $B --batch 4096 > $O/b160d_$T.json 2> $O/b160d_$T.err
