# Kernel trace of eager vs graph-replayed steps (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-gp}
cd $R && timeout -k 10 200 python3 tools/graph_vs_eager.py 3 > $O/gve_$T.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/gve_prof_$T -o run -- python3 $R/tools/graph_vs_eager.py 3 >> $O/gve_$T.txt 2>&1
