# eager vs replayed 4096 x 256^2 forward under a kernel trace (tools/graph_vs_eager.py 5): per-kernel durations by phase
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r06zf; mkdir -p $O; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/graph_vs_eager.py 5 4096 > $O/gve.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/gve.txt; exit $rc
