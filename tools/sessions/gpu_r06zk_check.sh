# final-tree check (tag $1): every GPU test and the smoke, as the driver runs them at round end
cd $GRAFT_REPO_ROOT
O=gpurun_out; T=${1:-r06h}
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1
rc=$?; tail -2 $O/gpu_tests_$T.log; tail -1 $O/smoke_$T.txt; exit $rc
