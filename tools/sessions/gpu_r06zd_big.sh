# sizes up to 4096 per side: the runtime-planned path's GPU tests (incl. the new > 1638 cases), the loud-error test
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zd; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_generic.py "tests/test_gpu_parity.py::test_errors_are_loud" -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; exit $rc
