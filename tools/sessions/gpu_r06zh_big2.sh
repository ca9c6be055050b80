# the > 1638 sizes again with the two-galaxy chunked batch and the Poisson chain at 2053 x 2500
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zh; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_generic.py -m gpu -x -v --timeout 300 --timeout-method thread -s -k "big" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; exit $rc
