R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05cap7}
cd $R && timeout -k 10 200 python3 tools/capture_repro.py 4096 160 0 > $O/capture_$T.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_serving.py tests/test_abi.py -m gpu -x -q -rf --timeout 120 --timeout-method thread >> $O/capture_$T.txt 2>&1
echo "rc=$?" >> $O/capture_$T.txt
