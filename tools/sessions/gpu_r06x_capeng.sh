# serving tests (persistent side-stream events), then the engine capture probe without torch; stops at a failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
eng() {
  echo "=== engine probe side $1" >> $O/log.txt
  timeout -k 10 120 ./variants/capture_engine_probe $1 330 160 6 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_serving.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/serving.txt 2>&1 &&
eng 0 && eng 3 && eng 1 && eng 2 && echo done
