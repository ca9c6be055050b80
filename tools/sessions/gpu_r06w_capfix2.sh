# capture crash: the engine diagnostic with persistent side-stream fork / join events and the guard lifted, the serving
# tests, then probe mode 11 (B joined to A through a temporary event destroyed after the wait); stops at a failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w; mkdir -p $O
info() {
  echo "=== capture_info $1" >> $O/log.txt
  timeout -k 10 240 python3 -u tools/capture_info.py $1 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
probe() {
  echo "=== probe PROBE_FRESH=$1 mode $2 K=$3" >> $O/log.txt
  PROBE_FRESH=$1 timeout -k 10 60 ./variants/capture_probe $2 $3 9 2 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
info "--n 330 --guard 0" && info "--n 4096 --guard 0 --chunks 8" &&
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_serving.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/serving.txt 2>&1 &&
probe 1 11 8 && probe 0 11 1 && echo done
