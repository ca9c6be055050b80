# capture crash: the plain-HIP probes against torch's bundled HIP runtime (ROCm 7.0): a directory whose
# libamdhip64.so.7 is torch/lib/libamdhip64.so, first on LD_LIBRARY_PATH; stops at the first failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zc; mkdir -p $O
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/rt70 && ln -sf $TL/libamdhip64.so /tmp/rt70/libamdhip64.so.7
run() {
  echo "=== runtime 7.0: $1" >> $O/log.txt
  LD_LIBRARY_PATH=/tmp/rt70:$TL timeout -k 10 120 $1 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
run "./variants/capture_engine_probe 0 330 160 6" && run "./variants/capture_probe 0 8 9 2" &&
run "./variants/capture_probe 2 8 9 2" && run "./variants/capture_engine_probe 1 330 160 6" && echo done
