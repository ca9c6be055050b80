# capture crash: the plain-HIP probes run against torch's bundled HIP runtime (ROCm 7.0, torch/lib) instead of
# /opt/rocm-7.2.0's; stops at the first failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06za; mkdir -p $O
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
echo "torch lib: $TL" >> $O/log.txt
run() {
  echo "=== runtime $1: $2" >> $O/log.txt
  if [ "$1" = "7.0" ]; then LD_LIBRARY_PATH=$TL timeout -k 10 120 $2 >> $O/log.txt 2>&1; else timeout -k 10 120 $2 >> $O/log.txt 2>&1; fi
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
run 7.0 "./variants/capture_engine_probe 0 330 160 6" && run 7.0 "./variants/capture_engine_probe 3 330 160 6" &&
run 7.0 "./variants/capture_probe 0 8 9 2" && run 7.0 "./variants/capture_probe 2 8 9 2" &&
run 7.0 "./variants/capture_engine_probe 1 330 160 6" && echo done
