# capture probe: mixed fork origins (modes 7 / 8) beside the known-good nested mode 2; stops at the first failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t; mkdir -p $O
run() {  # fresh mode K
  echo "=== PROBE_FRESH=$1 mode $2 K=$3" >> $O/probe.txt
  PROBE_FRESH=$1 timeout -k 10 60 ./variants/capture_probe $2 $3 9 2 >> $O/probe.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/probe.txt
  [ $rc -eq 0 ] || exit $rc
}
run 0 2 8 && run 1 2 8 && run 0 8 8 && run 1 8 8 && run 1 7 8 && run 0 7 8 && run 1 7 1 && echo done
