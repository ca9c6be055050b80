# torch-side bisection of the capture crash (tools/capture_torch_probe.py); stops at a failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y; mkdir -p $O
tp() {
  echo "=== torch probe $1" >> $O/log.txt
  timeout -k 10 180 python3 -u tools/capture_torch_probe.py $1 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
tp ${1:-main} && tp ${2:-hipcap} && echo done
