# engine capture diagnostic (tools/capture_info.py): shipped guard, then the guard lifted at 330 and 4096 x 160^2
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u; mkdir -p $O
step() {  # name, args
  echo "=== $1: $2" >> $O/capinfo.txt
  timeout -k 10 240 python3 -u tools/capture_info.py $2 >> $O/capinfo.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/capinfo.txt
  [ $rc -eq 0 ] || exit $rc
}
step guarded "--n 330 --guard 1" && step lifted330 "--n 330 --guard 0" && step lifted4096 "--n 4096 --guard 0 --chunks 8" && echo done
