R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05cap5}
cd $R && for args in "6 1 9 2 4"; do
  timeout -k 10 60 tools/bin/capture_probe $args >> $O/capture_$T.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/capture_$T.txt
  [ $rc -eq 0 ] || exit $rc
done
