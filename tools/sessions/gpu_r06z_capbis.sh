# capture crash bisection: C++ engine probe with torch-style streams and temporary events, then the torch probe on
# externally created streams; stops at a failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06z; mkdir -p $O
echo "=== engine probe side 4" >> $O/log.txt
timeout -k 10 120 ./variants/capture_engine_probe 4 330 160 6 >> $O/log.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ] || exit $rc
echo "=== torch probe ext" >> $O/log.txt
timeout -k 10 180 python3 -u tools/capture_torch_probe.py ext >> $O/log.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/log.txt; exit $rc
