# capture crash: the engine probe's runtime version under torch's HIP (7.0), then the ctypes-only sequence inside a
# torch process; stops at the first failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zb; mkdir -p $O
TL=$(python3 -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
echo "=== engine probe side 1, LD_LIBRARY_PATH=$TL" >> $O/log.txt
LD_LIBRARY_PATH=$TL timeout -k 10 120 ./variants/capture_engine_probe 1 330 160 6 >> $O/log.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ] || exit $rc
echo "=== engine probe side 1, /opt/rocm" >> $O/log.txt
timeout -k 10 120 ./variants/capture_engine_probe 1 330 160 6 >> $O/log.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ] || exit $rc
echo "=== torch probe pure" >> $O/log.txt
timeout -k 10 180 python3 -u tools/capture_torch_probe.py pure >> $O/log.txt 2>&1; rc=$?; echo "rc=$rc" >> $O/log.txt; exit $rc
