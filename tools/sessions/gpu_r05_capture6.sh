R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05cap6}
cd $R && echo "=== init inline under capture" >> $O/capture_$T.txt &&
GD_CAPTURE_PIPELINE=2 GD_EXP_INIT_INLINE_CAPTURE=1 timeout -k 10 200 python3 tools/capture_repro.py 4096 160 0 >> $O/capture_$T.txt 2>&1 &&
echo "=== persistent fork/join events" >> $O/capture_$T.txt &&
GD_CAPTURE_PIPELINE=2 GD_EXP_PERSIST_EVENTS=1 timeout -k 10 200 python3 tools/capture_repro.py 4096 160 0 >> $O/capture_$T.txt 2>&1
echo "rc=$?" >> $O/capture_$T.txt
