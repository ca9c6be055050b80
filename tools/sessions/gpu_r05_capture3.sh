# the capture crash under HIP API logging: mode 0 (serial) must pass; mode 2 with AMD_LOG_LEVEL=3 last
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05cap3}
cd $R && GD_CAPTURE_PIPELINE=0 timeout -k 10 200 python3 tools/capture_repro.py 4096 160 0 > $O/capture_$T.txt 2>&1 &&
GD_CAPTURE_PIPELINE=2 AMD_LOG_LEVEL=3 timeout -k 10 200 python3 tools/capture_repro.py 4096 160 0 > $O/capture_${T}_log.txt 2>&1
echo "rc=$?" >> $O/capture_$T.txt
