# r05 session B: streaming ceilings incl. k_gal_reg's own access pattern (layout A/B), then the capture probe
# (fresh events first; shared-event captures last since a crash ends the call).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; T=${1:-r05b}
cd $R &&
timeout -k 10 240 tools/bin/kbench_stream 4096 20 > $O/kstream_$T.txt 2>&1 &&
timeout -k 10 60 tools/bin/capture_probe 1 32 9 2 3 > $O/capture_$T.txt 2>&1 &&
timeout -k 10 60 tools/bin/capture_probe 0 1 9 2 3 >> $O/capture_$T.txt 2>&1 &&
timeout -k 10 60 tools/bin/capture_probe 0 2 9 2 3 >> $O/capture_$T.txt 2>&1 &&
timeout -k 10 60 tools/bin/capture_probe 0 8 9 2 3 >> $O/capture_$T.txt 2>&1 &&
timeout -k 10 60 tools/bin/capture_probe 0 32 9 2 3 >> $O/capture_$T.txt 2>&1
echo "exit $?" >> $O/capture_$T.txt
