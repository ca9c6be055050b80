# capture crash root cause: 4096 x 160^2 graphed forward with the chunked (pipelined) init under capture.
# mode 0 (serial under capture), mode 2 (fresh event set per operation), then mode 1 (shared events, the round-4
# crash) LAST: a host-side segfault there ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r05cap}; mkdir -p $O
B="python3 bench.py --size 160 --batch 4096 --fused-init 0 --steps 3 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline --no-extra --settle-s 0"
cd $R && for m in 0 2 1; do
  echo "=== GD_CAPTURE_PIPELINE=$m" >> $O/capture_$T.txt
  GD_CAPTURE_PIPELINE=$m timeout -k 10 200 $B > $O/capture_${T}_m$m.json 2>> $O/capture_$T.txt
  rc=$?; echo "rc=$rc" >> $O/capture_$T.txt
  [ $rc -eq 0 ] || exit $rc
done
