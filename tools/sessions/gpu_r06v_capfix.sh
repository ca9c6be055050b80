# capture crash: probe modes 10 / 9 (internal streams created inside the capture) and the engine diagnostic with the
# candidate fix (variants/libgdeconv_capearly.so: capture streams created by gd_set_capture_pipeline(2)); stops at a failure
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v; mkdir -p $O
probe() {
  echo "=== probe PROBE_FRESH=$1 mode $2 K=$3" >> $O/log.txt
  PROBE_FRESH=$1 timeout -k 10 60 ./variants/capture_probe $2 $3 9 2 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
info() {
  echo "=== capture_info $1" >> $O/log.txt
  timeout -k 10 240 python3 -u tools/capture_info.py $1 >> $O/log.txt 2>&1
  rc=$?; echo "rc=$rc" >> $O/log.txt; [ $rc -eq 0 ]
}
L=galaxy-deconv_amd/gdeconv/libgdeconv.so
probe 1 10 8 && cp $L /tmp/lib_orig.so && cp variants/libgdeconv_capearly.so $L && info "--n 330 --guard 0" && cp /tmp/lib_orig.so $L && probe 1 9 8 && probe 0 9 8 && echo done
