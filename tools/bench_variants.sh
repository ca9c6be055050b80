# time prebuilt libgdeconv variants (variants/*.so) with the default bench
R=${GRAFT_REPO_ROOT:-$(pwd)}
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in "$@"; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --no-e2e --fused 1 > $R/gpurun_out/var_$v.json 2> $R/gpurun_out/var_$v.err || { echo "variant $v failed rc=$?"; break; }
  echo "variant $v done"
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
