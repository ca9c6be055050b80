# A/B of argument pinning on one box: variants/pin0.so vs pin1.so, alternated, eager vs replay (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-ab}
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in pin0 pin1 pin0 pin1; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  echo "== $v" >> $O/pinab_$T.txt
  timeout -k 10 200 python3 $R/tools/graph_vs_eager.py 3 2>/dev/null | grep -E "^(eager|graph)" >> $O/pinab_$T.txt || break
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
