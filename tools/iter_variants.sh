# Time prebuilt engine variants (variants/<name>.so swapped in) on the default 256^2 bench.
#   bash tools/iter_variants.sh "name1 name2 ..."
R=${GRAFT_REPO_ROOT:-$(pwd)}
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in $1; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 150 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /tmp/sov.json 2>/dev/null || { echo "fail $v"; break; }
  python3 -c "import json; d=json.loads(open('/tmp/sov.json').read().strip().splitlines()[-1]); print('$v |', round(d['value']), {k: round(x['avg_ms'],3) for k,x in d['kernels'].items()})"
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
