# Time prebuilt engine variants (variants/<name>.so swapped in) under several bench configurations.
#   bash tools/so_variants.sh "name1 name2 ..."   (configs below)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in $1; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  for cfg in "--workload rl --steps 2 --warmup 1" "--steps 3 --warmup 1" "--steps 3 --warmup 1 --fused 0"; do
    timeout -k 10 150 python3 $R/bench.py $cfg --no-cpu-baseline --no-e2e --no-graph --no-ingest > /tmp/sov.json 2>/dev/null || { echo "fail $v $cfg"; continue; }
    python3 -c "import json; d=json.loads(open('/tmp/sov.json').read().strip().splitlines()[-1]); print('$v | $cfg |', round(d['value']), {k: round(x['avg_ms'],3) for k,x in d['kernels'].items()})"
  done
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
