# A/B of engine variants (variants/<name>.so swapped in, tag = $1, names = $2, bench args = $3): each
# variant's bench line, per-op times.  The in-tree .so is restored at the end.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-ab}; mkdir -p $O
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in $2; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 200 python3 $R/bench.py $3 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /tmp/sov.json 2>/tmp/sov.err || { echo "fail $v"; tail -5 /tmp/sov.err; cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/sov.json').read().strip().splitlines()[-1]); print('$v |', round(d['value']), {k: round(x['avg_ms'],3) for k,x in d['kernels'].items()})" | tee -a $O/ab_$T.txt
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
