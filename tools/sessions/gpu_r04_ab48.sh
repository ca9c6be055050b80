# 256 x 48^2 A/B of engine variants (variants/<name>.so swapped in; tag $1, names $2), then a 256^2 line per
# variant (names $3, may be empty): clean value, graphed / eager-interleaved, per-op times.  In-tree .so restored.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-ab48}; mkdir -p $O
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in $2; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 200 python3 $R/bench.py --size 48 --batch 256 --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-ingest > /tmp/sov.json 2>/tmp/sov.err || { echo "fail $v"; tail -5 /tmp/sov.err; cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/sov.json').read().strip().splitlines()[-1]); g=d['graphed']; print('48 $v |', round(d['value']), 'graphed', round(g['value']), 'eager', round(g['eager_interleaved']['value']), 'bitid', g['bit_identical_to_eager'], {k: round(x['avg_ms']*1e3,2) for k,x in d['kernels'].items()})" | tee -a $O/ab48_$T.txt
done
for v in $3; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 200 python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-ingest --no-graph > /tmp/sov.json 2>/tmp/sov.err || { echo "fail $v"; tail -5 /tmp/sov.err; cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/sov.json').read().strip().splitlines()[-1]); print('256 $v |', round(d['value']), {k: round(x['avg_ms'],4) for k,x in d['kernels'].items()})" | tee -a $O/ab48_$T.txt
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
