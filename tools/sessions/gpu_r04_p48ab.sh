# 48^2 Poisson A/B (tag $1): k_pois_small / the init role with 256 (p256) vs 512 (p512) threads per galaxy.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04p48ab}; mkdir -p $O
cd $R && cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in p256 p512 p256 p512; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 200 python3 bench.py --size 48 --batch 256 --llh Poisson --steps 100 --warmup 10 --no-e2e --no-ingest --no-cpu-baseline > /tmp/b.json 2>/tmp/b.err || { cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), 'graphed', round(d['graphed']['value']), d['roofline']['avg_launch_ms'], {k: round(x['avg_ms']*1e3,2) for k,x in d['kernels'].items()})" >> $O/p48ab_$T.txt
done
cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so
