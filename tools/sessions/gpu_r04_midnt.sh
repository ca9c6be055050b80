# Mid-size workgroup / prefetch A/B (tag $1): each variant's mid tests, then 4096-galaxy Gaussian lines at
# 80 / 112 / 144 / 160 for vA (default), vB (80^2 at 512 threads), vC (prefetch at every NT), vD (prefetch, 256 threads
# above 80^2), vE (256 threads above 80^2, no prefetch there).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04midnt}; mkdir -p $O
cd $R && cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so || exit 1
restore() { cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; }
for v in vB vC vD vE; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  timeout -k 10 200 python3 -u -m pytest tests/test_gpu_generic.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_mid or shared_psf" > $O/midnt_tests_${v}_$T.log 2>&1 || { restore; exit 1; }
done
for v in vA vB vC vD vE vA vB vC vD vE; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  for L in 80 112 144 160; do
    timeout -k 10 200 python3 bench.py --size $L --steps 3 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline --no-graph > /tmp/b.json 2>/tmp/b.err || { cp /tmp/b.err $O/midnt_err_$T.txt; restore; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$v $L', round(d['value']), {k: round(x['avg_ms'],4) for k,x in d['kernels'].items() if 'op_' in k})" >> $O/midnt_$T.txt
  done
done
restore
