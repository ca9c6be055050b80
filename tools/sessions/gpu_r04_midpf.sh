# k_gal_mid prefetch A/B (tag $1): the mid-size tests, then 4096-galaxy lines at 112 / 144 / 160 for pf0 / pf1.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04midpf}; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_mid or shared_psf" > $O/midpf_tests_$T.log 2>&1 &&
cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so &&
for v in pf0 pf1 pf0 pf1; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  for L in 112 144 160; do
    timeout -k 10 200 python3 bench.py --size $L --steps 3 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline --no-graph > /tmp/b.json 2>/tmp/b.err || { cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$v $L', round(d['value']), {k: round(x['avg_ms'],4) for k,x in d['kernels'].items() if 'op_' in k})" >> $O/midpf_$T.txt
  done
done
cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so
