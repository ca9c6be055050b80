# The 256-thread prefetching k_gal_mid at 80 / 112^2 as the default (all GPU tests, Gaussian lines), then the Poisson
# prefetch at every plan (vP: GD_POIS_PF=2) against vA (512-thread plans only): its tests, Poisson 64 / 80 lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04poispf}; mkdir -p $O
cd $R && timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 || exit 1
for L in 80 112; do
  timeout -k 10 200 python3 bench.py --size $L --no-e2e --no-ingest --no-cpu-baseline > $O/bench${L}_$T.json 2> $O/bench${L}_$T.err || exit 1
done
cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so || exit 1
restore() { cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; }
cp variants/vP.so galaxy-deconv_amd/gdeconv/libgdeconv.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_parity.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_poisson or init_overlap or shared_psf" > $O/poispf_tests_$T.log 2>&1 || { restore; exit 1; }
for v in vA vP vA vP; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  for L in 64 80; do
    timeout -k 10 200 python3 bench.py --size $L --llh Poisson --steps 3 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline --no-graph > /tmp/b.json 2>/tmp/b.err || { cp /tmp/b.err $O/poispf_err_$T.txt; restore; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$v $L', round(d['value']), {k: round(x['avg_ms'],4) for k,x in d['kernels'].items() if 'op_' in k})" >> $O/poispf_$T.txt
  done
done
restore
