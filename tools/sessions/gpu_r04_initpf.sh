# k_gal_mid_init y prefetch (vI: GD_MID_INIT_PF=1, the first y pair loaded before the PSF rows) against vA (tag $1):
# the mid tests on vI, then 4096-galaxy Gaussian lines at 96 / 112 / 144 / 160.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04initpf}; mkdir -p $O
cd $R && cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so || exit 1
restore() { cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; }
cp variants/vI.so galaxy-deconv_amd/gdeconv/libgdeconv.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_mid" > $O/initpf_tests_$T.log 2>&1 || { restore; exit 1; }
for v in vA vI vA vI; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  for L in 96 112 144 160; do
    timeout -k 10 200 python3 bench.py --size $L --steps 3 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline --no-graph > /tmp/b.json 2>/tmp/b.err || { cp /tmp/b.err $O/initpf_err_$T.txt; restore; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$v $L', round(d['value']), {k: round(x['avg_ms'],4) for k,x in d['kernels'].items() if 'op_' in k})" >> $O/initpf_$T.txt
  done
done
restore
