# Prefetch A/B round 2 (tag $1): the fused mid / fused Poisson tests, then 4096-galaxy lines for pf0 (GD_MID_PF=0,
# GD_POIS_PF=0) / pf1: Gaussian 112 / 144 / 160 (k_gal_mid_init's prefetch) and Poisson 48 / 96 / 112 (k_pois_small's).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04pf2}; mkdir -p $O
cd $R && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_parity.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_mid or shared_psf or fused_poisson or init_overlap" > $O/pf2_tests_$T.log 2>&1 &&
cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so &&
for v in pf0 pf1 pf0 pf1; do
  cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so
  for c in "112 Gaussian" "144 Gaussian" "160 Gaussian" "48 Poisson" "96 Poisson" "112 Poisson"; do
    set -- $c
    timeout -k 10 200 python3 bench.py --size $1 --llh $2 --steps 3 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline --no-graph > /tmp/b.json 2>/tmp/b.err || { cp /tmp/b.err $O/pf2_err_$T.txt; cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/b.json').read().strip().splitlines()[-1]); print('$v $1 $2', round(d['value']), {k: round(x['avg_ms'],4) for k,x in d['kernels'].items() if 'op_' in k})" >> $O/pf2_$T.txt
  done
done
cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so
