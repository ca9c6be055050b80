# Engine variants (variants/<name>.so swapped in, tag = $1, names = $2): Gaussian / Poisson / RL bench lines
# (no graph, no e2e), per-op times.  The in-tree .so is restored at the end.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-p}; mkdir -p $O
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in $2; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  for cfg in "--steps 5" "--llh Poisson --steps 3" "--workload rl --steps 2"; do
    timeout -k 10 200 python3 $R/bench.py $cfg --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /tmp/sov.json 2>/tmp/sov.err || { echo "fail $v $cfg"; cat /tmp/sov.err | tail -5; exit 1; }
    python3 -c "import json; d=json.loads(open('/tmp/sov.json').read().strip().splitlines()[-1]); print('$v | $cfg |', round(d['value']), {k: round(x['avg_ms'],3) for k,x in d['kernels'].items()})" | tee -a $O/variants_$T.txt
  done
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
