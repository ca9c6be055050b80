# SubNet feature kernel time per threads-per-galaxy variant (variants/sn*.so swapped in)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in 256 512 1024; do
  cp $R/variants/sn$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  for cfg in "48 256" "256 4096"; do
    set -- $cfg
    timeout -k 10 120 python3 $R/bench.py --size $1 --batch $2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /tmp/snv.json 2>/dev/null || { echo "fail $v $cfg"; break; }
    python3 -c "import json; d=json.loads(open('/tmp/snv.json').read().strip().splitlines()[-1]); print('threads $v size $1', round(d['value']), round(d['kernels']['k_subnet_features<128,FEATURES>']['avg_ms']*1e3,1), 'us')"
  done
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
