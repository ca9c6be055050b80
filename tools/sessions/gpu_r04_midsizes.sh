# Fused mid sizes (tag $1): the mid-size GPU tests; 4096-galaxy bench lines at 80^2 (variants m256 / m512: 256- vs
# 512-thread workgroups), 112^2 and 144^2, fused and with the runtime-planned chains (--fused 0 --fused-init 0);
# the 48^2 line (roofline timing from a replayed graph).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04mid}; mkdir -p $O
B="python3 bench.py --no-e2e --no-ingest --no-cpu-baseline --no-graph"
cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_serving.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_mid or chunked_pipeline" > $O/mid_tests_$T.log 2>&1 &&
cp galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so &&
for v in m512 m256; do cp variants/$v.so galaxy-deconv_amd/gdeconv/libgdeconv.so; timeout -k 10 300 $B --size 80 > $O/bench80${v}_$T.json 2> $O/bench80${v}_$T.err || { cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so; exit 1; }; done
cp /tmp/orig.so galaxy-deconv_amd/gdeconv/libgdeconv.so
for L in 80 112 144; do
  timeout -k 10 300 $B --size $L --fused 0 --fused-init 0 > $O/bench${L}chain_$T.json 2> $O/bench${L}chain_$T.err || exit 1
done
for L in 112 144; do timeout -k 10 300 $B --size $L > $O/bench${L}_$T.json 2> $O/bench${L}_$T.err || exit 1; done
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --steps 200 --warmup 20 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
