# k_rl_reg variants: RL parity tests + RL(100) bench line per prebuilt variants/<name>.so (tag = $1, names = $2)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-rl}
cp $R/galaxy-deconv_amd/gdeconv/libgdeconv.so /tmp/orig.so
for v in $2; do
  cp $R/variants/$v.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
  cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -rA -k richardson --timeout 120 --timeout-method thread > $O/rltests_${T}_$v.log 2>&1 || { echo "tests failed $v"; break; }
  timeout -k 10 300 python3 bench.py --workload rl --steps 3 --warmup 1 --no-e2e --no-ingest --no-graph --no-cpu-baseline > $O/bench_rl_${T}_$v.json 2> $O/bench_rl_${T}_$v.err || { echo "bench failed $v"; break; }
done
cp /tmp/orig.so $R/galaxy-deconv_amd/gdeconv/libgdeconv.so
