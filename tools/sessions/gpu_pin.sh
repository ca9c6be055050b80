# Argument pinning check (tag = $1): eager vs replay trace script, bench line, 256^2 fused-path GPU tests
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-pin}
cd $R && timeout -k 10 200 python3 tools/graph_vs_eager.py 3 > $O/gve_$T.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-cpu-baseline > $O/bench_pois_$T.json 2> $O/bench_pois_$T.err &&
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "256 or poisson or Poisson or fused or graph" > $O/pin_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py -x -q -rA --timeout 120 --timeout-method thread > $O/gen_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 80 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench80_$T.json 2> $O/bench80_$T.err &&
timeout -k 10 300 python3 bench.py --size 255 --batch 1024 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench255_$T.json 2> $O/bench255_$T.err
