# Poisson two-pass check: Poisson-related GPU tests, then the Poisson bench line (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-p}
cd $R && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "Poisson or poisson or admm48 or pipelined or full_model or scalar" > $O/pois_tests_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-graph --no-cpu-baseline > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err
