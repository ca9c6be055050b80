# Fused small / mid Poisson iteration (tag $1): the whole GPU suite (the new fused-vs-chain-vs-oracle test, the
# 48^2 Poisson goldens and per-iteration replays, graphs), then Poisson bench lines at 48^2 (graph) and 80^2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04pois}; mkdir -p $O
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -rfs --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --llh Poisson --steps 100 --warmup 10 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48p_$T.json 2> $O/bench48p_$T.err &&
timeout -k 10 300 python3 bench.py --size 80 --llh Poisson --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench80p_$T.json 2> $O/bench80p_$T.err


