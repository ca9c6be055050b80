# Bench-line check after the Poisson-small pricing change (tag $1): 48^2 Poisson and Gaussian, then the default line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04b48p}; mkdir -p $O
cd $R && timeout -k 10 300 python3 bench.py --size 48 --batch 256 --llh Poisson --steps 100 --warmup 10 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48p_$T.json 2> $O/bench48p_$T.err &&
timeout -k 10 300 python3 bench.py --size 80 --llh Poisson --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench80p_$T.json 2> $O/bench80p_$T.err &&
timeout -k 10 400 python3 bench.py > $O/bench_$T.json 2> $O/bench_$T.err
