# Poisson (the reference's default llh) at 48^2 / 80^2 (tag $1): bench lines with the graph.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04p48}; mkdir -p $O
cd $R && timeout -k 10 300 python3 bench.py --size 48 --batch 256 --llh Poisson --steps 100 --warmup 10 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48p_$T.json 2> $O/bench48p_$T.err &&
timeout -k 10 300 python3 bench.py --size 80 --llh Poisson --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench80p_$T.json 2> $O/bench80p_$T.err
