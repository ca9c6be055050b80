# Poisson fused (k_pois_small) vs three-kernel chain per size (tag $1), 4096 galaxies, no graph.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04psw}; mkdir -p $O
B="python3 bench.py --llh Poisson --no-e2e --no-ingest --no-cpu-baseline --no-graph --steps 3 --warmup 1"
cd $R && for L in 64 96 112; do
  timeout -k 10 200 $B --size $L > $O/bp${L}_$T.json 2> $O/bp${L}_$T.err || exit 1
  timeout -k 10 200 $B --size $L --fused 0 > $O/bp${L}chain_$T.json 2> $O/bp${L}chain_$T.err || exit 1
done
