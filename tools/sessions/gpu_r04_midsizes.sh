# Fused mid sizes (tag $1): 4096-galaxy bench lines at 80^2 / 112^2 / 144^2, fused (k_gal_mid + k_gal_mid_init) and
# the runtime-planned chains (--fused 0 --fused-init 0) for comparison.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04mid}; mkdir -p $O
cd $R && for L in 80 112 144; do
  timeout -k 10 300 python3 bench.py --size $L --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench${L}_$T.json 2> $O/bench${L}_$T.err || exit 1
  timeout -k 10 300 python3 bench.py --size $L --fused 0 --fused-init 0 --no-e2e --no-ingest --no-cpu-baseline --no-graph > $O/bench${L}chain_$T.json 2> $O/bench${L}chain_$T.err || exit 1
done
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --steps 200 --warmup 20 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
