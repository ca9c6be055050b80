# RL instruction-count variants (tag = $1): the RL parity tests on the default build, then an interleaved A/B of
# variants/rl_*.so on configs[4] (4096 x RL(100)).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r06o}; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "richardson" tests/ > $O/${T}_rl_tests.txt 2>&1 &&
bash tools/ab_variants.sh ${T}_ab 3 "${VARS:-rl_scaled rl_unscaled rl_unscaled_tab}" "--workload rl --steps 3 --warmup 1" > $O/${T}_ab.txt 2>&1
