# Round-4 combined session (tag $1): the batched MLP A/B (tools/bin/ksn_mlp fingerprints), then the final set
# (gpu_r04_final.sh: tests, smoke, PMC passes, rocprof stats, bench lines), then the SQ counters of the 48^2 kernels
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04z}; mkdir -p $O
for i in 1 2; do timeout -k 10 60 $R/tools/bin/ksn_mlp 4096 256 20 || exit 1; done > $O/ksn_mlp_$T.txt 2>&1 &&
bash $R/tools/sessions/gpu_r04_final.sh $T &&
bash $R/tools/sessions/gpu_r03_sq48.sh sq48_$T
