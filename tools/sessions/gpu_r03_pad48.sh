# Round-3 last session (tag = $1): padded LDS spectrum row stride in k_gal_small_t<48> (engine rev r03.7) -
# GPU tests on the in-tree build, 48^2 A/B against the r03.6 build (variants/st_old.so), then the whole final
# recipe (PMC for every workload, kernel stats, bench lines) on the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03pad}; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rf -k "48 or small or configs1 or overlap" --timeout 120 --timeout-method thread > $O/gpu_small_$T.log 2>&1 &&
bash tools/sessions/gpu_ab48.sh $T "st_old st_new st_old st_new st_old st_new" &&
bash tools/sessions/gpu_r03_final.sh $T
