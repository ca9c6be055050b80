# Round-3 session s (tag = $1): 8 x 6 transposing plan for the 48^2 iteration (k_gal_small_t) - A/B against
# the 4 x 12 kernel at 256 x 48^2 (graphed and eager), then the whole GPU suite on the in-tree build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03s}; mkdir -p $O
cd $R && timeout -k 10 200 python3 -u -m pytest tests -m gpu -x -q -rf -k "48 or small or configs1 or overlap" --timeout 120 --timeout-method thread > $O/gpu_small_$T.log 2>&1 &&
bash tools/sessions/gpu_ab48.sh $T "st0 st1 st0 st1 st0 st1" &&
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1
