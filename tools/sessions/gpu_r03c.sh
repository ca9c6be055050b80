# Round-3 session c: per-pixel parity vs fp64 with quantiles and raw dumps
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-c}; mkdir -p $O
cd $R && rm -f $O/parity_$T.jsonl
GD_PARITY_DUMP=$O/pixdump_$T GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pixel_parity.py -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pixpar_$T.log 2>&1
echo "pixel parity exit $?" >> $O/pixpar_$T.log
