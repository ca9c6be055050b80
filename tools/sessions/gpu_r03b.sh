# Round-3 session b: per-pixel parity vs fp64 (both columns), host-overhead profile of the eager 48^2 forward,
# the rest of the GPU suite, 48^2 bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-b}; mkdir -p $O
cd $R && rm -f $O/parity_$T.jsonl
GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pixel_parity.py tests/test_gpu_generic.py -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pixpar_$T.log 2>&1
echo "pixel parity exit $?" >> $O/pixpar_$T.log
timeout -k 10 300 python3 -u tools/host_profile.py > $O/hostprof_$T.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_pixel_parity.py > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
