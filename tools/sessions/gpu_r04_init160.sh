# 160^2 fused init check (tag $1): the 160^2 generic tests (fused vs chains vs oracle, n = 0 is init_l2 alone),
# then the 4096 x 160^2 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04i160}; mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py -m gpu -x -v -rfs -s --timeout 120 --timeout-method thread -k "fused_160" > $O/mid160_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 160 --no-e2e --no-ingest --no-cpu-baseline > $O/bench160_$T.json 2> $O/bench160_$T.err
