# Runtime-planned size cap 1024 -> 1638 (tag $1): the generic-size GPU tests (rfft2 round trips up to
# 1638 per side, Wiener / ADMM at 1638 x 1536 and 1200 x 1400 against the fp64 oracle) and the
# UnrolledADMMGaussian tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04large}; mkdir -p $O
cd $R && timeout -k 10 400 python3 -u -m pytest tests/test_gpu_generic.py tests/test_gpu_next.py -m gpu -x -v -rfs -s --timeout 120 --timeout-method thread > $O/large_tests_$T.log 2>&1
