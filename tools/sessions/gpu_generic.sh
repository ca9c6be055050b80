# Runtime-size path check (tag = $1): the generic-size GPU tests, then the size-dependent parity tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-g}
cd $R && GD_PARITY_LOG=$O/parity_gen_$T.jsonl timeout -k 10 400 python3 -u -m pytest tests/test_gpu_generic.py -x -v -rA --timeout 120 --timeout-method thread > $O/gen_tests_$T.log 2>&1
