# batched MLP A/B (tools/bin/ksn_mlp: k_subnet_mlp vs k_subnet_mlp_mfma fingerprints + the fused kernel's), then
# GPU tests, smoke, the default bench line ($1 tag)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r04mlp}; mkdir -p $O
for i in 1 2; do timeout -k 10 60 $R/tools/bin/ksn_mlp 4096 256 20 || exit 1; done > $O/ksn_$T.txt 2>&1 &&
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rfs --timeout 300 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py --no-ingest --no-e2e > $O/bench_$T.json 2> $O/bench_$T.err
