# Round-4 combined session (tag $1): the batched MLP A/B (tools/bin/ksn_mlp fingerprints); the new 160^2 fused
# iteration's tests on their own (a failing assertion is recorded, a fault / abort / timeout ends the session);
# then the final set (gpu_r04_final.sh: all GPU tests, smoke, PMC passes, rocprof stats, bench lines), the SQ
# counters of the 48^2 kernels and a 160^2 bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04z}; mkdir -p $O
for i in 1 2; do timeout -k 10 60 $R/tools/bin/ksn_mlp 4096 256 20 || exit 1; done > $O/ksn_mlp_$T.txt 2>&1 || exit 1
cd $R && timeout -k 10 300 python3 -u -m pytest tests/test_gpu_generic.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "fused_160" > $O/mid160_tests_$T.log 2>&1
rc=$?; echo "160 tests rc=$rc" >> $O/mid160_tests_$T.log
case $rc in 0) ;; 1) export PYTEST_DESELECT="not fused_160" ;; *) exit $rc ;; esac
bash $R/tools/sessions/gpu_r04_final.sh $T &&
bash $R/tools/sessions/gpu_r03_sq48.sh sq48_$T &&
timeout -k 10 300 python3 $R/bench.py --size 160 --no-e2e --no-ingest --no-cpu-baseline > $O/bench160_$T.json 2> $O/bench160_$T.err
