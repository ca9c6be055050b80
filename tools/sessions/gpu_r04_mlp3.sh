# One-launch SubNet MLP, second pass (tag $1): f0 = round-3 MLP, f1 / f2 = chunked W1 (16 / 32 rows) + layers 2-3 by
# v_readlane with LDS-staged weight columns; kernel A/B with fingerprints, traces, the 48^2 forward A/B, SubNet tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r04mlp3}; mkdir -p $O
bash $R/tools/sessions/gpu_r04_sn.sh $T "f0 f1 f2 f0 f1 f2" "f0t f1t f2t" &&
bash $R/tools/sessions/gpu_r04_ab48.sh $T "f0 f1 f2 f0 f1 f2" "" &&
cd $R && timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "subnet or admm48 or configs1" > $O/sn_tests_$T.log 2>&1
