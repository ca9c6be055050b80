# One-launch SubNet MLP rework (tag $1): kernel A/B with fingerprints (ksn_f0 = round-3 MLP, ksn_f1 = staged
# W2 / W3 + chunked W1), phase traces, the 256 x 48^2 forward A/B (variants f0 / f1), then the SubNet GPU tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r04mlp2}; mkdir -p $O
bash $R/tools/sessions/gpu_r04_sn.sh $T "f0 f1 f0 f1" "f0t f1t" &&
bash $R/tools/sessions/gpu_r04_ab48.sh $T "f0 f1 f0 f1" "" &&
cd $R && timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rfs --timeout 120 --timeout-method thread -k "subnet or admm48 or configs1" > $O/sn_tests_$T.log 2>&1
