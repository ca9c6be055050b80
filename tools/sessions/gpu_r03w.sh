# Round-3 session w (tag = $1): padded row stride of the SubNet's 16^2 stage (GD_SN_RS16) - kernel A/B with
# the torch-free microbenchmark (variants/ksn_rs16 / rs20 / rs24, rs20 phase trace), SubNet GPU tests and the
# 48^2 bench line on the in-tree build (rs20).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03w}; mkdir -p $O
cd $R && for v in rs16 rs20 rs24 rs16 rs20 rs24; do echo "variant $v" >> $O/ksn_$T.txt; timeout -k 10 60 variants/ksn_$v 4096 256 20 >> $O/ksn_$T.txt 2>&1 || exit 1; done &&
timeout -k 10 60 variants/ksn_rs20_tr 4096 256 5 > $O/ksn_tr_$T.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rf -k "subnet or SubNet or 48 or configs1 or overlap or full_model or rhos or xdense" --timeout 120 --timeout-method thread > $O/gpu_sn_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --steps 20 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
