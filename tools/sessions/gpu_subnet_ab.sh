# SubNet fused-launch A/B + SubNet GPU tests + 48^2 bench (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-sn}
cd $R && timeout -k 10 200 python3 tools/subnet_ab.py > $O/snab_$T.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "subnet or SubNet or full_model or admm48 or configs" > $O/sn_tests_$T.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
