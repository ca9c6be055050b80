R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "subnet or full or admm48 or configs or scalar or broadcast or gx or serving" > $O/sn_tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/sn_bench48.json 2> $O/sn_bench48.err &&
timeout -k 10 300 python3 bench.py --no-e2e --no-ingest --no-cpu-baseline > $O/sn_bench.json 2> $O/sn_bench.err
