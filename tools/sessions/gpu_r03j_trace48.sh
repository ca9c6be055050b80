# 48^2 kernel trace: per-dispatch durations and gaps of the graphed / eager forward (configs[1]).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03j}
cd $R && mkdir -p $O &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof48_$T -o run -- python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline --steps 20 > $O/bench48_$T.json 2> $O/bench48_$T.err
