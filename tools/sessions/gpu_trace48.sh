# Kernel trace of the 48^2 x 256 forward, eager and hipGraph-replayed (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-t48}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace48_$T -o run -- python3 $R/bench.py --size 48 --batch 256 --steps 20 --no-e2e --no-ingest --no-cpu-baseline > $O/trace48_$T.json 2> $O/trace48_$T.err
