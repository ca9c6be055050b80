# 160^2 graph fix check (tag $1): the serving tests (chunked-pipeline capture included), then the
# 4096 x 160^2 bench line with the graph; and the kernel timeline of the 48^2 graphed forward.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04fix}; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 300 python3 -u -X faulthandler -m pytest tests/test_gpu_serving.py -m gpu -x -q -rfs --timeout 120 --timeout-method thread > $O/serving_$T.log 2>&1 &&
timeout -k 10 300 python3 -X faulthandler bench.py --size 160 --no-e2e --no-ingest --no-cpu-baseline > $O/bench160_$T.json 2> $O/bench160_$T.err &&
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d $O/gt48_$T -o run --output-format csv -- python3 $R/tools/graph_trace.py 20 256 48 > $O/gt48_$T.txt 2>&1 &&
cd $R && python3 tools/graph_timeline.py $O/gt48_$T/run_kernel_trace.csv 0 10 >> $O/gt48_$T.txt 2>&1
