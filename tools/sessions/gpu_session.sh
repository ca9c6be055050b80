#!/bin/bash
# One GPU-box session: smoke -> all GPU tests -> bench -> rocprofv3 kernel trace -> PMC passes.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
TAG=${TAG:-s}
run() { echo "[session] $*" >&2; }
run smoke && timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > $O/smoke.log 2>&1 &&
run tests && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
run bench && timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err &&
run trace && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_trace -o trace --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > $O/trace_bench.json 2> $O/trace.err) &&
run pmc_fetch && (cd /tmp && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_col|k_row|k_gal|k_psf|k_subnet" -d $O/prof_fetch -o fetch --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /dev/null 2> $O/pmc_fetch.err) &&
run pmc_write && (cd /tmp && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_col|k_row|k_gal|k_psf|k_subnet" -d $O/prof_write -o write --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest > /dev/null 2> $O/pmc_write.err)
rc=$?
[ $rc -eq 0 ] && run torchrun1 && timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $O/bench_torchrun1.json 2> $O/bench_torchrun1.err
rc=$?
[ $rc -eq 0 ] && run bench48 && timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-cpu-baseline > $O/bench48.json 2> $O/bench48.err
rc=$?
[ $rc -eq 0 ] && run bench_rl && timeout -k 10 300 python3 bench.py --workload rl > $O/bench_rl.json 2> $O/bench_rl.err
rc=$?
echo "[session] rc=$rc" >&2
exit $rc
