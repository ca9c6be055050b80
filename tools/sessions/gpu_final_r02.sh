# Final round-2 check on the committed tree (tag = $1): SubNet kbench, GPU tests, smoke, bench lines
# (256^2 default, 48^2, RL(100), Poisson, torchrun N=1), rocprofv3 kernel stats of the default bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-rc}; mkdir -p $O
timeout -k 10 60 $R/tools/kbench_subnet 4096 256 20 > $O/ksn_$T.txt 2>&1 &&
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 500 python3 bench.py --workload rl --no-e2e --no-ingest > $O/bench_rl_$T.json 2> $O/bench_rl_$T.err &&
timeout -k 10 400 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-graph > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-ingest > $O/bench_torchrun1_$T.json 2> $O/bench_torchrun1_$T.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ps_$T -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest --steps 3 --warmup 1 > $O/bench_stats_$T.json 2> $O/stats_$T.err
