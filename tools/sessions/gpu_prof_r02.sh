# Round-2 evidence for the current engine (tag = $1): PMC traffic (FETCH / WRITE in separate passes) for
# the default 256^2 bench, the 48^2 and RL(100) workloads, kernel stats, then the bench lines.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r02}
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-graph --no-ingest"
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pf_$T -o fetch --output-format csv -- $B --steps 1 --warmup 1 > /dev/null 2> $O/pmc_$T.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pw_$T -o write --output-format csv -- $B --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ps_$T -o run --output-format csv -- $B --steps 3 --warmup 1 > $O/bench_stats_$T.json 2>> $O/pmc_$T.err &&
cd $R && python3 tools/pmc_summary.py $O/pf_$T/fetch_counter_collection.csv $O/pw_$T/write_counter_collection.csv $O/pmc_traffic_$T.json --batch 4096 --size 256 --n-iters 8 > $O/pmc_summary_$T.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pf48_$T -o fetch --output-format csv -- $B --size 48 --batch 256 --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pw48_$T -o write --output-format csv -- $B --size 48 --batch 256 --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
cd $R && python3 tools/pmc_summary.py $O/pf48_$T/fetch_counter_collection.csv $O/pw48_$T/write_counter_collection.csv $O/pmc_traffic48_$T.json --batch 256 --size 48 --n-iters 8 > $O/pmc_summary48_$T.txt 2>&1 &&
cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gd::" -d $O/pfrl_$T -o fetch --output-format csv -- $B --workload rl --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gd::" -d $O/pwrl_$T -o write --output-format csv -- $B --workload rl --steps 1 --warmup 1 > /dev/null 2>> $O/pmc_$T.err &&
cd $R && python3 tools/pmc_summary.py $O/pfrl_$T/fetch_counter_collection.csv $O/pwrl_$T/write_counter_collection.csv $O/pmc_trafficrl_$T.json --batch 4096 --size 256 --rl-calls 2 --n-iters 100 > $O/pmc_summaryrl_$T.txt 2>&1 &&
cp $O/pmc_traffic_$T.json $R/profiles/pmc_traffic.json && cp $O/pmc_traffic48_$T.json $R/profiles/pmc_traffic_48.json &&
cp $O/pmc_trafficrl_$T.json $R/profiles/pmc_traffic_rl.json &&
timeout -k 10 400 python3 bench.py > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 > $O/bench48_$T.json 2> $O/bench48_$T.err &&
timeout -k 10 500 python3 bench.py --workload rl --no-e2e > $O/bench_rl_$T.json 2> $O/bench_rl_$T.err &&
timeout -k 10 400 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-graph > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-ingest > $O/bench_torchrun1_$T.json 2> $O/bench_torchrun1_$T.err
