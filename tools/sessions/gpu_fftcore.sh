# FFT-core change check: GPU parity tests, kernel bench + phase trace, bench lines (256^2 default, RL, Poisson, 48^2).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-fc}
cd $R && GD_PARITY_LOG=$O/parity_$T.jsonl timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/gpu_tests_$T.log 2>&1 &&
timeout -k 10 100 tools/kbench_reg 4096 20 > $O/kreg_$T.txt 2>&1 &&
timeout -k 10 100 tools/kbench_reg_trace 4096 10 > $O/kregtr_$T.txt 2>&1 &&
timeout -k 10 400 python3 bench.py --no-e2e --no-ingest > $O/bench_$T.json 2> $O/bench_$T.err &&
timeout -k 10 500 python3 bench.py --workload rl --no-e2e --no-ingest --no-graph --no-cpu-baseline > $O/bench_rl_$T.json 2> $O/bench_rl_$T.err &&
timeout -k 10 400 python3 bench.py --llh Poisson --no-e2e --no-ingest --no-graph --no-cpu-baseline > $O/bench_poisson_$T.json 2> $O/bench_poisson_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48_$T.json 2> $O/bench48_$T.err
