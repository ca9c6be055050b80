# register-transpose fused iteration (k_gal_iter2): phase traces of both variants, fused parity subset, bench
timeout -k 10 60 ./tools/kbench_fused 4096 1 > gpurun_out/kbf1.txt 2>&1 || exit 1
timeout -k 10 60 ./tools/kbench_fused 4096 2 > gpurun_out/kbf2.txt 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "admm256 or fused or full_batch" > gpurun_out/gpu_tests_iter2.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --fused 2 > gpurun_out/bench_f2.json 2>gpurun_out/bench_f2.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --fused 1 > gpurun_out/bench_f1.json 2>gpurun_out/bench_f1.err
