# fused-kernel iteration loop: phase trace microbenchmark, Gaussian parity subset, bench (fused vs three-kernel)
timeout -k 10 120 ./tools/kbench_fused > gpurun_out/kbf.txt 2>&1 || exit 1
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x -k "admm or fused or full_batch or pipelined" > gpurun_out/gpu_tests.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e --fused 1 > gpurun_out/bench_f1.json 2>gpurun_out/bench_f1.err
