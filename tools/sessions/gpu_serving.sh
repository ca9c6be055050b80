timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "serving or full_model" > gpurun_out/gpu_serving.log 2>&1 || { tail -40 gpurun_out/gpu_serving.log; exit 1; }
tail -3 gpurun_out/gpu_serving.log
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --no-cpu-baseline > gpurun_out/bench48.json 2> gpurun_out/bench48.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench256.json 2> gpurun_out/bench256.err || exit 1
