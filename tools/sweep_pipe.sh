#!/bin/bash
# Parity, then bench the spectral engine over pipeline streams x chunk MiB.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -m pytest tests -m gpu -q -rA > $O/gpu_tests.log 2>&1 || { echo "[sweep] parity failed" >&2; exit 1; }
for cfg in ${CFGS:-"2 96" "2 128" "2 160" "3 96" "3 128" "1 0"}; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --pipe-streams $1 --chunk-mb $2 > $O/pipe_$1_$2.json 2> $O/pipe_$1_$2.err || { echo "[sweep] bench failed at $cfg" >&2; exit 1; }
  echo "[sweep] $cfg done" >&2
done
