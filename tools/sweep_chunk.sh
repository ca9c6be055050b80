#!/bin/bash
# Parity, then bench the spectral engine at several Infinity-Cache chunk sizes (MiB).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 600 python3 -m pytest tests -m gpu -q -rA > $O/gpu_tests.log 2>&1 || { echo "[sweep] parity failed" >&2; exit 1; }
for mb in ${CHUNKS:-0 32 64 96 128 192}; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --chunk-mb $mb > $O/sweep_$mb.json 2> $O/sweep_$mb.err || { echo "[sweep] bench failed at $mb" >&2; exit 1; }
  echo "[sweep] chunk=$mb done" >&2
done
