# final tree: the default bench line once more (another box) and the self-spawned 2-rank gloo rehearsal of the
# distributed path on one GPU
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zl; mkdir -p $O
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
GD_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-e2e --no-ingest --no-graph --cpu-seconds 3 --cpu-sample 8 > $O/bench_g2gloo.json 2> $O/bench_g2gloo.err
