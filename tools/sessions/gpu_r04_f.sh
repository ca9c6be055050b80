# Round-4 final set (engine rev r04.6) (tag $1): gpu_r04_final.sh (all GPU tests, smoke, PMC passes, kernel stats
# at 256^2 and 48^2, the graphed 48^2 timeline, bench lines 256 / 48 / Poisson / RL), then the 160^2 and gloo
# 2-rank lines, plus 144 / 128 / 112 / 96 / 80^2.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04f}; mkdir -p $O
bash $R/tools/sessions/gpu_r04_final.sh $T &&
cd $R && timeout -k 10 300 python3 bench.py --size 160 --no-e2e --no-ingest > $O/bench160_$T.json 2> $O/bench160_$T.err &&
timeout -k 10 300 python3 bench.py --size 144 --no-e2e --no-ingest --no-cpu-baseline > $O/bench144_$T.json 2> $O/bench144_$T.err &&
timeout -k 10 300 python3 bench.py --size 112 --no-e2e --no-ingest --no-cpu-baseline > $O/bench112_$T.json 2> $O/bench112_$T.err &&
timeout -k 10 300 python3 bench.py --size 128 --no-e2e --no-ingest --no-cpu-baseline > $O/bench128_$T.json 2> $O/bench128_$T.err &&
timeout -k 10 300 python3 bench.py --size 96 --no-e2e --no-ingest --no-cpu-baseline > $O/bench96_$T.json 2> $O/bench96_$T.err &&
timeout -k 10 300 python3 bench.py --size 80 --no-e2e --no-ingest --no-cpu-baseline > $O/bench80_$T.json 2> $O/bench80_$T.err &&
timeout -k 10 300 python3 bench.py --size 48 --batch 256 --llh Poisson --steps 100 --warmup 10 --no-e2e --no-ingest --no-cpu-baseline > $O/bench48p_$T.json 2> $O/bench48p_$T.err &&
GD_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-e2e --no-ingest --no-graph --cpu-seconds 3 --cpu-sample 8 > $O/bench_g2gloo_$T.json 2> $O/bench_g2gloo_$T.err
