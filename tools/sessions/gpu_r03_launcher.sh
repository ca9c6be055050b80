# Driver-form launcher rehearsal on the 1-GPU box (tag = $1): torch.distributed.run N = 1 over RCCL (the
# driver's scaling command), and `bench.py --gpus 2` without a launcher on one GPU (must exit != 0: RCCL
# would get fewer GPUs than ranks).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03launch}; mkdir -p $O
cd $R && timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 > $O/launch_n1_$T.json 2> $O/launch_n1_$T.err &&
{ timeout -k 10 200 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-e2e --no-ingest --no-cpu-baseline > $O/launch_g2_$T.json 2> $O/launch_g2_$T.err; echo "bench.py --gpus 2 on one GPU: exit $?" > $O/launch_g2_$T.rc; }
