# SQ counters of the configs[1] kernels (256 x 48^2: k_gal_small_t<48>, k_subnet_rhos_init<48>) in two passes of
# 8 SQ counters each (tag = $1), through bench.py --steps 1 --warmup 1 --no-graph.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-sq48}; mkdir -p $O
B="python3 $R/bench.py --size 48 --batch 256 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest"
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "gd::" -d $O/sq1_$T -o p --output-format csv -- $B > $O/sq1_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "gd::" -d $O/sq2_$T -o p --output-format csv -- $B > $O/sq2_$T.log 2>&1
