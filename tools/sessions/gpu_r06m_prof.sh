# Round-6 profile set for the kernels below their targets (tag = $1): k_rl_reg time + phase trace + SQ counters;
# configs[1] (256 x 48^2) SQ counters through bench.py and the graph timeline of one replayed forward.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r06m}; mkdir -p $O
B48="python3 $R/bench.py --size 48 --batch 256 --steps 1 --warmup 1 --settle-s 0 --blocks 1 --no-cpu-baseline --no-e2e --no-graph --no-ingest --no-extra"
cd $R && timeout -k 10 120 variants/kbench_rl 4096 100 2 > $O/krl_$T.txt 2>&1 &&
timeout -k 10 120 variants/kbench_rl_trace 4096 100 1 > $O/krltr_$T.txt 2>&1 &&
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "k_rl_reg" -d $O/rsq1_$T -o p --output-format csv -- $R/variants/kbench_rl 4096 20 1 > $O/rsq1_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "k_rl_reg" -d $O/rsq2_$T -o p --output-format csv -- $R/variants/kbench_rl 4096 20 1 > $O/rsq2_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "gd::" -d $O/sq1_48$T -o p --output-format csv -- $B48 > $O/sq1_48$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "gd::" -d $O/sq2_48$T -o p --output-format csv -- $B48 > $O/sq2_48$T.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/gt48_$T -o run --output-format csv -- python3 $R/tools/graph_trace.py 20 256 48 > $O/gt48_$T.txt 2>&1 &&
cd $R && python3 tools/sq_summary.py $O/rsq1_$T/p_counter_collection.csv $O/rsq2_$T/p_counter_collection.csv > $O/rsq_summary_$T.txt 2>&1 &&
python3 tools/sq_summary.py $O/sq1_48$T/p_counter_collection.csv $O/sq2_48$T/p_counter_collection.csv > $O/sq48_summary_$T.txt 2>&1 &&
python3 tools/graph_timeline.py $O/gt48_$T/run_kernel_trace.csv 0 10 >> $O/gt48_$T.txt 2>&1
