# k_rl_reg at engine r06.2: time and SQ counters (the r06m passes), for the Nyquist-column change's wait cycles
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06zm; mkdir -p $O; export TMPDIR=/tmp
cd $R && timeout -k 10 120 tools/sq/kbench_rl 4096 100 2 > $O/krl.txt 2>&1 &&
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "k_rl_reg" -d $O/rsq1 -o p --output-format csv -- $R/tools/sq/kbench_rl 4096 20 1 > $O/rsq1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "k_rl_reg" -d $O/rsq2 -o p --output-format csv -- $R/tools/sq/kbench_rl 4096 20 1 > $O/rsq2.log 2>&1 &&
cd $R && python3 tools/sq_summary.py $(find $O/rsq1 $O/rsq2 -name "*counter_collection.csv") > $O/sq_rl.txt 2>&1
