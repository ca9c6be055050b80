# k_rl_reg: time + phase trace (kbench_rl), SQ counters, HBM traffic (FETCH / WRITE passes).  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-rl}
timeout -k 10 120 $R/tools/kbench_rl 4096 100 2 > $O/krl_$T.txt 2>&1 &&
timeout -k 10 120 $R/tools/kbench_rl_trace 4096 100 1 > $O/krltr_$T.txt 2>&1 &&
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "k_rl_reg" -d $O/rsq1_$T -o p --output-format csv -- $R/tools/kbench_rl 4096 20 1 > $O/rsq1_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "k_rl_reg" -d $O/rsq2_$T -o p --output-format csv -- $R/tools/kbench_rl 4096 20 1 > $O/rsq2_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_rl_reg" -d $O/rf_$T -o p --output-format csv -- $R/tools/kbench_rl 4096 20 1 > $O/rf_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rl_reg" -d $O/rw_$T -o p --output-format csv -- $R/tools/kbench_rl 4096 20 1 > $O/rw_$T.log 2>&1
