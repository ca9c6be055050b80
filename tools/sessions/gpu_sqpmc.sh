# SQ counters for the fused kernels (kbench_reg): issue / wait / LDS breakdown, one pass per counter set.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-sq}; BIN=${2:-tools/kbench_reg}
cd /tmp && (rocprofv3 -L > $O/counters_list.txt 2>&1 || true) &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "k_gal_reg" -d $O/sq1_$T -o p --output-format csv -- $R/$BIN 4096 3 > $O/sq1_$T.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "k_gal_reg" -d $O/sq2_$T -o p --output-format csv -- $R/$BIN 4096 3 > $O/sq2_$T.log 2>&1
