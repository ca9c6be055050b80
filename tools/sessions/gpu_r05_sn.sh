# SubNet kernels (kbench_subnet: batched k_subnet_features_psf at 4096, one-launch k_subnet_rhos_psf at 256): time,
# phase trace and SQ counters incl. LDS bank conflicts (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r05sn}; mkdir -p $O
cd $R && timeout -k 10 120 tools/bin/kbench_subnet 4096 256 20 > $O/ksn_$T.txt 2>&1 &&
timeout -k 10 120 tools/bin/kbench_subnet_trace 4096 256 5 > $O/ksntr_$T.txt 2>&1 &&
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "subnet" -d $O/snsq1_$T -o p --output-format csv -- $R/tools/bin/kbench_subnet 4096 256 3 > $O/snsq1_$T.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --kernel-include-regex "subnet" -d $O/snsq2_$T -o p --output-format csv -- $R/tools/bin/kbench_subnet 4096 256 3 > $O/snsq2_$T.log 2>&1 &&
cd $R && python3 tools/sq_summary.py $O/snsq1_$T/p_counter_collection.csv $O/snsq2_$T/p_counter_collection.csv > $O/snsq_summary_$T.txt 2>&1
