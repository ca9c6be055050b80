# Round-3 session f: SubNet W1 prefetch A/B, phase trace, SQ counters of the one-round kernel
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-f}; mkdir -p $O
cd $R && for v in "" _nopf ""; do echo "variant '$v'" >> $O/ksn_$T.txt; timeout -k 10 60 tools/kbench_subnet$v 4096 256 20 >> $O/ksn_$T.txt 2>&1 || exit 1; done &&
timeout -k 10 60 tools/kbench_subnet_trace 4096 256 5 >> $O/ksn_$T.txt 2>&1 &&
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $O/rocprof_counters_$T.txt 2>&1 ; cd /tmp &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --kernel-trace --stats -d $O/pmc_sn_$T -o sn -- $R/tools/kbench_subnet 256 256 5 > $O/pmc_sn_$T.log 2>&1
