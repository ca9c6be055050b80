# SubNet kernels: time + phase trace (kbench_subnet).  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r02}; mkdir -p $O
timeout -k 10 60 $R/tools/kbench_subnet 4096 256 20 > $O/ksn_$T.txt 2>&1 &&
timeout -k 10 60 $R/tools/kbench_subnet_trace 4096 256 5 >> $O/ksn_$T.txt 2>&1
