# k_rl_reg: stored OTF vs OTF built in the kernel (COTF), timing + output comparison, tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-rl}
cd $R && timeout -k 10 200 tools/bin/kbench_rl 4096 100 2 > $O/kbrl_$T.txt 2>&1 &&
timeout -k 10 100 tools/bin/kbench_rl 256 100 3 >> $O/kbrl_$T.txt 2>&1
