# SubNet conv input-channel unroll A/B (kbench_subnet variants).  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r02}; mkdir -p $O
for v in "" _px4 _q4 _px8q4 ""; do echo "variant '$v'" >> $O/ksnu_$T.txt; timeout -k 10 60 $R/tools/kbench_subnet$v 4096 256 20 >> $O/ksnu_$T.txt 2>&1 || exit 1; done
