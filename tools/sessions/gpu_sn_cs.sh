# SubNet output-channel split caps for layers 5 / 6-7 (kbench_subnet variants).  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r02}; mkdir -p $O
for v in "" _c5 _c67 _c567 ""; do echo "variant '$v'" >> $O/ksnc_$T.txt; timeout -k 10 60 $R/tools/kbench_subnet$v 4096 256 20 >> $O/ksnc_$T.txt 2>&1 || exit 1; done
