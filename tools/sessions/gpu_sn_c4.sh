# SubNet batched kernel: layer-4 channel-split cap A/B.  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r02}; mkdir -p $O
for v in "" _c4 "" _c4; do echo "variant '$v'" >> $O/ksn4_$T.txt; timeout -k 10 60 $R/tools/kbench_subnet$v 4096 256 20 >> $O/ksn4_$T.txt 2>&1 || exit 1; done
