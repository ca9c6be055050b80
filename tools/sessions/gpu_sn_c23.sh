# SubNet batched kernel: layers 2-3 channel-split cap A/B, then the SubNet GPU tests.  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r02}; mkdir -p $O
for v in "" _c23 "" _c23; do echo "variant '$v'" >> $O/ksn23_$T.txt; timeout -k 10 60 $R/tools/kbench_subnet$v 4096 256 20 >> $O/ksn23_$T.txt 2>&1 || exit 1; done
cd $R && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "subnet or full or admm48 or configs" > $O/sn_tests_$T.log 2>&1
