R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-r05rev}
cd $R && for round in 1 2 3; do for rv in 0 1; do
  echo "=== KB_REV=$rv round $round" >> $O/ab_$T.txt
  KB_REV=$rv timeout -k 10 120 tools/bin/kbench_reg_rev 4096 20 >> $O/ab_$T.txt 2>&1 || exit 1
done; done
