# k_gal_reg_init A/B: paired line FFTs (GD_INIT_PAIR 0 / 1 / 2 / 3), 3 interleaved rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-initpair}
cd $R && for round in 1 2 3; do for b in kbench_reg_ip0 kbench_reg_ip1 kbench_reg_ip2 kbench_reg_ip3; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  KB_REV=1 timeout -k 10 120 tools/bin/$b 4096 20 >> $O/ab_$T.txt 2>&1 || exit 1
done; done
