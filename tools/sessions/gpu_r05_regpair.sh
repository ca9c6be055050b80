# k_gal_reg A/B: paired column transforms (GD_REG_PAIR 0 / 1 / 2 / 3), 3 interleaved rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-regpair}
cd $R && for round in 1 2 3; do for b in kbench_reg_rp0 kbench_reg_rp1 kbench_reg_rp2 kbench_reg_rp3; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  KB_REV=1 timeout -k 10 120 tools/bin/$b 4096 20 >> $O/ab_$T.txt 2>&1 || exit 1
done; done
