# End-of-workgroup store drain + barrier (GD_REG_DRAIN 1 = before) vs none (0): k_gal_reg / init and Poisson pass A,
# 3 interleaved rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-drain}
cd $R && for round in 1 2 3; do for b in kbench_reg_dr1 kbench_reg_dr0 kbench_pois_dr1 kbench_pois_dr0; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  KB_REV=1 timeout -k 10 120 tools/bin/$b 4096 20 >> $O/ab_$T.txt 2>&1 || exit 1
done; done
