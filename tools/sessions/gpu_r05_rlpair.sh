# k_rl_reg A/B: paired line FFTs (GD_RL_PAIR 0 / 1 / 3 / 7), 3 interleaved rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-rlpair}
cd $R && for round in 1 2 3; do for b in kbench_rl_p0 kbench_rl_p1 kbench_rl_p3 kbench_rl_p7; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  timeout -k 10 120 tools/bin/$b 4096 100 2 >> $O/ab_$T.txt 2>&1 || exit 1
done; done
