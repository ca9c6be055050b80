# Poisson pass A A/B: state prefetch across the column FFTs (GD_POIS_SPF 0 / 1, depth 2 / 1), 3 rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-poisspf}
cd $R && for round in 1 2 3; do for b in kbench_pois_s0 kbench_pois_s1 kbench_pois_s1d1; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  timeout -k 10 120 tools/bin/$b 4096 20 >> $O/ab_$T.txt 2>&1 || exit 1
done; done
