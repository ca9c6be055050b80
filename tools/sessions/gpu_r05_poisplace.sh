# Poisson two-pass state: gap between the slots (KB_PAD bytes), pass A / pass B timing, 2 rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-poisplace}
cd $R && for round in 1 2 3; do for p in 0 262144 393216; do
  echo "=== pad $p round $round" >> $O/place_$T.txt
  KB_PAD=$p timeout -k 10 120 tools/bin/kbench_pois 4096 20 >> $O/place_$T.txt 2>&1 || exit 1
done; done
