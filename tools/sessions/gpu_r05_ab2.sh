# A/B of kbench variants with alternating galaxy order: bash gpu_r05_ab2.sh TAG BIN1 BIN2 ... (3 rounds)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=$1; shift
cd $R && for round in 1 2 3; do for b in "$@"; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  KB_REV=1 timeout -k 10 120 tools/bin/$b 4096 20 >> $O/ab_$T.txt 2>&1 || { echo "FAILED $b rc=$?" >> $O/ab_$T.txt; exit 1; }
done; done
