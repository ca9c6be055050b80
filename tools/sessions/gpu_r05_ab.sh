# A/B of kbench variants, interleaved: bash gpu_r05_ab.sh TAG BIN1 BIN2 [BIN3 ...] (each tools/bin/<BIN> 4096 20, two rounds)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=$1; shift
cd $R && for round in 1 2; do for b in "$@"; do
  echo "=== $b round $round" >> $O/ab_$T.txt
  timeout -k 10 120 tools/bin/$b 4096 20 >> $O/ab_$T.txt 2>&1 || { echo "FAILED $b rc=$?" >> $O/ab_$T.txt; exit 1; }
done; done
