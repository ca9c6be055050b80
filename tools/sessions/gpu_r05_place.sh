# Placement experiment: k_gal_reg timing with padding between the state slots (KB_PAD) and in front of z / zin
# (KB_ZPAD), 2 interleaved rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-place}
cd $R && for round in 1 2; do for cfg in "0 0" "4096 0" "65536 0" "2101248 0" "12288 8192" "262144 131072"; do
  set -- $cfg
  echo "=== pad $1 zpad $2 round $round" >> $O/place_$T.txt
  KB_REV=1 KB_PAD=$1 KB_ZPAD=$2 timeout -k 10 120 tools/bin/kbench_reg 4096 20 2>&1 | grep -E "k_gal_reg<|FAIL" >> $O/place_$T.txt || exit 1
done; done
