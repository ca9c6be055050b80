# Placement experiment 2: the engine's slot layout (KB_LAYOUT=1), z == zin (KB_ALIAS=1), slot padding KB_PAD and
# z offset KB_ZPAD (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-place3}
cd $R && for round in 1 2; do for cfg in "0 0" "131072 0" "262144 0" "524288 0" "262144 131072" "0 131072" "393216 0" "1048576 0"; do
  set -- $cfg
  echo "=== engine layout, z==zin, pad $1 zpad $2 round $round" >> $O/place_$T.txt
  KB_LAYOUT=1 KB_ALIAS=1 KB_REV=1 KB_PAD=$1 KB_ZPAD=$2 timeout -k 10 120 tools/bin/kbench_reg 4096 20 2>&1 | grep -E "k_gal_reg<|FAIL" >> $O/place_$T.txt || exit 1
done; done
