# k_rl_reg placement: x offset (KB_XPAD) and OTF offset (KB_OPAD) relative to y, 3 rounds (tag = $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; T=${1:-rlplace}
cd $R && for round in 1 2 3; do for cfg in "0 0" "131072 0" "0 131072" "131072 65536"; do
  set -- $cfg
  echo "=== xpad $1 opad $2 round $round" >> $O/place_$T.txt
  KB_XPAD=$1 KB_OPAD=$2 timeout -k 10 120 tools/bin/kbench_rl 4096 100 2 2>&1 | grep -E "^k_rl_reg|fnv" >> $O/place_$T.txt || exit 1
done; done
