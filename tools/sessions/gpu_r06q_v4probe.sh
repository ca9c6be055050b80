# k_gal_reg speed-of-light probe (tag = $1): 16-byte z / zin accesses with a wrong lane mapping (timing only)
# against the engine's kernel, alternating, 3 rounds, engine layout and galaxy-order alternation.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r06q}; mkdir -p $O
cd $R && for i in 1 2 3; do
  KB_REV=1 KB_LAYOUT=1 timeout -k 10 120 variants/kbench_reg 4096 20 noparity > $O/${T}_base_$i.txt 2>&1 || exit 1
  KB_REV=1 KB_LAYOUT=1 timeout -k 10 120 variants/kbench_reg_v4 4096 20 noparity > $O/${T}_v4_$i.txt 2>&1 || exit 1
done
