# k_rl_reg: line 0 forms the Nyquist column's products itself (GD_RL_NYQL) vs base, interleaved, 4096 x RL(100)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zj; mkdir -p $O
for rd in 1 2 3; do
  for v in base nyql; do
    timeout -k 10 120 ./variants/krl_$v 4096 100 3 > $O/krl_${v}_$rd.txt 2>&1 || exit 1
  done
done
echo done
