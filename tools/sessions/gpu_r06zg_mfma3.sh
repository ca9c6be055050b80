# SubNet layer 3 on the matrix cores (GD_SN_MFMA3) vs base, interleaved on one box; fingerprints must match
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06zg; mkdir -p $O
for rd in 1 2 3; do
  for v in ${VARIANTS:-base mfma3}; do
    timeout -k 10 60 ./variants/kbs_$v 256 48 200 > $O/kbs_${v}_$rd.txt 2>&1 || exit 1
    timeout -k 10 60 ./variants/ksn_$v 4096 256 20 > $O/ksn_${v}_$rd.txt 2>&1 || exit 1
  done
done
for v in ${VARIANTS:-base mfma3}; do
  timeout -k 10 60 ./variants/ksnt_$v 4096 256 5 > $O/ksnt_$v.txt 2>&1 || exit 1
done
echo done
