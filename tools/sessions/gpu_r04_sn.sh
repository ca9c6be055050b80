# SubNet VALU (m0) vs MFMA layers 4-7 (m1) vs MFMA layers 0-7 (m2) A/B with bitwise fingerprints of features and
# rhos, + phase traces (tag $1)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04sn}; mkdir -p $O
for v in m0 m1 m2 m0 m1 m2; do echo "variant $v"; timeout -k 10 60 $R/tools/bin/ksn_$v 4096 256 20 || exit 1; done > $O/ksn_$T.txt 2>&1 &&
for v in m0t m1t m2t; do echo "trace $v"; timeout -k 10 60 $R/tools/bin/ksn_$v 4096 256 5 || exit 1; done >> $O/ksn_$T.txt 2>&1
