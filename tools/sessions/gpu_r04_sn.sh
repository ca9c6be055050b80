# SubNet kernel A/B (tools/bin/ksn_<v>, variants $2, traces $3) with bitwise fingerprints of features and rhos ($1 tag)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04sn}; mkdir -p $O
for v in $2; do echo "variant $v"; timeout -k 10 60 $R/tools/bin/ksn_$v 4096 256 20 || exit 1; done > $O/ksn_$T.txt 2>&1 &&
for v in $3; do echo "trace $v"; timeout -k 10 60 $R/tools/bin/ksn_$v 4096 256 5 || exit 1; done >> $O/ksn_$T.txt 2>&1
