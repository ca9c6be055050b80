# Round-3 session g: SubNet layers 4-7 weights from LDS (A/B), phase trace
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-g}; mkdir -p $O
cd $R && for v in "" _nowlds "" _nowlds; do echo "variant '$v'" >> $O/ksn_$T.txt; timeout -k 10 60 tools/kbench_subnet$v 4096 256 20 >> $O/ksn_$T.txt 2>&1 || exit 1; done &&
timeout -k 10 60 tools/kbench_subnet_trace 4096 256 5 >> $O/ksn_$T.txt 2>&1
