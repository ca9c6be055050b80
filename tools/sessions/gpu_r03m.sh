# Workgroup placement probe and the fused init + SubNet block maps (256 x 48^2).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; export TMPDIR=/tmp; T=${1:-r03m}
cd $R && mkdir -p $O &&
timeout -k 10 60 tools/kbenchsm0 256 48 400 1 > $O/ksmall_$T.txt 2>&1 &&
timeout -k 10 60 tools/kbenchsm0 256 48 400 >> $O/ksmall_$T.txt 2>&1
