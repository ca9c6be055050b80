# r05 session A: streaming ceilings (rewritten kbench_stream), k_gal_reg timing + phase trace, SQ counters.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; T=${1:-r05a}
cd $R &&
timeout -k 10 240 tools/bin/kbench_stream 4096 20 > $O/kstream_$T.txt 2>&1 &&
timeout -k 10 100 tools/bin/kbench_reg 4096 20 > $O/kreg_$T.txt 2>&1 &&
timeout -k 10 100 tools/bin/kbench_reg_trace 4096 10 > $O/kregtr_$T.txt 2>&1 &&
bash tools/sessions/gpu_sqpmc.sh $T tools/bin/kbench_reg
