# SubNet conv A/B: tap-major weights + 2x2 blocks (kbench_subnet) vs tap-major per pixel (kbench_subnet_q0), trace; SubNet GPU tests.  tag = $1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r02}; mkdir -p $O
timeout -k 10 60 $R/tools/kbench_subnet 4096 256 20 > $O/ksn_$T.txt 2>&1 &&
timeout -k 10 60 $R/tools/kbench_subnet_q0 4096 256 20 >> $O/ksn_$T.txt 2>&1 &&
timeout -k 10 60 $R/tools/kbench_subnet_trace 4096 256 5 >> $O/ksn_$T.txt 2>&1 &&
cd $R && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread -k "subnet or full or admm48 or configs" > $O/sn_tests_$T.log 2>&1
