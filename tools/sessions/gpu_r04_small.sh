# 48^2 engine microbenchmarks (tag $1, variants $2): iteration, graphed forward, SubNet + init one launch, phase trace
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; T=${1:-r04small}; mkdir -p $O
for v in $2; do echo "variant $v"; timeout -k 10 60 $R/tools/bin/$v 256 48 200 || exit 1; done > $O/ksmall_$T.txt 2>&1
