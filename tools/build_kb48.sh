# Build the 48^2 SubNet / init kernel-bench variants into variants/ (kbench_small: init + SubNet launch and the
# graphed forward; kbench_subnet: the SubNet kernels, plus a phase-trace build).  usage: bash tools/build_kb48.sh [name] ["-DFLAG=1 ..."]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
F="--offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result"
build() {  # name, flags
  /opt/rocm/bin/hipcc $F $2 -o $R/variants/kbs_$1 $R/tools/kbench_small.hip 2>/dev/null &&
  /opt/rocm/bin/hipcc $F $2 -o $R/variants/ksn_$1 $R/tools/kbench_subnet.hip 2>/dev/null &&
  /opt/rocm/bin/hipcc $F $2 -DGD_SN_TRACE=1 -o $R/variants/ksnt_$1 $R/tools/kbench_subnet.hip 2>/dev/null &&
  echo "built $1"
}
# round 6 (profiles/r06s_subnet48_variants_ab.txt) built base plus -DGD_SN_WPIPE=1, -DGD_SN_WPF=1,
# "-DGD_SN_PSFLD=1 -DGD_SI_YLD=1" and all three from a patched tree; none was kept
build ${1:-base} "${2:-}"

