set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
for rd in 1 2; do
for v in old new; do
  timeout -k 10 60 ./variants/kbsn_$v 4096 256 20 > gpurun_out/r06c/kbsn_${v}_$rd.txt 2>&1 || exit 1
done; done
for v in oldt newt; do
  timeout -k 10 60 ./variants/kbsn_$v 4096 256 20 > gpurun_out/r06c/kbsn_${v}.txt 2>&1 || exit 1
done
for v in old new; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/r06c/pmc_$v -o sq --output-format csv -- ./variants/kbsn_$v 4096 256 2 > gpurun_out/r06c/pmc_$v.log 2>&1 || exit 1
done
