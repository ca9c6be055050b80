# Interleaved A/B of prebuilt engine variants (variants/<name>.so swapped in for libgdeconv.so) on one box:
#   bash tools/ab_variants.sh OUT_PREFIX ROUNDS "v1 v2 ..." [bench configs separated by ';']
# Each round runs every variant under every config (default: configs[2] Gaussian, the Poisson 256^2 line, RL(100)),
# so the variants alternate in one clock window; one JSON summary line per (round, variant, config) on stdout and
# the full bench records in gpurun_out/<OUT_PREFIX>_<round>_<variant>_<i>.json.  The original library is restored.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$1; ROUNDS=$2; VARS=$3
CFGS=${4:-"--steps 20 --warmup 3;--steps 20 --warmup 3 --llh Poisson;--workload rl --steps 5 --warmup 1"}
LIB=$R/galaxy-deconv_amd/gdeconv/libgdeconv.so
cp $LIB /tmp/ab_orig.so
mkdir -p $R/gpurun_out
rc=0
for rd in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    cp $R/variants/$v.so $LIB
    i=0
    IFS=';' read -ra CA <<< "$CFGS"
    for cfg in "${CA[@]}"; do
      f=$R/gpurun_out/${OUT}_${rd}_${v}_${i}.json
      timeout -k 10 240 python3 $R/bench.py $cfg --no-cpu-baseline --no-e2e --no-graph --no-ingest --no-extra > $f 2> $f.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "FAIL rc=$rc $v $cfg"; tail -5 $f.err; cp /tmp/ab_orig.so $LIB; exit $rc; fi
      python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('round $rd | $v | $cfg |', round(d['value']), d['blocks']['eager_ms_per_step'], {k: round(x['avg_ms'], 4) for k, x in d['kernels'].items()})"
      i=$((i+1))
    done
  done
done
cp /tmp/ab_orig.so $LIB
