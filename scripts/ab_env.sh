#!/bin/bash
# A/B of the c4 leg under two settings of one environment variable:
#   AB_VAR=NAME AB_A=value AB_B=value [PARITY_K=...] bash scripts/ab_env.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
if [ -n "$PARITY_K" ]; then
  timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_partition.py -x -q -p no:cacheprovider \
    --timeout 400 --timeout-method thread -k "$PARITY_K" > $OUT/parity_ab.log 2>&1
  rc=$?; tail -3 $OUT/parity_ab.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for val in "$AB_A" "$AB_B"; do
  env $AB_VAR="$val" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_env_${val:-0} -o run -- \
    python3 bench.py --only-large --legs c4 > $OUT/ab_env_${val:-0}.json 2>&1 || exit $?
  echo "== $AB_VAR=$val"; grep -o '"ms_per_step": [0-9.]*\|"us_per_round": {[^}]*}' $OUT/ab_env_${val:-0}.json | head -2
  python3 scripts/round_breakdown.py $OUT/prof_env_${val:-0}/run_kernel_trace.csv k_stats 5 25 | head -8
done
