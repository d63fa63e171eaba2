#!/bin/bash
# Round 6 iteration: (optional) selected GPU tests, then bench legs under env variants.
#   TAG=...  TESTS="..."  LEGS=c4  VARIANTS="GS_MV_PERSIST=0;GS_MV_PERSIST=1"  BENCH_ARGS=...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/${TAG:-iter}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TO:-600} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -4 $OUT/gpu_tests.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; exit $rc; fi
fi
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-}"
for v in "${VS[@]}"; do
  i=$((i+1))
  echo "== variant $i: $v"
  env $v timeout -k 10 ${LEG_TO:-300} python3 bench.py --only-large --legs ${LEGS:-c4} ${BENCH_ARGS:-} > $OUT/leg_$i.log 2>&1 \
    || { tail -20 $OUT/leg_$i.log; exit 1; }
  tail -1 $OUT/leg_$i.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
for k,v in d.items():
    print(k, round(v['ms_per_step'],3), v.get('us_per_round'), (v.get('bfs_roofline') or {}).get('frac'))"
done
if [ -n "${TRACE:-}" ]; then  # TRACE="ENV=..": one traced run of the legs, round ROUND's dispatch sequence
  echo "== trace: $TRACE"
  env $TRACE timeout -k 10 ${LEG_TO:-300} rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --only-large --legs ${LEGS:-c4} ${BENCH_ARGS:-} > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
  python3 scripts/round_seq.py $OUT/trace/run_kernel_trace.csv ${MARK:-k_mv_gather} ${ROUND:-12} > $OUT/round_seq.txt
  cat $OUT/round_seq.txt
fi
