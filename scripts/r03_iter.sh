#!/bin/bash
# Round 3 iteration on the GPU box: an optional pytest subset (TESTS="file::test ..." or
# K="-k expr"), then optionally the c4 leg under a kernel trace with one round's dispatch
# sequence (C4=1), the C2 bench (C2=1), or bench legs (LEGS=c4,c5).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-iter}
mkdir -p $OUT
if [ -n "$TESTS$K" ]; then
  timeout -k 10 ${TEST_TO:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 600 \
    --timeout-method thread ${K:+-k "$K"} > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log
  if [ $rc -ne 0 ]; then grep -m5 -B2 -A30 "Error\|assert" $OUT/tests.log | head -80; exit $rc; fi
fi
if [ "${C4:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --only-large --legs c4 > $OUT/c4.json 2>&1 || { tail -20 $OUT/c4.json; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"us_per_round": {[^}]*}\|"frac": [0-9.]*' $OUT/c4.json | head -3
  python3 scripts/round_seq.py $OUT/trace/run_kernel_trace.csv ${MARK:-k_stats_final} ${ROUND:-12} > $OUT/c4_round.txt
  tail -3 $OUT/c4_round.txt
fi
if [ -n "$LEGS" ]; then
  timeout -k 10 ${LEG_TO:-600} python3 bench.py --only-large --legs $LEGS > $OUT/legs.json 2>&1 || { tail -20 $OUT/legs.json; exit 1; }
  cut -c1-3000 $OUT/legs.json
fi
if [ "${C2:-0}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --no-large --no-cpu-baseline ${C2_ARGS:---steps 20 --warmup 5} > $OUT/c2.json 2>&1 || { tail -20 $OUT/c2.json; exit 1; }
  grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' $OUT/c2.json | head -4
fi
