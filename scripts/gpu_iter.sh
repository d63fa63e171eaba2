#!/bin/bash
# Iteration loop on the GPU box: optional parity subset (PARITY_K), then the c4 leg under a
# kernel trace with the per-round breakdown (rounds 5-24), optionally the C2 bench (C2=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/iter
mkdir -p $OUT
if [ -n "$PARITY_K" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_partition.py -x -q -p no:cacheprovider \
    --timeout 400 --timeout-method thread -k "$PARITY_K" > $OUT/parity.log 2>&1
  rc=$?; tail -3 $OUT/parity.log
  if [ $rc -ne 0 ]; then grep -m5 -A30 "Error\|assert" $OUT/parity.log | head -60; exit $rc; fi
fi
if [ "${C4:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --only-large --legs c4 > $OUT/c4.json 2>&1 || { tail -20 $OUT/c4.json; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"us_per_round": {[^}]*}\|"frac": [0-9.]*' $OUT/c4.json | head -3
  python3 scripts/round_breakdown.py $OUT/trace/run_kernel_trace.csv k_stats_final 5 25 | head -16
fi
if [ "${C2:-0}" = 1 ]; then
  timeout -k 10 300 python3 bench.py --no-large --no-cpu-baseline --no-steady > $OUT/c2.json 2>&1 || { tail -20 $OUT/c2.json; exit 1; }
  grep -o '"value": [0-9.e+]*\|"avg_launch_us": [0-9.]*\|"frac": [0-9.]*' $OUT/c2.json | head -3
fi
if [ "${PH:-0}" = 1 ]; then
  GS_PHASE_PROFILE=1 timeout -k 10 300 python3 bench.py --only-large --legs c4 > $OUT/c4ph.json 2>&1 || { tail -20 $OUT/c4ph.json; exit 1; }
  grep -o '"gather_phases_wg_ms": {[^}]*}' $OUT/c4ph.json
fi
