#!/bin/bash
# One GPU session: parity tests, PMC traffic of the round kernel, bench, rocprof
# kernel-trace summary. Every GPU step has its own time limit; a fault/abort/timeout
# (exit >= 124 or signals) ends the script, an ordinary test failure (exit 1) does not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND_DIR=${ROUND_DIR:-profiles/r01}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|GPU fault|HSA_STATUS_ERROR" "gpurun_out/$name.log"; then
    echo "stopping after $name: GPU fault signature in the log"; exit 99
  fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
  # HBM traffic of the round kernel over the bench's own default timed steps (separate passes)
  BENCH_ARGS="--steps 100 --warmup 20 --no-cpu-baseline --no-profile --no-large" bash scripts/pmc.sh fetch:FETCH_SIZE write:WRITE_SIZE || exit $?
  python3 scripts/pmc_summary.py --kernel k_round_wg --launches 100 --bench-args "--steps 100 --warmup 20" \
    --out gpurun_out/pmc_k_round_wg_3000x3000.json && mkdir -p $ROUND_DIR && \
    cp gpurun_out/pmc_k_round_wg_3000x3000.json $ROUND_DIR/
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py
  tail -1 gpurun_out/bench.log > gpurun_out/bench.json
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline
  python3 scripts/launch_times.py gpurun_out/prof k_round_wg
fi
