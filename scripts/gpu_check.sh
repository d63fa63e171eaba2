#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout (exit >= 124 or
# signals) ends the script, an ordinary test failure (exit 1) does not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
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
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline
  find gpurun_out/prof -name "*stats*" | head
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
  # HBM traffic of the round kernel over the bench's own default timed steps
  BENCH_ARGS="--steps 100 --warmup 20 --no-cpu-baseline --no-profile" bash scripts/pmc.sh fetch:FETCH_SIZE write:WRITE_SIZE || exit $?
  python3 scripts/pmc_summary.py --kernel k_round_wg --launches 100 --bench-args "--steps 100 --warmup 20" \
    --out gpurun_out/pmc_k_round_wg_3000x3000.json
fi
