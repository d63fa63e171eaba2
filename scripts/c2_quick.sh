#!/bin/bash
# Round-kernel parity subset, then the C2 bench line (no large legs, no CPU baseline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "${PARITY_K:-c2 or fused or 1-}" > $OUT/parity_wg.log 2>&1
rc=$?; tail -3 $OUT/parity_wg.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --no-large --no-cpu-baseline ${BENCH_ARGS} > $OUT/c2_quick.json 2>&1 || exit $?
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|avg_launch_us": [0-9.]*' $OUT/c2_quick.json
