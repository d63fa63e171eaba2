#!/bin/bash
# Round 4: the full GPU test suite (-m gpu), then the driver's bench window, untraced.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04/${TAG:-check}
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TO:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 400 \
    --timeout-method thread ${TEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -4 $OUT/gpu_tests.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TO:-600} python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
  grep -h '"metric"' $OUT/bench.log | tail -1 > $OUT/bench.json
  cut -c1-2500 $OUT/bench.json
fi
