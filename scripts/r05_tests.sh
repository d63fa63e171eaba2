#!/bin/bash
# Round 5: run selected GPU tests (TESTS="node ids"), then optional bench legs (LEGS, VARIANTS as r05_iter.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-tests}
mkdir -p $OUT
timeout -k 10 ${TEST_TO:-900} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout ${PER_TEST_TO:-300} \
  --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/gpu_tests.log | tail -40
if [ $rc -ne 0 ]; then grep -E "Error|error|assert" $OUT/gpu_tests.log | head -30; exit $rc; fi
