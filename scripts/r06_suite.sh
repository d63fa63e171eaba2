#!/bin/bash
# Round 6: the whole -m gpu suite (durations), log under gpurun_out/r06/suite_$TAG.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/suite_${TAG:-a}
mkdir -p $OUT
timeout -k 10 ${TEST_TO:-1080} python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 900 \
  --timeout-method thread --durations=40 ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $OUT/gpu_tests.log | tail -3
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $OUT/gpu_tests.log | head -30; fi
exit $rc
