#!/bin/bash
# Round 6: selected GPU tests (TESTS, pytest -k expression K), then c4 legs (VARIANTS) as r06_iter.sh.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/${TAG:-quick}
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TO:-600} python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${K:+-k "$K"} > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -5 $OUT/gpu_tests.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error|assert" $OUT/gpu_tests.log | head -30; exit $rc; fi
fi
TESTS= TAG=${TAG:-quick} scripts/r06_iter.sh
