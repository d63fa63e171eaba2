#!/bin/bash
# The full GPU test suite, then smoke().
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
  > $OUT/gpu_full.log 2>&1
rc=$?; tail -5 $OUT/gpu_full.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
