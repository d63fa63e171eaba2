#!/bin/bash
# Partition tests (small gloo/nccl, 1M gloo), MULTI parity subset, then the fused A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_partition.py -x -v -p no:cacheprovider --timeout 600 \
  --timeout-method thread > $OUT/part.log 2>&1
rc=$?; tail -8 $OUT/part.log
if [ $rc -ge 124 ]; then exit $rc; fi
PARITY_K="${PARITY_K:-4 or c4}" bash scripts/ab_fused.sh
