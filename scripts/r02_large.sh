#!/bin/bash
# Multi-source BFS check + profile: MULTI parity subset, then the bench's c4/c3 legs
# under rocprofv3 --kernel-trace, then a per-round breakdown of the c4 leg.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "${PARITY_K:-4 or multi or c4 or c3}" > $OUT/parity_large.log 2>&1
rc=$?; tail -3 $OUT/parity_large.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_large -o run -- \
  python3 bench.py --only-large --large-mode ${LARGE_MODE:-4} > $OUT/large.json 2>&1 || exit $?
tail -c 1800 $OUT/large.json; echo
python3 scripts/round_breakdown.py $OUT/prof_large/run_kernel_trace.csv ${ENDK:-k_mv_gather} 5 25
