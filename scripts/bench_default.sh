#!/bin/bash
# The driver's default bench line (python bench.py), under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/default
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep -h '"metric"' $OUT/bench.log | tail -1 > $OUT/bench.json
cut -c1-3000 $OUT/bench.json
