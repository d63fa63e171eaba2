#!/bin/bash
# Round 3: the driver's bench window at HEAD (untraced), one JSON line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-base}
mkdir -p $OUT
timeout -k 10 ${BENCH_TO:-600} python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
grep -h '"metric"' $OUT/bench.log | tail -1 > $OUT/bench.json
cut -c1-3000 $OUT/bench.json
