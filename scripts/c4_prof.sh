#!/bin/bash
# C4 leg under rocprofv3 kernel trace: per-kernel time per round (rounds 5-24) and the
# multi BFS's per-group level/entry/record counts (GS_MV_DIAG=1 in a second, untraced run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/c4prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --only-large --legs c4 > $OUT/c4.json 2>&1 || { tail -20 $OUT/c4.json; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"us_per_round": {[^}]*}' $OUT/c4.json | head -2
python3 scripts/round_breakdown.py $OUT/trace/run_kernel_trace.csv k_stats 5 25 | head -30
GS_MV_DIAG=1 timeout -k 10 200 python3 bench.py --only-large --legs c4 > $OUT/diag.log 2>&1 || exit 1
grep GS_MV_DIAG $OUT/diag.log | tail -4
