#!/bin/bash
# A/B of the C3 leg (two concurrent one-slot engines) across library builds: round-5 close,
# the first persistent-BFS commit, and the current tree. Prints each run's c3 line.
set -o pipefail
mkdir -p gpurun_out/r06/c3ab
for v in ${VARS:-variants/r5 variants/pb .}; do
  n=$(basename $v)
  (cd $v && timeout -k 10 300 python -u bench.py --only-large --legs c3 > $GRAFT_REPO_ROOT/gpurun_out/r06/c3ab/$n.log 2>&1) || { echo "fail $v"; exit 1; }
  python - gpurun_out/r06/c3ab/$n.log $n <<'P'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); c=d.get('c3') or d
        print(sys.argv[2], json.dumps({k:c.get(k) for k in ('ms_per_step','us_per_round')}), c.get('bfs_roofline',{}).get('avg_launch_us'))
P
done
# per-kernel stats of the C3 leg for the builds in PROF
for v in $PROF; do
  n=$(basename $v)
  (cd $v && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT/$v && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06/c3ab/prof_$n -o run -- python3 bench.py --only-large --legs c3 > $GRAFT_REPO_ROOT/gpurun_out/r06/c3ab/prof_$n.log 2>&1) || { echo "prof fail $v"; exit 1; }
done
