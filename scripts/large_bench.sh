#!/bin/bash
# Large-N propagation: 100k x 16 slots and 1M x 8 slots, level (2) vs binned (3) BFS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "100000 16" "1000000 8"; do
  set -- $cfg
  for m in ${MODES:-2 3}; do
    timeout -k 10 400 python bench.py --nodes $1 --slots $2 --steps ${STEPS:-20} --warmup 5 --bfs-mode $m --no-cpu-baseline \
      > gpurun_out/large_$1_$m.log 2>&1 || { echo "n=$1 mode=$m failed"; tail -20 gpurun_out/large_$1_$m.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/large_$1_$m.log').read().strip().splitlines()[-1]); r=d['roofline']
print('n=$1 S=$2 mode=$m', 'ms/step %.3f'%d['ms_per_step'], 'edges/s %.3e'%d['value'], r['kernel'], 'bfs us/round %s'%r['avg_launch_us'], 'frac %s'%r['frac'])"
  done
done
