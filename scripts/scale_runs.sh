#!/bin/bash
# Larger SURVEY 8(d) shapes on one GPU: C3-shaped 100k x 16 slots, C4-shaped 1M x 8
# (rocprofv3 kernel stats), C5-scale 10M nodes x 2 slots. Every step has its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <tag> <secs> <bench args...>
  local tag=$1 secs=$2; shift 2
  timeout -k 10 "$secs" python3 bench.py --no-cpu-baseline --no-large "$@" > "gpurun_out/scale_$tag.log" 2>&1 \
    || { echo "$tag failed rc=$?"; tail -5 "gpurun_out/scale_$tag.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/scale_$tag.log').read().strip().splitlines()[-1]); r=d['roofline'] or {}
print('$tag', 'ms/step %.3f' % d['ms_per_step'], 'edges/s %.3e' % d['value'], 'bfs_us/round', r.get('avg_launch_us'), 'frac', r.get('frac'))"
}
run c3_100k_x16 300 --nodes 100000 --slots 16 --steps 40 --warmup 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1m -o run -- \
  python3 bench.py --nodes 1000000 --slots 8 --steps 20 --warmup 5 --no-cpu-baseline --no-large > gpurun_out/scale_c4_1m_x8.log 2>&1 \
  || { echo "1M profile failed"; tail -5 gpurun_out/scale_c4_1m_x8.log; exit 1; }
tail -1 gpurun_out/scale_c4_1m_x8.log | cut -c1-400
run c5_10m_x2 600 --nodes 10000000 --slots 2 --steps 6 --warmup 2
