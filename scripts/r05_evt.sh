#!/bin/bash
# Round 5: the headline's per-launch timing events -- C2 driver window with the round
# kernel's events (default) and without (GS_PROFILE_ONLY=bfs), alternating, 3 runs each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05/${TAG:-evt}
mkdir -p $OUT
for i in 1 2 3; do
  for v in default bfs; do
    if [ $v = default ]; then E=""; else E="GS_PROFILE_ONLY=bfs"; fi
    env $E timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-large --no-steady > $OUT/${v}_$i.log 2>&1 || { tail -5 $OUT/${v}_$i.log; exit 1; }
    grep '"metric"' $OUT/${v}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $i, round(d['ms_per_step'],4), (d['roofline'] or {}).get('avg_launch_us'))"
  done
done
