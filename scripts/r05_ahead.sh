#!/bin/bash
# Round 5: rotation ahead of the fused round -- C2 shares with it (default) and without
# (GS_ROT_AHEAD=0), driver window, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r05/${TAG:-ahead}
mkdir -p $OUT
for s in 3000 375; do
  for v in on off on off; do
    if [ $v = on ]; then E=""; else E="GS_ROT_AHEAD=0"; fi
    env $E timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --slots $s --no-cpu-baseline --no-large --no-steady > $OUT/${v}_$s.log 2>&1 || { tail -5 $OUT/${v}_$s.log; exit 1; }
    grep '"metric"' $OUT/${v}_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $s, round(d['ms_per_step'],4), (d['roofline'] or {}).get('avg_launch_us'))"
  done
done
