#!/bin/bash
# Round 5: one-GPU timings of the per-rank shares behind DESIGN.md section 7's multi-GPU
# predictions (every row unmeasured on more than one GPU):
#   C2 strong: 1,500 / 750 / 375 origins of the one trial (--slots; driver window);
#   C4 sweep sharding over 8 ranks: the 2-sim share (sims 0 and 8) and a 1-sim share;
#   C5 origin sharding over 8 ranks: 2 origin slots of the 10M-node graph.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-shares}
mkdir -p $OUT
for s in 3000 1500 750 375; do
  echo "== c2 slots $s"
  timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --slots $s --no-cpu-baseline --no-large --no-steady \
    > $OUT/c2_$s.log 2>&1 || { tail -5 $OUT/c2_$s.log; exit 1; }
  grep '"metric"' $OUT/c2_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', $s, round(d['ms_per_step'],4), d['roofline']['avg_launch_us'])"
done
for sims in "0,1,2,3,4,5,6,7,8,9,10,11,12" "0,8" "5"; do
  echo "== c4 sims $sims"
  timeout -k 10 200 python3 bench.py --only-large --legs c4 --c4-sims $sims > $OUT/c4_$sims.log 2>&1 || { tail -5 $OUT/c4_$sims.log; exit 1; }
  tail -1 $OUT/c4_$sims.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['c4']; print('c4', '$sims', round(d['ms_per_step'],4), d['us_per_round'])"
done
for sl in 16 2; do
  echo "== c5 slots $sl"
  timeout -k 10 300 python3 bench.py --only-large --legs c5 --c5-slots $sl > $OUT/c5_$sl.log 2>&1 || { tail -5 $OUT/c5_$sl.log; exit 1; }
  tail -1 $OUT/c5_$sl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['c5']; print('c5', $sl, round(d['ms_per_step'],4), d['us_per_round'])"
done
echo "== c3 leg (2 one-slot engines: active-set sizes 12 and 20)"
timeout -k 10 200 python3 bench.py --only-large --legs c3 > $OUT/c3_leg.log 2>&1 || { tail -5 $OUT/c3_leg.log; exit 1; }
tail -1 $OUT/c3_leg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['c3']; print('c3 leg', round(d['ms_per_step'],4), d['bfs_mode'])"
echo "== c3 workload, all 16 sims on one GPU"
timeout -k 10 300 python3 bench.py --workload c3 --warmup 5 --steps 20 > $OUT/c3_w16.log 2>&1 || { tail -5 $OUT/c3_w16.log; exit 1; }
grep '"metric"' $OUT/c3_w16.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 16 sims', round(d['ms_per_step'],4))"
