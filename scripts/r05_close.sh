#!/bin/bash
# Round 5 closing extras at the final hash: C2 origin shares (strong-scaling prediction),
# the default bench line (no flags), smoke(), and the two-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-close}
mkdir -p $OUT
for s in 3000 1500 750 375; do
  timeout -k 10 200 python3 bench.py --warmup 5 --steps 20 --slots $s --no-cpu-baseline --no-large --no-steady \
    > $OUT/c2_$s.log 2>&1 || { tail -5 $OUT/c2_$s.log; exit 1; }
  grep '"metric"' $OUT/c2_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', $s, round(d['ms_per_step'],4), d['roofline']['avg_launch_us'])"
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.log 2>&1 || { tail -5 $OUT/bench_default.log; exit 1; }
grep '"metric"' $OUT/bench_default.log | tail -1 | cut -c1-200
TAG=${TAG:-close} bash scripts/r05_mg.sh
