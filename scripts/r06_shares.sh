#!/bin/bash
# Round 6 closing: one-GPU shares of the multi-GPU configurations (what one rank of an
# N-GPU run does), full bench lines -> profiles/r06/shares/ (copied back via gpurun_out).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/${TAG:-shares}
mkdir -p $OUT
run() {  # run <name> <args...>
  local n=$1; shift
  echo "== $n: $*"
  timeout -k 10 ${TO:-400} python3 bench.py "$@" > $OUT/$n.log 2>&1 || { tail -20 $OUT/$n.log; exit 1; }
  tail -1 $OUT/$n.log | cut -c1-300
}
for s in 375 750 1500 3000; do run c2_$s --warmup 5 --steps 20 --slots $s --no-cpu-baseline --no-large --no-steady; done
run c4_0,8 --only-large --legs c4 --c4-sims 0,8
run c4_5 --only-large --legs c4 --c4-sims 5
run c5_2 --only-large --legs c5 --c5-slots 2
run c3_w16 --warmup 5 --steps 20 --workload c3 --no-cpu-baseline
