#!/bin/bash
# Round 5: k_round_wg phase clocks (GS_PHASE_PROFILE=1, workgroup-ms per phase) for the
# driver window's ordinary rounds (5-18), the prune-wave round (19), the rounds after it,
# and the 375-slot share.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r05/${TAG:-c2ph}
mkdir -p $OUT
WINS=${WINS:-"5,14,3000 19,1,3000 20,5,3000 5,14,375 19,1,375"}
for w in $WINS; do
  w=${w//,/ }
  set -- $w
  echo "== warmup $1 steps $2 slots $3"
  env GS_PHASE_PROFILE=1 $ENVX timeout -k 10 200 python3 bench.py --warmup $1 --steps $2 --slots $3 --no-cpu-baseline --no-large --no-steady \
    > $OUT/ph_$1_$2_$3.log 2>&1 || { tail -5 $OUT/ph_$1_$2_$3.log; exit 1; }
  grep '"metric"' $OUT/ph_$1_$2_$3.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); n=$2*$3
print(round(d['ms_per_step'],4), d['roofline']['avg_launch_us'], {k: round(v/n*1e3,2) for k,v in d['phases_wg_ms'].items()}, 'us/wg')"
done
