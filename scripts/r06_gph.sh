#!/bin/bash
# Round 6: gather phase clocks (GS_PHASE_PROFILE=1) of the c4 / c5 legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r06/gph; mkdir -p $OUT
for leg in ${LEGS:-c4}; do
  GS_PHASE_PROFILE=1 timeout -k 10 400 python3 bench.py --only-large --legs $leg > $OUT/$leg.log 2>&1 || { tail -20 $OUT/$leg.log; exit 1; }
  tail -1 $OUT/$leg.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
for k,v in d.items(): print(k, v.get('ms_per_step'), v.get('us_per_round'), v.get('gather_phases_wg_ms'))"
done
