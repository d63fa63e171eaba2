#!/bin/bash
# A/B of library variants on a bench leg (LEGS, default c4), interleaved, two reps.
# "head" = the in-tree build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r03/${TAG:-legvar}
mkdir -p $OUT
for rep in 1 2; do
  for v in "$@"; do
    lab=$v; [ "$v" = head ] && v=""
    GS_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --only-large --legs ${LEGS:-c4} > $OUT/$lab.json 2>&1 || { tail -5 $OUT/$lab.json; exit 1; }
    echo "$lab rep $rep: $(grep -o '"ms_per_step": [0-9.]*\|"us_per_round": {[^}]*}' $OUT/$lab.json | tr '\n' ' ')"
  done
done
