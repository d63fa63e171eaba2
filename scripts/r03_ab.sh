#!/bin/bash
# A/B of env settings on the c4 leg: each CASE is "label:ENV=.. ENV=..", one c4 run each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-ab}
mkdir -p $OUT
for spec in "$@"; do
  lab=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 200 python3 bench.py --only-large --legs ${LEGS:-c4} > $OUT/$lab.json 2>&1 || { echo "$lab failed"; tail -5 $OUT/$lab.json; exit 1; }
  echo "$lab: $(grep -o '"ms_per_step": [0-9.]*\|"us_per_round": {[^}]*}' $OUT/$lab.json | tr '\n' ' ')"
done
