#!/bin/bash
# Round 3: FETCH_SIZE and WRITE_SIZE passes (one rocprofv3 --pmc run each, kernel trace only)
# over a bench leg, summarised per round of the BFS family into profiles-ready JSON.
#   LEG=c5|c3|c4  FAMILY=...  MARKER=...  ROUNDS=a,b | ALL=1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
LEG=${LEG:-c5}
OUT=gpurun_out/r03/pmc_$LEG
mkdir -p $OUT
for pass in fetch:FETCH_SIZE write:WRITE_SIZE; do
  tag=${pass%%:*}; ctr=${pass#*:}
  timeout -k 10 ${PMC_TO:-400} rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/$tag -o run -- \
    python3 bench.py --only-large --legs $LEG > $OUT/$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $OUT/$tag.log; exit 1; }
done
python3 scripts/pmc_round.py --dir $OUT --family "$FAMILY" --marker "$MARKER" --rounds "${ROUNDS:-0,0}" \
  ${ALL:+--all} --out $OUT/pmc_bfs_$LEG.json
