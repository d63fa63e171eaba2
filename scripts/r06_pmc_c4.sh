#!/bin/bash
# Round 6: c4 leg BFS-family PMC (FETCH_SIZE, WRITE_SIZE) and per-kernel write split (A/B).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
d=gpurun_out/r06/${TAG:-pmc_c4}
mkdir -p $d
for pass in fetch:FETCH_SIZE write:WRITE_SIZE; do
  tag=${pass%%:*}; ctr=${pass#*:}
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $d/$tag -o run -- \
    python3 bench.py --only-large --legs c4 > $d/$tag.log 2>&1 || { tail -5 $d/$tag.log; exit 1; }
done
python3 scripts/pmc_round.py --dir $d --family k_mv_expand,k_mv_apply,k_mv_small,k_mv_pbfs,k_mv_gather \
  --marker k_mv_gather --rounds 5,24 --out $d/pmc_bfs_multi_c4.json
for k in k_mv_pbfs k_mv_gather; do
  python3 scripts/pmc_round.py --dir $d --family $k --marker k_mv_gather --rounds 5,24 --out $d/pmc_$k.json | cut -c1-400
done
