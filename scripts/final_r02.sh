#!/bin/bash
# Round-2 closing measurements: the C5 leg alone, the default bench line under a kernel
# trace, and the c4 leg's BFS-family PMC traffic (FETCH_SIZE / WRITE_SIZE passes).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/final
mkdir -p $OUT
if [ "${SKIP_C5:-0}" != 1 ]; then
  timeout -k 10 400 python3 bench.py --only-large --legs c5 > $OUT/c5.json 2>&1 || { tail -20 $OUT/c5.json; exit 1; }
  tail -c 1200 $OUT/c5.json; echo
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  grep -h '"metric"' $OUT/bench.log | tail -1 > $OUT/bench.json
  cut -c1-1500 $OUT/bench.json
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    sub=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_c4/$sub -o run -- \
      python3 bench.py --only-large --legs c4 > $OUT/pmc_c4_$sub.log 2>&1 || { tail -5 $OUT/pmc_c4_$sub.log; exit 1; }
  done
  python3 scripts/pmc_round.py --dir $OUT/pmc_c4 --marker k_mv_gather --rounds 5,24 --out $OUT/pmc_bfs_multi_c4.json
fi
