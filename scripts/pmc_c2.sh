#!/bin/bash
# PMC traffic of k_round_wg for the C2 bench windows the bench reports: the driver's
# (--warmup 5 --steps 20: rounds 5-24) and the steady leg (rounds 60-159). One counter per
# rocprofv3 run (FETCH_SIZE, WRITE_SIZE), summaries into profiles/r02/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for win in "5 20" "60 100"; do
  set -- $win; w=$1; s=$2; tag=c2_r$w-$((w + s - 1))
  d=gpurun_out/pmc_$tag
  mkdir -p $d
  for c in FETCH_SIZE WRITE_SIZE; do
    sub=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
    timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d/$sub -o run -- \
      python3 bench.py --warmup $w --steps $s --no-cpu-baseline --no-profile --no-large --no-steady > $d/$sub.log 2>&1 \
      || { tail -5 $d/$sub.log; exit 1; }
  done
  python3 scripts/pmc_summary.py --dir $d --kernel k_round_wg --launches $s \
    --bench-args "--warmup $w --steps $s" --out gpurun_out/pmc_k_round_wg_$tag.json || exit 1
done
