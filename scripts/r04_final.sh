#!/bin/bash
# Round 4 closing measurements at HEAD, every summary stamped with the kernel hash
# (gossip_sim_amd.kernel_hash) that bench.py checks before reporting it:
#   1. C2 PMC traffic (FETCH_SIZE, WRITE_SIZE; one counter per rocprofv3 run) of the driver's
#      window (rounds 5-24) and the steady window (60-159) -> profiles/r04/pmc_k_round_wg_*.json
#   2. the c4 / c5 / c3 BFS families' PMC traffic per round -> profiles/r04/pmc_bfs_*.json
#   3. one SQ/TA counter pass of k_round_wg (driver window) and of the c4 / c5 BFS families
#   4. the driver's window under rocprofv3 --kernel-trace --stats: the stats CSV and the
#      window's k_round_wg launches -> profiles/r04/trace_k_round_wg_c2_r5-24.json
#   5. the bench lines (driver window, default) that read them
# Steps: STEPS="pmc_c2 pmc_legs sq trace bench" (default all).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r04/${TAG:-final}
P=profiles/r04
mkdir -p $OUT $P
STEPS=${STEPS:-"pmc_c2 pmc_legs sq trace bench"}
has() { case " $STEPS " in *" $1 "*) return 0;; *) return 1;; esac; }

if has pmc_c2; then
  for win in "5 20" "60 100"; do
    set -- $win; w=$1; s=$2; tag=c2_r$w-$((w + s - 1))
    d=$OUT/pmc_$tag
    mkdir -p $d
    for c in FETCH_SIZE WRITE_SIZE; do
      sub=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
      echo "== pmc $tag $c"
      timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d/$sub -o run -- \
        python3 bench.py --warmup $w --steps $s --no-cpu-baseline --no-profile --no-large --no-steady > $d/$sub.log 2>&1 \
        || { tail -5 $d/$sub.log; exit 1; }
    done
    python3 scripts/pmc_summary.py --dir $d --kernel k_round_wg --launches $s \
      --bench-args "--warmup $w --steps $s" --out $P/pmc_k_round_wg_$tag.json || exit 1
  done
fi

legpmc() {  # legpmc <leg> <family> <marker> <rounds|all> <timeout>
  local leg=$1 fam=$2 mark=$3 rounds=$4 to=$5 d=$OUT/pmc_$1
  mkdir -p $d
  for pass in fetch:FETCH_SIZE write:WRITE_SIZE; do
    local tag=${pass%%:*} ctr=${pass#*:}
    echo "== pmc $leg $ctr"
    timeout -s KILL $to rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $d/$tag -o run -- \
      python3 bench.py --only-large --legs $leg > $d/$tag.log 2>&1 || { echo "pmc $leg $tag failed"; tail -5 $d/$tag.log; return 1; }
  done
  if [ "$rounds" = all ]; then
    python3 scripts/pmc_round.py --dir $d --family "$fam" --marker "$mark" --all --out $P/pmc_bfs_$6_$leg.json
  else
    python3 scripts/pmc_round.py --dir $d --family "$fam" --marker "$mark" --rounds "$rounds" --out $P/pmc_bfs_$6_$leg.json
  fi
}
if has pmc_legs; then
  MV=k_mv_expand,k_mv_apply,k_mv_small,k_mv_levels,k_mv_gather
  legpmc c4 $MV k_mv_gather 5,24 400 multi || exit 1
  legpmc c5 $MV k_mv_gather 3,12 600 multi || exit 1
  legpmc c3 k_bin_small,k_bin_expand,k_bin_apply,k_bin_gather,k_bin_seed k_bin_gather all 400 binned || exit 1
fi

if has sq; then
  d=$OUT/sq
  mkdir -p $d
  echo "== sq k_round_wg"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    SQ_INSTS_LDS TA_BUSY_avr --kernel-trace --output-format csv -d $d/c2 -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-profile --no-large --no-steady > $d/c2.log 2>&1 \
    || { tail -5 $d/c2.log; exit 1; }
  for leg in c4 c5; do
    echo "== sq $leg"
    timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
      SQ_INSTS_LDS TA_BUSY_avr --kernel-trace --output-format csv -d $d/$leg -o run -- \
      python3 bench.py --only-large --legs $leg > $d/$leg.log 2>&1 || { tail -5 $d/$leg.log; exit 1; }
  done
  python3 scripts/pmc_table.py $d/c2/run_counter_collection.csv k_round_wg > $P/sq_k_round_wg_c2.txt 2>&1 || true
  for leg in c4 c5; do
    python3 scripts/pmc_table.py $d/$leg/run_counter_collection.csv k_mv_ > $P/sq_bfs_multi_$leg.txt 2>&1 || true
  done
fi

if has trace; then
  echo "== trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  python3 scripts/trace_window.py --csv $OUT/prof/run_kernel_trace.csv --kernel k_round_wg --first 5 --count 20 \
    --bench-args "--warmup 5 --steps 20" --out $P/trace_k_round_wg_c2_r5-24.json || exit 1
  cp $OUT/prof/run_kernel_stats.csv $P/rocprof_kernel_stats_driver_window.csv
  grep '"metric"' $OUT/prof.log | tail -1 > $P/bench_driver_window_traced.json
fi

if has bench; then
  echo "== bench driver window"
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 1; }
  grep '"metric"' $OUT/bench_driver.log | tail -1 > $P/bench_driver_window.json
  cut -c1-400 $P/bench_driver_window.json
fi
