#!/bin/bash
# Round 6 closing measurements at HEAD, every summary stamped with the kernel hash
# (gossip_sim_amd.kernel_hash) that bench.py checks before reporting it:
#   1. C2 PMC traffic (FETCH_SIZE, WRITE_SIZE; one counter per rocprofv3 run) of the driver's
#      window (rounds 5-24) and the steady window (60-159) -> profiles/r04/pmc_k_round_wg_*.json
#   2. the c4 / c5 / c3 BFS families' PMC traffic per round -> profiles/r04/pmc_bfs_*.json
#   3. one SQ/TA counter pass of k_round_wg (driver window) and of the c4 / c5 BFS families
#   4. the driver's window under rocprofv3 --kernel-trace --stats: the stats CSV and the
#      window's k_round_wg launches -> profiles/r04/trace_k_round_wg_c2_r5-24.json
#   5. the bench lines (driver window, default) that read them
# Steps: STEPS="pmc_c2 pmc_legs sq trace trace_default bench" (default all).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/${TAG:-final}
P=profiles/r06
mkdir -p $OUT $P
STEPS=${STEPS:-"pmc_c2 pmc_legs sq trace trace_default bench"}
has() { case " $STEPS " in *" $1 "*) return 0;; *) return 1;; esac; }
# (the box's profiles/r06 is read by the later steps' bench runs; only gpurun_out/ comes back:
# every exit copies it there)
# (only what this call wrote: a later call of a split run must not overwrite an earlier
# call's fresh summaries with the tree's old ones)
touch $OUT/.start_$$
trap 'mkdir -p $OUT/profiles_r06 && find $P -maxdepth 1 -type f -newer $OUT/.start_$$ -exec cp {} $OUT/profiles_r06/ \;' EXIT

if has pmc_c2; then
  for win in "5 20" "60 100" "20 100"; do  # (20 100: bench.py's defaults)
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
  MV=k_mv_expand,k_mv_apply,k_mv_small,k_mv_pbfs,k_mv_gather
  legpmc c4 $MV k_mv_gather 5,24 400 multi || exit 1
  legpmc c5 $MV k_mv_gather 3,12 600 multi || exit 1
  # (c3: two one-slot engines run concurrently, two gather markers per round: marker
  # intervals 10..49 are the engine-rounds of rounds 5..24, the leg's launches)
  legpmc c3 $MV k_mv_gather 10,49 400 multi || exit 1
fi

if has sq; then
  SQC=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,TA_BUSY_avr
  d=$OUT/sq
  mkdir -p $d
  echo "== sq k_round_wg"
  timeout -s KILL 300 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $d/c2 -o run -- \
    python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --no-profile --no-large --no-steady > $d/c2.log 2>&1 \
    || { tail -5 $d/c2.log; exit 1; }
  for leg in c4 c5; do
    echo "== sq $leg"
    timeout -s KILL 600 rocprofv3 --pmc $SQC --kernel-trace --output-format csv -d $d/$leg -o run -- \
      python3 bench.py --only-large --legs $leg > $d/$leg.log 2>&1 || { tail -5 $d/$leg.log; exit 1; }
  done
  KH=$(python3 -c "import bench; print(bench.load_pkg().kernel_hash())")
  for leg in c2 c4 c5; do
    { echo "kernel_hash: $KH (SQ/TA counters, one rocprofv3 --pmc pass; bench legs as in r06_final.sh)";
      python3 scripts/pmc_table.py $d $leg; } > $P/sq_counters_$leg.txt 2>&1 || true
  done
fi

if has trace; then
  echo "== trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  python3 scripts/trace_window.py --csv $OUT/prof/run_kernel_trace.csv --kernel k_round_wg --first 5 --count 20 \
    --bench-args "--warmup 5 --steps 20" --out $P/trace_k_round_wg_c2_r5-24.json || exit 1
  # the steady leg of the same run: rounds 60-159 (launches 60.. of k_round_wg)
  python3 scripts/trace_window.py --csv $OUT/prof/run_kernel_trace.csv --kernel k_round_wg --first 60 --count 100 \
    --bench-args "--warmup 5 --steps 20 (steady leg)" --out $P/trace_k_round_wg_c2_r60-159.json || exit 1
  cp $OUT/prof/run_kernel_stats.csv $P/rocprof_kernel_stats_driver_window.csv
  grep '"metric"' $OUT/prof.log | tail -1 > $P/bench_driver_window_traced.json
  echo "== trace legs"
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/proflegs -o run -- \
    python3 bench.py --only-large --legs c4,c5 > $OUT/proflegs.log 2>&1 || { tail -20 $OUT/proflegs.log; exit 1; }
  MVT=k_mv_expand,k_mv_apply,k_mv_small,k_mv_pbfs,k_mv_gather
  python3 scripts/trace_window.py --csv $OUT/proflegs/run_kernel_trace.csv --family $MVT --marker k_mv_gather \
    --rounds 5,24 --bench-args "--only-large --legs c4" --out $P/trace_bfs_multi_c4.json || exit 1
  # (c5's rounds follow c4's 25 in the same trace: c4 rounds 0-24 end at marker 24)
  python3 scripts/trace_window.py --csv $OUT/proflegs/run_kernel_trace.csv --family $MVT --marker k_mv_gather \
    --rounds 28,37 --bench-args "--only-large --legs c5" --out $P/trace_bfs_multi_c5.json || exit 1
  echo "== trace c3 leg"
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/profc3 -o run -- \
    python3 bench.py --only-large --legs c3 > $OUT/profc3.log 2>&1 || { tail -20 $OUT/profc3.log; exit 1; }
  python3 scripts/trace_window.py --csv $OUT/profc3/run_kernel_trace.csv --family $MVT --marker k_mv_gather \
    --rounds 10,49 --bench-args "--only-large --legs c3 (engine-rounds)" --out $P/trace_bfs_multi_c3.json || exit 1
fi

if has trace_default; then  # bench.py with no flags: rounds 20-119
  echo "== trace default window"
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/profd -o run -- \
    python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-large --no-steady > $OUT/profd.log 2>&1 || { tail -20 $OUT/profd.log; exit 1; }
  python3 scripts/trace_window.py --csv $OUT/profd/run_kernel_trace.csv --kernel k_round_wg --first 20 --count 100 \
    --bench-args "--warmup 20 --steps 100" --out $P/trace_k_round_wg_c2_r20-119.json || exit 1
fi

if has bench; then
  echo "== bench driver window"
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 1; }
  grep '"metric"' $OUT/bench_driver.log | tail -1 > $P/bench_driver_window.json
  cut -c1-400 $P/bench_driver_window.json
fi
