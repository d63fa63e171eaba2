#!/bin/bash
# Round 3 closing measurements at HEAD: the default bench line (all legs, CPU baselines),
# the driver's window untraced, the driver's window under rocprofv3 --kernel-trace --stats;
# first the C2 PMC traffic of the bench windows (FETCH_SIZE, WRITE_SIZE; one counter per run),
# which the bench lines then report as roofline.traffic.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/final
mkdir -p $OUT
set -o pipefail
if [ "${PMC:-1}" = 1 ]; then
  for win in "5 20" "20 100" "60 100"; do
    set -- $win; w=$1; s=$2; tag=c2_r$w-$((w + s - 1))
    d=$OUT/pmc_$tag
    mkdir -p $d
    for c in FETCH_SIZE WRITE_SIZE; do
      sub=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
      timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $d/$sub -o run -- \
        python3 bench.py --warmup $w --steps $s --no-cpu-baseline --no-profile --no-large --no-steady > $d/$sub.log 2>&1 \
        || { tail -5 $d/$sub.log; exit 1; }
    done
    python3 scripts/pmc_summary.py --dir $d --kernel k_round_wg --launches $s \
      --bench-args "--warmup $w --steps $s" --out $OUT/pmc_k_round_wg_$tag.json > /dev/null || exit 1
  done
  mkdir -p profiles/r03 && cp $OUT/pmc_k_round_wg_*.json profiles/r03/  # (the benches below read them)
  ls $OUT/pmc_k_round_wg_*.json
fi

if [ "${DEF:-1}" = 1 ]; then
  timeout -k 10 600 python3 bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
  grep '"metric"' $OUT/bench_default.log | tail -1 > $OUT/bench_default.json
  echo "default: $(cut -c1-300 $OUT/bench_default.json)"
fi
if [ "${DRV:-1}" = 1 ]; then
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 1; }
  grep '"metric"' $OUT/bench_driver.log | tail -1 > $OUT/bench_driver_window.json
  echo "driver: $(cut -c1-300 $OUT/bench_driver_window.json)"
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
  grep '"metric"' $OUT/prof.log | tail -1 > $OUT/bench_traced.json
fi
