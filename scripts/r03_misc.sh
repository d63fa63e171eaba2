#!/bin/bash
# Round 3: C5 partition test, the c5 leg (16 origins), the C4 per-level diagnostics and
# the C2 per-rank shares (strong-scaling prediction).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r03/${TAG:-misc}
mkdir -p $OUT
if [ "${C5T:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -v -p no:cacheprovider --timeout 850 \
    --timeout-method thread -k c5 > $OUT/c5test.log 2>&1
  rc=$?; tail -3 $OUT/c5test.log
  if [ $rc -ne 0 ]; then grep -m5 -B2 -A30 "Error\|assert" $OUT/c5test.log | head -80; exit $rc; fi
fi
if [ "${C5L:-1}" = 1 ]; then
  timeout -k 10 400 python3 bench.py --only-large --legs c5 > $OUT/c5leg.json 2>&1 || { tail -20 $OUT/c5leg.json; exit 1; }
  cut -c1-2500 $OUT/c5leg.json
fi
if [ "${DIAG:-1}" = 1 ]; then
  GS_MV_DIAG=1 timeout -k 10 300 python3 bench.py --only-large --legs c4 > $OUT/c4diag.log 2>&1 || { tail -20 $OUT/c4diag.log; exit 1; }
  grep "GS_MV_DIAG levels" $OUT/c4diag.log | tail -2
fi
if [ "${SHARES:-1}" = 1 ]; then
  for s in 375 750 3000; do
    timeout -k 10 200 python3 bench.py --no-large --no-cpu-baseline --no-steady --slots $s --steps 20 --warmup 5 > $OUT/c2_s$s.json 2>&1 || { tail -20 $OUT/c2_s$s.json; exit 1; }
    echo "slots $s: $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $OUT/c2_s$s.json | tr '\n' ' ')"
  done
fi
