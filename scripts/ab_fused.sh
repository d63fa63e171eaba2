#!/bin/bash
# A/B of gs_round's multi path: fused gather+consume vs gather then k_cg_consume (c4 leg).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02
mkdir -p $OUT
if [ -n "$PARITY_K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -k "$PARITY_K" > $OUT/parity_ab.log 2>&1
  rc=$?; tail -3 $OUT/parity_ab.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for fu in 0 1; do
  GS_MV_FUSED=$fu timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_ab$fu -o run -- \
    python3 bench.py --only-large --large-mode 4 > $OUT/ab$fu.json 2>&1 || exit $?
  echo "== fused=$fu"; grep -o '"c4".*"bfs_roofline"' $OUT/ab$fu.json
  python3 scripts/round_breakdown.py $OUT/prof_ab$fu/run_kernel_trace.csv k_stats 5 25 | head -14
done
