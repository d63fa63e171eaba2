#!/bin/bash
# A/B: parity tests on the main build, then the bench on the main build and on
# each variant under gossip-sim_amd/variants/<name> (same sources, other flags).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -z "$NO_TEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/ab_pytest.log 2>&1; rc=$?
  tail -5 gpurun_out/ab_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
for v in ${ORDER:-main ${VARIANTS}}; do
  if [ "$v" = main ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1])
print('$v', 'ms/step %.4f'%d['ms_per_step'], 'edges/s %.3e'%d['value'], 'kernel us %s'%d['roofline']['avg_launch_us'], 'frac %s'%d['roofline']['frac'], d.get('phases_wg_ms',''))"
done
