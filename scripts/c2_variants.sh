#!/bin/bash
# C2 bench line with the round kernel built at 768 (default), 640 and 576 threads.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r02
mkdir -p $OUT
for v in "" t640 t576; do
  GS_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --no-large --no-cpu-baseline --steps 100 --warmup 20 \
    > $OUT/c2_${v:-t768}.json 2> $OUT/c2_${v:-t768}.err || exit $?
  echo "== ${v:-t768}"; python3 -c "import json,sys; d=json.loads(open('$OUT/c2_${v:-t768}.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('avg_launch_us'))"
done
