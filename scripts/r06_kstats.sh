#!/bin/bash
# Per-kernel totals (rocprofv3 --stats) of bench legs under env variants.
#   TAG=... LEGS=c4 VARIANTS="A=1;A=0"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/${TAG:-kstats}
mkdir -p $OUT
i=0
IFS=';' read -ra VS <<< "${VARIANTS:-X=1}"
for v in "${VS[@]}"; do
  i=$((i+1))
  echo "== variant $i: $v"
  env $v timeout -k 10 ${LEG_TO:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$i -o run -- \
    python3 bench.py --only-large --legs ${LEGS:-c4} > $OUT/v$i.log 2>&1 || { tail -20 $OUT/v$i.log; exit 1; }
  python3 - $OUT/v$i/run_kernel_stats.csv <<'P'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
P
done
