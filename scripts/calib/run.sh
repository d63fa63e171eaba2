#!/bin/bash
# Builds (on the CPU side beforehand) and runs the FETCH/WRITE calibration passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r02/calib
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o run -- \
    ./scripts/calib/calib_fetch > $OUT/$c.log 2>&1 || { tail -5 $OUT/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/r02/calib/{c}/run_counter_collection.csv")):
        d[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for k, v in d.items():
        print(c, k, [round(x / 1024, 1) for x in v], "MiB-equivalent (KiB/1024) per dispatch")
PY
