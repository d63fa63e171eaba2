#!/usr/bin/env python3
"""Per-launch durations (us) of one kernel from a rocprofv3 --kernel-trace csv directory."""
import csv
import glob
import sys

d, kern = sys.argv[1], sys.argv[2]
for f in glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True):
    t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f))
         if kern in r["Kernel_Name"]]
    print(f"{kern}: {len(t)} launches, mean {sum(t) / max(len(t), 1):.1f} us; last 60:",
          " ".join(f"{x:.0f}" for x in t[-60:]))
