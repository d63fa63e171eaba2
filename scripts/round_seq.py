#!/usr/bin/env python3
"""One round's dispatch sequence from a rocprofv3 --kernel-trace csv: kernel, start offset
from the round's first dispatch, duration and the idle gap before it (us).
usage: round_seq.py trace.csv ROUND_MARK_KERNEL ROUND_INDEX"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mark, ridx = sys.argv[2], int(sys.argv[3])
# rounds end at each dispatch of the mark kernel
ends = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
lo = ends[ridx - 1] + 1 if ridx > 0 else 0
hi = ends[ridx] + 1
t0 = int(rows[lo]["Start_Timestamp"])
prev = t0
busy = 0
for r in rows[lo:hi]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{r['Kernel_Name'][:34]:34s} at {(s - t0) / 1e3:8.1f}  dur {(e - s) / 1e3:7.1f}  gap {(s - prev) / 1e3:6.1f}"
          f"  grid {r['Grid_Size_X']}")
    prev = e
print(f"round span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
