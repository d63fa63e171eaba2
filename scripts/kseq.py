#!/usr/bin/env python3
"""Print the kernel sequence (name, us, grid) of the last `n` dispatches of a rocprofv3 trace."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
for r in rows[-n:]:
    print(f"{r['Kernel_Name'][:40]:40s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000:8.1f} {r['Grid_Size_X']}")
