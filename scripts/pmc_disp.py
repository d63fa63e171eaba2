#!/usr/bin/env python3
"""Counters of ONE dispatch of a kernel family from rocprofv3 --pmc csv directories: the
dispatch with the largest value of a ranking counter in the first directory (e.g. the
prune wave's k_cg_prune), matched by dispatch order in the others.

usage: pmc_disp.py <kernel substring> <rank counter> <dir>..."""
import collections
import csv
import os
import sys


def load(d, kern):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if kern in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] = per[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    kern, rank, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    runs = [load(d, kern) for d in dirs]
    i = max(range(len(runs[0])), key=lambda j: runs[0][j].get(rank, 0))
    print(f"{kern}: dispatch #{i} of {len(runs[0])} (largest {rank})")
    for r in runs:
        if i < len(r):
            for c, v in sorted(r[i].items()):
                print(f"  {c:28s} {v:16.1f}")


if __name__ == "__main__":
    main()
