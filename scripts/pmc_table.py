#!/usr/bin/env python3
"""Per-kernel PMC averages from scripts/pmc_large.sh output directories.

usage: pmc_table.py <dir> <tag>... ; prints for each kernel family the mean of every
counter per dispatch (FETCH_SIZE / WRITE_SIZE in KiB as reported: raw)."""
import collections
import csv
import os
import sys

FAM = ['k_round_wg', 'k_mv_expand', 'k_mv_apply', 'k_mv_small', 'k_mv_levels', 'k_mv_gather', 'k_mv_consume', 'k_cg_consume', 'k_cg_prune', 'k_bin_expand', 'k_bin_apply', 'k_bin_gather', 'k_stats_pass', 'k_rotate_entries']


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    nd = collections.defaultdict(lambda: collections.defaultdict(set))
    for tag in sys.argv[2:]:
        path = os.path.join(d, tag, "run_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            fam = next((f for f in FAM if f in r["Kernel_Name"]), None)
            if not fam:
                continue
            acc[fam][r["Counter_Name"]] += float(r["Counter_Value"])
            nd[fam][r["Counter_Name"]].add(r["Dispatch_Id"])
    for fam in FAM:
        if fam not in acc:
            continue
        print(fam)
        for c, v in sorted(acc[fam].items()):
            n = len(nd[fam][c])
            print(f"   {c:28s} {v / n:16.1f} per dispatch  ({n} dispatches)")


if __name__ == "__main__":
    main()
