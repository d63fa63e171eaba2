#!/usr/bin/env python3
"""Per-round HBM traffic of a kernel family from rocprofv3 --pmc passes of the bench's
c4 leg (scripts/pmc_large.sh with LEGS=c4): the FETCH_SIZE and WRITE_SIZE of every
dispatch of the family between the end-marker kernel's dispatches that bound the timed
rounds, summed per round and averaged. Corrections as in profiles/r02/fetch_calibration.json
(FETCH_SIZE x2 for the 4-B, 16-B and scattered read patterns measured there; WRITE_SIZE
as is)."""
import argparse
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_hash():
    """The hash of the kernel sources this profile measured (bench.py checks it)."""
    sys.path.insert(0, ROOT)
    import bench
    return bench.load_pkg().kernel_hash()


def load(path, counter):
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    d = collections.OrderedDict()
    for i, k, v in sorted(rows):
        if i not in d:
            d[i] = [k, 0.0]
        d[i][1] += v
    return [(i, k, v) for i, (k, v) in d.items()]


def per_round(rows, family, marker, first, last):
    ends = [n for n, (_, k, _) in enumerate(rows) if marker in k]
    tot, n = 0.0, 0
    for r in range(first, last + 1):
        lo, hi = ends[r - 1] + 1 if r else 0, ends[r] + 1
        tot += sum(v for _, k, v in rows[lo:hi] if any(f in k for f in family))
        n += 1
    return tot / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--family", default="k_mv_expand,k_mv_apply,k_mv_small,k_mv_seed,k_mv_gather")
    ap.add_argument("--marker", default="k_mv_gather")
    ap.add_argument("--rounds", default="5,24")
    ap.add_argument("--out", required=True)
    ap.add_argument("--all", action="store_true",
                    help="every round of the run (engines interleaved): family total / marker dispatches")
    a = ap.parse_args()
    fam = a.family.split(",")
    r0, r1 = (int(x) for x in a.rounds.split(","))
    fr = load(os.path.join(a.dir, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    wr = load(os.path.join(a.dir, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    if a.all:
        def whole(rows):
            n = sum(1 for _, k, _ in rows if a.marker in k)
            return sum(v for _, k, v in rows if any(x in k for x in fam)) / n
        f, w = whole(fr), whole(wr)
        r0, r1 = "all", "all"
    else:
        f = per_round(fr, fam, a.marker, r0, r1)
        w = per_round(wr, fam, a.marker, r0, r1)
    out = {"kernels": fam, "kernel_hash": kernel_hash(), "rounds": [r0, r1], "fetch_size_kib_raw_per_round": f, "write_size_kib_raw_per_round": w,
           "fetch_bytes_corrected": f * 1024 * 2, "write_bytes": w * 1024,
           "traffic_bytes_per_launch": f * 1024 * 2 + w * 1024, "launch": "one round of the family",
           "correction": "FETCH_SIZE x2, WRITE_SIZE as is (profiles/r02/fetch_calibration.json); KiB -> bytes"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
