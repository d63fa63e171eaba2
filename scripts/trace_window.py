#!/usr/bin/env python3
"""Kernel durations of a bench window from a rocprofv3 --kernel-trace CSV.

`--stats` averages every launch of a kernel in the whole run (warm-up, timed window,
steady leg, secondary legs). This script keeps the launches of one kernel that fall in
the timed window -- launches [first, first + count) of that kernel in dispatch order (one
launch per round for k_round_wg, so rounds W .. W + K - 1 of `bench.py --warmup W --steps
K`) -- and writes their average, min, max and every duration, stamped with the kernel hash
of the sources measured, so a bench line's `roofline.avg_launch_us` can be recomputed
from profiles/.

  python3 scripts/trace_window.py --csv gpurun_out/.../run_kernel_trace.csv \\
      --kernel k_round_wg --first 5 --count 20 --out profiles/r04/trace_k_round_wg_c2_r5-24.json
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_hash():
    sys.path.insert(0, ROOT)
    import bench
    return bench.load_pkg().kernel_hash()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--csv", required=True)
    ap.add_argument("--kernel", default="", help="substring of the kernel name")
    ap.add_argument("--first", type=int, default=0, help="index of the first launch kept")
    ap.add_argument("--count", type=int, default=0)
    ap.add_argument("--family", default="", help="family mode: comma-separated kernel names summed per round")
    ap.add_argument("--marker", default="", help="family mode: the kernel whose dispatches end the rounds")
    ap.add_argument("--rounds", default="", help="family mode: first,last round (0-based, of the marker's count)")
    ap.add_argument("--bench-args", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    if a.family:
        return family_mode(a)
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            if a.kernel in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             r["Kernel_Name"]))
    rows.sort()
    win = rows[a.first:a.first + a.count]
    if len(win) != a.count:
        raise SystemExit(f"{len(rows)} launches of {a.kernel}; window [{a.first}, {a.first + a.count}) incomplete")
    us = [(e - s) / 1e3 for _, s, e, _ in win]
    out = {"kernel": win[0][3][:120], "kernel_hash": kernel_hash(), "bench_args": a.bench_args,
           "launches_in_run": len(rows), "window_launches": [a.first, a.first + a.count],
           "avg_us": sum(us) / len(us), "min_us": min(us), "max_us": max(us),
           "durations_us": [round(x, 2) for x in us],
           "source": "rocprofv3 --kernel-trace (Start/End_Timestamp, ns)"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "durations_us"}))


def family_mode(a):
    """Per-round device time of a kernel family: the durations of every dispatch of the
    family between the marker dispatches that end rounds r0-1 and r1 (one engine; the
    round that a marker dispatch ends is counted from 0), summed per round and averaged --
    the time a bench leg's bfs_roofline divides by (its hipEvents span the same kernels)."""
    fam = a.family.split(",")
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, (_, _, k) in enumerate(rows) if a.marker in k]
    r0, r1 = (int(x) for x in a.rounds.split(","))
    per = []
    for r in range(r0, r1 + 1):
        lo, hi = (ends[r - 1] + 1 if r else 0), ends[r] + 1
        per.append(sum(e - s for s, e, k in rows[lo:hi] if any(x in k for x in fam)) / 1e3)
    out = {"kernels": fam, "marker": a.marker, "kernel_hash": kernel_hash(), "bench_args": a.bench_args,
           "rounds": [r0, r1], "avg_us": sum(per) / len(per), "min_us": min(per), "max_us": max(per),
           "per_round_us": [round(x, 1) for x in per], "launch": "one round of the family",
           "source": "rocprofv3 --kernel-trace (Start/End_Timestamp, ns)"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_round_us"}))


if __name__ == "__main__":
    main()
