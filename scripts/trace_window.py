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
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--first", type=int, required=True, help="index of the first launch kept")
    ap.add_argument("--count", type=int, required=True)
    ap.add_argument("--bench-args", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
