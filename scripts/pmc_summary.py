#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from separate rocprofv3 --pmc passes.

Reads gpurun_out/pmc/<tag>/run_counter_collection.csv for the FETCH_SIZE and
WRITE_SIZE passes (scripts/pmc.sh), keeps the last `--launches` dispatches of
the kernel (the bench's timed steps), and writes a JSON summary that bench.py
reports as roofline.traffic.

Units and corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced read, so the fetch figure is doubled; WRITE_SIZE is taken as is.
Both raw and corrected values are kept.
"""
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


def per_dispatch(path, kernel, counter):
    d = collections.defaultdict(float)
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                d[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="gpurun_out/pmc")
    ap.add_argument("--kernel", default="k_round_wg")
    ap.add_argument("--launches", type=int, default=100)
    ap.add_argument("--bench-args", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fetch = per_dispatch(os.path.join(a.dir, "fetch", "run_counter_collection.csv"), a.kernel, "FETCH_SIZE")
    write = per_dispatch(os.path.join(a.dir, "write", "run_counter_collection.csv"), a.kernel, "WRITE_SIZE")
    fetch, write = fetch[-a.launches:], write[-a.launches:]
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    out = {
        "kernel": a.kernel,
        "kernel_hash": kernel_hash(),
        "launches_averaged": len(fetch),
        "bench_args": a.bench_args,
        "fetch_size_kib_raw": fk,
        "write_size_kib_raw": wk,
        "fetch_bytes_corrected": fk * 1024 * 2,
        "write_bytes": wk * 1024,
        "traffic_bytes_per_launch": fk * 1024 * 2 + wk * 1024,
        "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE as is; KiB -> bytes",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
