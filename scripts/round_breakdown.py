#!/usr/bin/env python3
"""Per-round kernel time breakdown from a rocprofv3 --kernel-trace csv.

usage: round_breakdown.py <trace.csv> <round-end kernel substring> <first round> <last round>
Rounds are delimited by the dispatches of the round-end kernel (e.g. k_mv_gather,
k_bin_gather, k_round_wg); prints per-family device time per round and the idle gaps
between consecutive dispatches (GPU time with nothing running)."""
import collections
import csv
import sys

FAMILIES = ["k_mv_expand", "k_mv_apply", "k_mv_gather", "k_mv_seed", "k_mv_fused", "k_bin_expand", "k_bin_apply",
            "k_bin_gather", "k_bfs_level", "k_cg_consume", "k_cg_prune", "k_round_wg", "k_stats", "k_rotate",
            "k_own_rows", "copyBuffer", "fillBuffer"]


def main():
    path, endk, r0, r1 = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rounds, cur = [], []
    for r in rows:
        cur.append(r)
        if endk in r["Kernel_Name"]:
            rounds.append(cur)
            cur = []
    sel = [x for rr in rounds[r0:r1] for x in rr]
    tot, cnt, prev, gap = collections.Counter(), collections.Counter(), None, 0.0
    mx = collections.Counter()
    for r in sel:
        n = next((f for f in FAMILIES if f in r["Kernel_Name"]), r["Kernel_Name"][:40])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev is not None and s > prev:
            gap += (s - prev) / 1e3
        prev = max(prev or 0, e)
        tot[n] += (e - s) / 1e3
        cnt[n] += 1
        mx[n] = max(mx[n], (e - s) / 1e3)
    k = max(1, r1 - r0)
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / k
    print(f"rounds {r0}..{r1 - 1}: wall {wall:.1f} us/round, idle gaps {gap / k:.1f} us/round")
    for n, t in tot.most_common():
        print(f"  {n:28s} {t / k:9.1f} us/round  {cnt[n] / k:6.1f} launches/round  {t / cnt[n]:8.1f} us/launch  max {mx[n]:8.1f}")


if __name__ == "__main__":
    main()
