"""The simulations both sides of tests/test_partition.py run.

small: a 3,000-node network (rank ranges of whole 1,024-id bins: [0, 2048), [2048, 3000)),
       three origins with their own prune thresholds / min-ingress, node failures at round
       3, heavy rotation, 34 rounds of which the last 24 are recorded. Every per-node
       array is compared, caches included.
large: 1M nodes (power-law stakes), four slots (origin rank 1 with two thresholds, a
       fail-nodes slot, a second origin), 24 rounds through the first prune wave; caches
       are compared on a sample of nodes on both sides of the rank boundary.
c5:    BASELINE C5 as configured -- 10M nodes (power-law stakes), origin ranks 1..16 as 16
       slots, 22 rounds through the first prune wave (rounds 2..21 recorded). Per-node
       arrays are compared by SHA-256 digests of each rank's owned range (and of the
       replicated prune state), caches on a sample around the rank boundary."""
import hashlib

import numpy as np

CASES = {
    "small": dict(n=3000, origins=[0, 57, 2601], mi=[2, 1, 3], thr=[0.15, 0.0, 0.4], fail=[0.0, 0.1, 0.05],
                  fail_at=3, rounds=34, warm=10, seed=21, p=0.06, synth="network"),
    "large": dict(n=1_000_000, origins=None, mi=[2, 2, 2, 1], thr=[0.15, 0.4, 0.15, 0.05], fail=[0.0, 0.0, 0.2, 0.0],
                  fail_at=0, rounds=24, warm=4, seed=0x5EED0003, p=0.013333, synth="power_law"),
    "c5": dict(n=10_000_000, origins="ranks", mi=[2] * 16, thr=[0.15] * 16, fail=[0.0] * 16, fail_at=None,
               rounds=22, warm=2, seed=0x5EED0003, p=0.013333, synth="power_law", digest=True),
}


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def stakes_of(case, synth):
    c = CASES[case]
    if c["synth"] == "network":
        return synth.network(c["n"])[1]
    return synth.power_law_stakes(c["n"])


def origins_of(case, stakes):
    c = CASES[case]
    if isinstance(c["origins"], list):
        return c["origins"]
    order = np.lexsort((np.arange(len(stakes)), -np.asarray(stakes, dtype=np.float64)))
    if c["origins"] == "ranks":  # origin ranks 1..S (gossip_main.rs:279-290)
        return [int(x) for x in order[:len(c["mi"])]]
    top = int(order[0])  # origin rank 1: largest stake, lowest id on ties
    return [top, top, top, int(order[100])]


def cache_sample(case):
    n = CASES[case]["n"]
    if n <= 5000:
        return None  # every node
    if case == "c5":  # both sides of the two-rank boundary, the ends
        b = ((-(-n // 2)) + 1023) & ~1023
        return sorted(set([0, 1, 2, 1000, n - 2, n - 1] + list(range(b - 24, b + 24))))
    return sorted(set([0, 1, 2, n // 2 - 300, n // 2 - 1, n // 2, n // 2 + 300, n - 2, n - 1] +
                      list(range(499_700, 499_720)) + list(range(500_280, 500_300))))


def run_case(eng, case, stakes, ranges=None, on_round=None):
    """Runs a case on an Engine or a PartitionedEngine; returns the state to compare.
    Digest cases hash the per-node arrays over each (lo, hi) of `ranges`."""
    c = CASES[case]
    S = len(c["mi"])
    eng.set_slots(origins_of(case, stakes), c["mi"], c["thr"])
    eng.init_active_sets()
    for r in range(c["rounds"]):
        if r == c["fail_at"]:
            eng.fail_nodes(c["fail"])
        eng.round(r, record=r >= c["warm"])
        if on_round:
            on_round(r, eng)
    out = {"summaries": eng.summaries()}
    if c.get("digest"):
        for k in range(S):
            eg, ing, pr, st, hh = eng.accumulators(k)
            hops = eng.hops(k)
            out[f"hist{k}"] = np.asarray(hh)
            out[f"pruned{k}"] = np.array([digest(eng.pruned_all(k))])
            out[f"dig{k}"] = np.array([[digest(a[lo:hi]) for a in (eg, ing, pr, st, hops)] for lo, hi in ranges])
        return out
    sample = cache_sample(case)
    for k in range(S):
        eg, ing, pr, st, hh = eng.accumulators(k)
        out[f"acc{k}"] = np.stack([np.asarray(eg, np.uint64), np.asarray(ing, np.uint64), np.asarray(pr, np.uint64),
                                   np.asarray(st, np.uint64)])
        out[f"hist{k}"] = np.asarray(hh)
        out[f"hops{k}"] = eng.hops(k)
        out[f"pruned{k}"] = eng.pruned_all(k)
        if sample is None:
            up, ln, keys, sc = eng.caches(k)
            out[f"cache{k}"] = np.concatenate([up[:, None].astype(np.uint64), ln[:, None].astype(np.uint64),
                                               keys.astype(np.uint64), sc.astype(np.uint64)], axis=1)
    return out


def cache_rows(eng, case, k, lo=0, hi=None):
    """ReceivedCache entries of the sampled nodes in [lo, hi) (num_upserts, keys, scores)."""
    hi = CASES[case]["n"] if hi is None else hi
    rows = {}
    for v in cache_sample(case) or []:
        if lo <= v < hi:
            rows[v] = eng.cache(k, v)
    return rows
