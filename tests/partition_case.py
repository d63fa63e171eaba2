"""The simulation both sides of tests/test_partition.py run: a 700-node network, three
origins with their own prune thresholds / min-ingress, node failures at round 3, heavy
rotation, 34 rounds of which the last 24 are recorded."""
import numpy as np

CASE = dict(n=700, origins=[0, 57, 601], mi=[2, 1, 3], thr=[0.15, 0.0, 0.4], fail=[0.0, 0.1, 0.05], fail_at=3,
            rounds=34, warm=10, seed=21, p=0.06)


def run_case(eng):
    """Runs CASE on an Engine or a PartitionedEngine; returns the state to compare."""
    c = CASE
    eng.set_slots(c["origins"], c["mi"], c["thr"])
    eng.init_active_sets()
    for r in range(c["rounds"]):
        if r == c["fail_at"]:
            eng.fail_nodes(c["fail"])
        eng.round(r, record=r >= c["warm"])
    out = {"summaries": eng.summaries()}
    for k in range(len(c["origins"])):
        eg, ing, pr, st, hh = eng.accumulators(k)
        out[f"acc{k}"] = np.stack([np.asarray(eg, np.uint64), np.asarray(ing, np.uint64), np.asarray(pr, np.uint64),
                                   np.asarray(st, np.uint64)])
        out[f"hist{k}"] = np.asarray(hh)
        out[f"hops{k}"] = eng.hops(k)
        out[f"pruned{k}"] = eng.pruned_all(k)
        up, ln, keys, sc = eng.caches(k)
        out[f"cache{k}"] = np.concatenate([up[:, None].astype(np.uint64), ln[:, None].astype(np.uint64),
                                           keys.astype(np.uint64), sc.astype(np.uint64)], axis=1)
    return out
