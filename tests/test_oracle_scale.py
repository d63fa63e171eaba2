"""Oracle parity above the sizes the reference-structure oracle can initialise itself.

The oracle's initialize_gossip is O(25 N^2) (every entry shuffles all N candidates), so
the whole-simulation parity tests stop at 3,000 nodes. Two checks pin the engine to the
oracle at large N anyway:

- Active sets at 1M and 10M nodes: the determinism contract makes a node's entries a
  function of (seed, its id, the rounds) only, so the oracle replays ONE node's
  initialize_gossip (gossip.rs:805-813) and chance_to_rotate (gossip.rs:739-754) -- the
  same Philox INIT / DECIDE / ROTATE streams, PushActiveSetEntry::rotate over the
  id-ordered candidates (push_active_set.rs:73-114, 153-187) -- and every entry of sampled
  nodes must equal the engine's (its prefix-sum index tables at L = 17 and 20).
- Whole rounds at 100k nodes: the oracle is handed the engine's active sets (bulk entry
  upload) and then runs the reference's rounds itself; p = 0 keeps the sets fixed. For
  24 rounds, through the first prune wave, every BFS/consume variant of the engine must
  match it in hops, inbound (src, hop) lists, prunes, counters, prune state and received
  caches (node ids above 65,535; 4-byte and 8-byte binned records; the grid-wide and the
  single-workgroup level kernels).

Node pubkeys are stand-ins 0xA5 || 0^23 || id (big-endian): all encode to 44 base58
characters, so base58 order -- the reference's consume tie-break (gossip.rs:639-645) and
the node-id rule of the determinism contract -- is id order.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import engine_bind as eb
import oracle_bind as ob
from test_oracle_replay import stand_in_pubkeys

gs = eb.gs
pytestmark = pytest.mark.gpu
U64MAX = np.uint64(2**64 - 1)


def engine_entries(eng, node):
    out = np.full((25, eng.active_set_size), 0xFFFFFFFF, dtype=np.uint32)
    lens = np.zeros(25, dtype=np.uint8)
    for k in range(25):
        e = eng.get_entry(node, k)
        lens[k] = len(e)
        out[k, :len(e)] = e
    return out, lens


def check_replay(eng, st, seed, nodes, p, rounds):
    """Every entry of `nodes` equals the oracle's one-node replay; returns rotations per node."""
    asz = eng.active_set_size
    with ThreadPoolExecutor(max_workers=8) as ex:  # (the C replay releases the GIL)
        reps = list(ex.map(lambda v: ob.replay_node_entries(seed, st, v, asz, p, rounds), nodes))
    rot = {}
    for v, (peers, lens, nrot) in zip(nodes, reps):
        gp, gl = engine_entries(eng, v)
        np.testing.assert_array_equal(gl, lens, err_msg=f"entry lengths of node {v} after {rounds} rounds")
        np.testing.assert_array_equal(gp, peers, err_msg=f"entries of node {v} after {rounds} rounds")
        rot[v] = nrot
    return rot


@pytest.mark.parametrize("n,n_sample", [(1_000_000, 16), (10_000_000, 4)])
def test_active_sets_match_oracle_replay_at_scale(n, n_sample):
    """initialize_gossip and 20 rounds of chance_to_rotate at 1M / 10M nodes, sampled nodes'
    every entry (16 x 25 / 4 x 25 entries) against the oracle's replay of that node."""
    seed, p, rounds = 0x5EED0003, 0.05, 20
    st = eb.synth.power_law_stakes(n)
    rng = np.random.default_rng(n)
    eng = gs.Engine(st, 1, rotation_probability=p, seed=seed)
    eng.set_slots([0])
    eng.init_active_sets()
    fixed = [0, 1, n // 2, n - 1]  # the two largest stakes (top buckets), the middle, the smallest
    init_nodes = sorted(set(fixed[:max(2, n_sample // 4)] + rng.choice(n, n_sample, replace=False).tolist()))
    check_replay(eng, st, seed, init_nodes, p, 0)
    for r in range(rounds):
        eng.chance_to_rotate(r)
    # nodes that rotated at least once (P = 1 - 0.95^20 = 0.64) and some that did not
    rot_nodes = sorted(set(init_nodes[:2] + rng.choice(n, 2 * n_sample, replace=False).tolist()))
    rot = check_replay(eng, st, seed, rot_nodes, p, rounds)
    assert sum(1 for x in rot.values() if x > 0) >= n_sample // 2, rot
    eng.close()


# ------------------------------------------------------- 100k: whole rounds ----
VARIANTS = {  # name: engine kwargs (one origin slot each; results must be identical)
    "binned": dict(bfs_mode=gs.GS_BFS_BINNED),  # default hybrid: single-workgroup small levels, direct levels
    "binned_grid_direct": dict(bfs_mode=gs.GS_BFS_BINNED, no_small_levels=True),
    "binned_all": dict(bfs_mode=gs.GS_BFS_BINNED, binned_all_levels=True),  # 4-byte records
    "binned_all_wide": dict(bfs_mode=gs.GS_BFS_BINNED, binned_all_levels=True, wide_records=True),
    "multi": dict(bfs_mode=gs.GS_BFS_MULTI),
    "multi_no_small": dict(bfs_mode=gs.GS_BFS_MULTI, no_small_levels=True),
    "level": dict(bfs_mode=gs.GS_BFS_LEVEL),
}


def test_rounds_match_oracle_with_engine_active_sets_100k():
    n, seed, rounds, thr, mi = 100_000, 0x5EED0007, 24, 0.15, 2
    st = eb.synth.power_law_stakes(n)
    origin = int(np.lexsort((np.arange(n), -st.astype(np.float64)))[0])  # origin rank 1
    engs = {}
    for name, kw in VARIANTS.items():
        e = gs.Engine(st, 1, rotation_probability=0.0, seed=seed, **kw)
        e.set_slots([origin], mi, thr)
        e.init_active_sets()
        engs[name] = e
    peers, lens = engs["binned"].active_sets()
    for name, e in engs.items():
        if name != "binned":
            p2, l2 = e.active_sets()
            assert np.array_equal(p2, peers) and np.array_equal(l2, lens), name
    sim = ob.Sim(ob.PHILOX, seed, stand_in_pubkeys(n), st, 6)
    sim.set_entries(peers, lens)
    del peers, lens
    pruned_total = 0
    for r in range(rounds):
        sim.run_gossip(origin)
        want_d = sim.distances()
        w_off, w_src, w_hop = sim.orders_all(64 * n)
        for name, e in engs.items():
            e.run_gossip()
            np.testing.assert_array_equal(e.distances(0), want_d, err_msg=f"{name} hops round {r}")
            off, src, hop = e.inbound(0, cap=len(w_src) + 1)
            np.testing.assert_array_equal(off, w_off, err_msg=f"{name} in-degrees round {r}")
            np.testing.assert_array_equal(src[:len(w_src)], w_src, err_msg=f"{name} inbound sources round {r}")
            np.testing.assert_array_equal(hop[:len(w_hop)], w_hop, err_msg=f"{name} inbound hops round {r}")
        sim.consume_messages(origin)
        sim.send_prunes(origin, thr, mi)
        want_p = sim.prunes()
        pruned_total += len(want_p)
        full = r % 6 == 0 or 18 <= r <= 21 or r == rounds - 1
        if full:
            oup, oln, okeys, osc = sim.caches(origin)
            has = oup != 0xFFFFFFFF
        for name, e in engs.items():
            e.consume_messages()
            e.send_prunes()
            assert e.prunes(0) == want_p, f"{name} prunes round {r}"
            if full:
                up, ln, keys, sc = e.caches(0)
                np.testing.assert_array_equal(up[has], oup[has], err_msg=f"{name} upserts round {r}")
                np.testing.assert_array_equal(up[~has], 0)
                np.testing.assert_array_equal(ln, oln, err_msg=f"{name} cache lengths round {r}")
                np.testing.assert_array_equal(keys, okeys, err_msg=f"{name} cache keys round {r}")
                np.testing.assert_array_equal(sc, osc, err_msg=f"{name} cache scores round {r}")
        sim.prune_connections()
        oe, oi, op = sim.counters()
        om = sim.pruned_all(origin)
        for name, e in engs.items():
            e.prune_connections()
            eg, ig, pr = e.counters(0)
            np.testing.assert_array_equal(eg, np.where(oe == U64MAX, 0, oe), err_msg=f"{name} egress round {r}")
            np.testing.assert_array_equal(ig, np.where(oi == U64MAX, 0, oi), err_msg=f"{name} ingress round {r}")
            np.testing.assert_array_equal(pr, op, err_msg=f"{name} prune-sent round {r}")
            np.testing.assert_array_equal(e.pruned_all(0), om, err_msg=f"{name} prune state round {r}")
    assert pruned_total > 0  # the first prune wave happened inside the window
    assert int(w_src.max()) >= 65536  # ids beyond u16
    for e in engs.values():
        e.close()


# ------------------------------------------- 100k: C4's sweep semantics, gs_round ----
C4_SLOTS = [  # (origin stake rank, fail fraction, prune-stake threshold, min-ingress)
    (1, 0.3, 0.15, 2),   # the fail-nodes sweep (when-to-fail 0): failed peers burn their slot
    (1, 0.0, 0.05, 1),   # the threshold sweep's ends, with other min-ingress values
    (1, 0.0, 0.40, 3),
    (2, 0.1, 0.15, 2),   # a second origin with failures
    (1, 0.5, 0.25, 2),
]
# C5's shape: distinct origins (stake ranks 1..8) without failures -- every slot is a plain
# slot whose own origin goes through the multi BFS's LDS origin hash (gs_mv_dev.h
# mv_origin_slots) -- plus one slot with failures sharing rank 1's origin (the per-slot path
# in the same waves)
C5_SLOTS = [(r, 0.0, 0.15, 2) for r in range(1, 9)] + [(1, 0.1, 0.15, 2)]

SWEEP_CASES = {  # id: (nodes, slots, bfs mode, environment at engine creation)
    "c4_multi": (100_000, C4_SLOTS, gs.GS_BFS_MULTI, {}),
    "c4_binned": (100_000, C4_SLOTS, gs.GS_BFS_BINNED, {}),
    # 64-node coarse bins: 625 >= 512 of them, so the multi BFS takes C5's 1,024-entry expand
    # slices (MvGeom::XT = 1,024, chosen at >= 512 coarse bins; gs_bfs_multi.hip mv_geometry)
    "c5_multi_wide": (40_000, C5_SLOTS, gs.GS_BFS_MULTI, {"GS_MV_BSC": "6"}),
}


@pytest.mark.parametrize("case", list(SWEEP_CASES))
def test_c4_sweep_semantics_match_oracle_100k(case, monkeypatch):
    """BASELINE C4's semantics at 100k nodes against the oracle, through the production
    round (gs_round: the BFS, k_cg_consume, k_cg_prune, the statistics kernels), with the
    sweep values as slots of ONE engine: fail fractions 0.3 / 0.1 / 0.5 at when-to-fail 0
    (gossip_main.rs:449-452; Cluster::fail_nodes gossip.rs:756-771; a failed peer burns its
    fanout slot, gossip.rs:527-541), thresholds 0.05 .. 0.40 and min-ingress 1 / 2 / 3
    (ReceivedCache::prune, received_cache.rs:100-131), two origins. One oracle sim per slot
    holds the engine's active sets (p = 0). For 22 rounds, through the first prune wave:
    failed sets, hops, inbound (src, hop) lists, prunes, counters, prune state, received
    caches and the per-round summaries' integer fields. The c5 case runs C5's slot shape
    (eight distinct origins) through the multi BFS's wide-geometry paths at 40k nodes."""
    n, slots, mode, env = SWEEP_CASES[case]
    sweep_vs_oracle(n, slots, mode, env, monkeypatch)


def test_c4_slots_match_oracle_large(monkeypatch):
    """Whole rounds at the north star's size: BASELINE C4's network with two of its
    13 sweep sims as the slots of one engine -- fail-nodes 0.3 (when-to-fail 0) and
    prune-stake threshold 0.40 -- through gs_round (the production path: the multi-source
    BFS, its gather, k_cg_consume, k_cg_prune, the statistics kernels) for 22 rounds, through
    the first prune wave, against two oracle sims that hold the engine's active sets and run
    the reference's rounds themselves (gossip.rs:494-737, received_cache.rs:38-131): failed
    sets, hops, inbound (src, hop) lists, prunes, counters, prune state, received caches (every
    fourth round and the wave) and the round summaries' integers.
    N: GS_ORACLE_C4_N, default 200,000. The oracle (maps keyed by 32-byte pubkeys, one
    thread per sim) costs ~45 us per node and round, so at C4's 1M nodes the 22 rounds take
    ~17 min: more than the whole `-m gpu` step; the 1M run (GS_ORACLE_C4_N=1000000) is
    committed under profiles/r06/ (DESIGN 3). The engine runs the same persistent BFS at both
    sizes (one launch, 256 workgroups that own interleaved fine bins)."""
    n = int(os.environ.get("GS_ORACLE_C4_N", "200000"))
    slots = [(1, 0.3, 0.15, 2), (1, 0.0, 0.40, 2)]
    sweep_vs_oracle(n, slots, gs.GS_BFS_MULTI, {}, monkeypatch, full_every=4)


def test_rounds_with_rotation_match_oracle_100k(monkeypatch):
    """Rotation inside whole-round parity at 100k nodes: rotation probability 0.002 (about 200
    nodes rotate per round), so after the first prune wave rotated entries drop the replaced
    ring slot's prune filter while the retained peers keep theirs (Cluster::chance_to_rotate
    gossip.rs:739-754 -> PushActiveSet::rotate push_active_set.rs:153-187: the new key gets a
    fresh filter, shift_remove_index(0) drops the oldest key's). The oracle sims get the
    engine's active sets once (after initialize_gossip) and then rotate on their own (the
    same Philox DECIDE / ROTATE streams, the determinism contract); the engine runs gs_round
    (multi BFS, rotation fused into one launch above 16K nodes, the deferred prune-bit clear).
    Two slots (a failure slot, a threshold slot), 24 rounds: everything the sweep test
    compares, plus the active sets of every rotated node each round."""
    slots = [(1, 0.1, 0.15, 2), (2, 0.0, 0.30, 3)]
    sweep_vs_oracle(100_000, slots, gs.GS_BFS_MULTI, {}, monkeypatch, rounds=24, p=0.002, check_rotation=True)


def sweep_vs_oracle(n, slots, mode, env, monkeypatch, rounds=22, p=0.0, full_every=5, check_rotation=False):
    """One engine with `slots` = [(origin stake rank, fail fraction, threshold, min-ingress)]
    run by gs_round against one oracle sim per slot (see the tests above)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    seed, asz = 0x5EED0011, 12
    st = eb.synth.power_law_stakes(n)
    rank_order = np.lexsort((np.arange(n), -st.astype(np.float64)))
    S = len(slots)
    origins = [int(rank_order[r - 1]) for r, _, _, _ in slots]
    fr = [f for _, f, _, _ in slots]
    thr = [t for _, _, t, _ in slots]
    mi = [m for _, _, _, m in slots]
    eng = gs.Engine(st, S, rotation_probability=p, seed=seed, bfs_mode=mode, active_set_size=asz)
    for k in env:
        monkeypatch.delenv(k)
    if "GS_MV_BSC" in env:
        assert eng.bfs_geometry()["expand_slice"] == 1024, eng.bfs_geometry()
    eng.set_slots(origins, mi, thr)
    eng.init_active_sets()
    peers, lens = eng.active_sets()
    pks = stand_in_pubkeys(n)

    def make_sim(k):
        s = ob.Sim(ob.PHILOX, seed, pks, st, 6)
        s.set_entries(peers, lens)
        assert s.fail_nodes(fr[k]) == int(fr[k] * n)  # when-to-fail 0: before the first BFS
        return s

    with ThreadPoolExecutor(max_workers=S) as ex:
        sims = list(ex.map(make_sim, range(S)))
    if not check_rotation:
        del peers, lens
    eng.fail_nodes(fr)
    for k, s in enumerate(sims):
        np.testing.assert_array_equal(eng.failed(k), s.failed(), err_msg=f"failed set slot {k}")
    pruned_total = [0] * S
    rotated_pruned = 0  # rotated entries whose node held prune state (the filter rule ran)

    def oracle_round(k, r, full):  # the reference's round for slot k (the C calls release the GIL)
        s, o = sims[k], origins[k]
        s.run_gossip(o)
        w = {"mn": s.rmr_mn(), "stranded": len(s.stranded()), "dist": s.distances(), "orders": s.orders_all(64 * n)}
        s.consume_messages(o)  # (send_prunes adds the prunes to RMR's m: read above)
        s.send_prunes(o, thr[k], mi[k])
        w["prunes"] = s.prunes()
        if full:
            w["caches"] = s.caches(o)
        s.prune_connections()
        w["counters"] = s.counters()
        if p > 0:
            w["pruned_before_rotation"] = s.pruned_all(o)
            s.chance_to_rotate(asz, p, r)
        w["pruned"] = s.pruned_all(o)
        return w

    with ThreadPoolExecutor(max_workers=S) as ex:
        for r in range(rounds):
            print(f"sweep_vs_oracle n={n} slots={S} p={p}: round {r}", flush=True)  # (progress, pytest -s)
            full = r % full_every == 0 or 18 <= r <= 20 or r == rounds - 1
            futs = [ex.submit(oracle_round, k, r, full) for k in range(S)]
            eng.round(r, record=True)
            summ_r = eng.summaries()[r]
            for k in range(S):
                w = futs[k].result()
                np.testing.assert_array_equal(eng.distances(k), w["dist"], err_msg=f"hops slot {k} round {r}")
                w_off, w_src, w_hop = w["orders"]
                off, src, hop = eng.inbound(k, cap=len(w_src) + 1)
                np.testing.assert_array_equal(off, w_off, err_msg=f"in-degrees slot {k} round {r}")
                np.testing.assert_array_equal(src[:len(w_src)], w_src, err_msg=f"inbound sources slot {k} round {r}")
                np.testing.assert_array_equal(hop[:len(w_hop)], w_hop, err_msg=f"inbound hops slot {k} round {r}")
                del off, src, hop, w_off, w_src, w_hop
                pruned_total[k] += len(w["prunes"])
                assert eng.prunes(k) == w["prunes"], f"prunes slot {k} round {r}"
                if full:
                    up, ln, keys, sc = eng.caches(k)
                    oup, oln, okeys, osc = w["caches"]
                    has = oup != 0xFFFFFFFF
                    np.testing.assert_array_equal(up[has], oup[has], err_msg=f"upserts slot {k} round {r}")
                    np.testing.assert_array_equal(up[~has], 0)
                    np.testing.assert_array_equal(ln, oln, err_msg=f"cache lengths slot {k} round {r}")
                    np.testing.assert_array_equal(keys, okeys, err_msg=f"cache keys slot {k} round {r}")
                    np.testing.assert_array_equal(sc, osc, err_msg=f"cache scores slot {k} round {r}")
                    del up, ln, keys, sc, oup, oln, okeys, osc, has
                eg, ig, pr = eng.counters(k)
                oe, oi, op = w["counters"]
                np.testing.assert_array_equal(eg, np.where(oe == U64MAX, 0, oe), err_msg=f"egress slot {k} round {r}")
                np.testing.assert_array_equal(ig, np.where(oi == U64MAX, 0, oi), err_msg=f"ingress slot {k} round {r}")
                np.testing.assert_array_equal(pr, op, err_msg=f"prune-sent slot {k} round {r}")
                # (after the round's rotation: replaced ring slots' bits are dropped)
                np.testing.assert_array_equal(eng.pruned_all(k), w["pruned"], err_msg=f"prune state slot {k} round {r}")
                # the round summary's integers (gossip_main.rs:480-563): RMR m / n, stranded, prunes
                m_, n_ = w["mn"]
                sm = summ_r[k]
                assert int(sm["pushes"]) == m_ and int(sm["visited"]) == n_, (k, r, sm, m_, n_)
                assert int(sm["stranded"]) == w["stranded"], (k, r)
                assert int(sm["prunes"]) == len(w["prunes"]), (k, r)
                if check_rotation and k == 0:
                    p2, l2 = eng.active_sets()
                    chg = np.nonzero((p2 != peers).any(axis=(1, 2)) | (l2 != lens).any(axis=1))[0]
                    for v in chg[:64].tolist():  # the rotated nodes' entries equal the oracle's
                        for b in range(25):
                            want = sims[0].entry(v, b)
                            np.testing.assert_array_equal(p2[v, b, :l2[v, b]], want,
                                                          err_msg=f"entry ({v}, {b}) after round {r}")
                    rotated_pruned += int(np.count_nonzero(w["pruned_before_rotation"][chg]))
                    peers, lens = p2, l2
    assert all(x > 0 for x in pruned_total), pruned_total  # every slot went through a prune wave
    if check_rotation:
        assert rotated_pruned > 0, "no rotated node held prune state"
    eng.close()
