"""GPU parity: the HIP engine (through the C ABI) against the oracle.

Bit-exact integer comparisons throughout: hops, inbound (src, hop) lists,
prune sets, received caches, prune state, active sets, counters, per-round
summaries and the final f64 statistics.
"""
import json
import os

import numpy as np
import pytest

import engine_bind as eb
import oracle_bind as ob

gs = eb.gs
pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
U64MAX = np.uint64(2**64 - 1)
# GS_BFS_HYBRID (gs_bfs_hybrid.hip, opt-in, never picked by AUTO: DESIGN 5.4) keeps one
# oracle test of its own (test_hybrid_bfs_round_by_round_parity) instead of a column of this matrix
MODES = [gs.GS_BFS_WORKGROUP, gs.GS_BFS_LEVEL, gs.GS_BFS_BINNED, gs.GS_BFS_MULTI]


def ekw(mode):
    """Engine kwargs of a BFS mode; small binned engines bin every level (else the
    hybrid hands levels below 2^17 frontier pairs to the level kernel)."""
    return dict(bfs_mode=mode, binned_all_levels=mode == gs.GS_BFS_BINNED)


# ------------------------------------------------------------ reference KATs ----
def six_node():
    d = json.load(open(os.path.join(HERE, "golden", "six_node_cluster.json")))
    pks = [bytes.fromhex(h) for h in d["pubkeys_hex"]]
    ids = gs.ids_from_pubkeys(pks)  # pubkey-order index -> node id (base58 rank)
    stakes_by_id = np.zeros(6, dtype=np.uint64)
    for i, s in enumerate(d["stakes"]):
        stakes_by_id[ids[i]] = s
    return d, ids, stakes_by_id


def upload_entries(eng, d, ids):
    for n, ks in d["entries"].items():
        for k, peers in ks.items():
            if peers:
                eng.set_entry(ids[int(n)], int(k), [ids[p] for p in peers])


@pytest.mark.parametrize("mode", MODES)
def test_mst_kat_on_gpu(mode):
    """gossip.rs test_mst (1040-1163) through the HIP BFS."""
    d, ids, st = six_node()
    eng = gs.Engine(st, 1, fanout=2, active_set_size=12, rotation_probability=0.2, seed=1, **ekw(mode))
    upload_entries(eng, d, ids)
    eng.set_slots([ids[5]])
    eng.run_gossip()
    dist = eng.distances(0)
    assert [int(dist[ids[i]]) for i in range(6)] == d["expect_distances"]
    lists = eng.inbound_lists(0)
    inv = {v: k for k, v in enumerate(ids)}
    assert [len(lists[ids[i]]) for i in range(5)] == d["expect_num_inbound"]
    assert lists[ids[5]] == []  # the origin never receives (orders has no key for it)
    for dest, src, hop in d["expect_hops"]:
        got = {inv[s]: h for s, h in lists[ids[dest]]}
        assert got[src] == hop
    e, i, p = eng.counters(0)
    assert int(i.sum()) == int(e.sum()) == sum(d["expect_num_inbound"])
    # the MST asserts of test_mst (gossip.rs:1136-1155): first discoverers in FIFO order
    mst = {inv[u]: sorted(inv[v] for v in vs) for u, vs in eng.mst(0).items()}
    assert mst == {5: [2, 4], 4: [0, 3], 0: [1]}
    # the debug dumps (gossip.rs:365-431) print these records
    import io
    import gossip_sim_amd.dumps as dumps
    keys = [f"K{inv[v]}" for v in range(6)]
    buf = io.StringIO()
    dumps.print_mst(eng, 0, keys, out=buf)
    dumps.print_pushes(eng, 0, keys, out=buf)
    dumps.print_hops(eng, 0, keys, out=buf)
    dumps.print_node_orders(eng, 0, keys, out=buf)
    lines = buf.getvalue().splitlines()
    assert all(" INFO  gossip_sim::gossip] " in ln for ln in lines)
    msgs = [ln.split("] ", 1)[1] for ln in lines]
    assert msgs[0] == "MST: "
    i5 = msgs.index("##### src: K5 #####")
    assert sorted(msgs[i5 + 1:i5 + 3]) == ["dest: K2", "dest: K4"]
    assert "PUSHES: " in msgs and "DISTANCES FROM ORIGIN" in msgs and "NODE ORDERS" in msgs
    assert "dest node, hops: (K5, 0)" in msgs
    n_push = sum(len(v) for v in eng.pushes(0).values())
    assert sum(1 for m in msgs if m.startswith("Dest: ")) == n_push == sum(d["expect_num_inbound"])


@pytest.mark.parametrize("mode", MODES)
def test_pruning_kat_on_gpu(mode):
    """gossip_main.rs test_pruning (1071-1163): no prunes before iteration 19, then {3->M, M->h, j->P}."""
    d, ids, st = six_node()
    eng = gs.Engine(st, 1, fanout=2, active_set_size=12, rotation_probability=0.2, seed=1, **ekw(mode))
    upload_entries(eng, d, ids)
    eng.set_slots([ids[5]], min_ingress=2, thresholds=0.15)
    inv = {v: k for k, v in enumerate(ids)}
    for it in range(21):
        eng.run_gossip()
        assert (eng.hops(0) != 0xFF).sum() == 6
        eng.consume_messages()
        eng.send_prunes()
        prunes = sorted((inv[a], inv[b]) for a, b in eng.prunes(0))
        if it <= 18:
            assert prunes == []
        if it == 19:
            assert prunes == sorted(tuple(x) for x in d["expect_prunes_iteration_19"])
        eng.prune_connections()
        eng.chance_to_rotate(it)


# ------------------------------------------------------ Philox-mode parity ----
def make_pair(n, origin_ranks, *, asz=12, fanout=6, p=0.013333, seed=7, thr=0.15, mi=2, mode=gs.GS_BFS_AUTO,
              extra=None, stakes=None):
    pks, st = eb.synth.network(n)
    if stakes is not None:
        st = np.ascontiguousarray(stakes, dtype=np.uint64)
    S = len(origin_ranks)
    eng = gs.Engine(st, S, fanout=fanout, active_set_size=asz, rotation_probability=p, seed=seed,
                    **{**ekw(mode), **(extra or {})})
    sims = [ob.Sim(ob.PHILOX, seed, pks, st, fanout) for _ in range(S)]
    origins = [sims[0].find_nth_largest(r) for r in origin_ranks]
    eng.set_slots(origins, mi, thr)
    eng.init_active_sets()
    for s in sims:
        s.init_philox(asz)
    return eng, sims, origins, st


def assert_entries(eng, sim, asz):
    gp, gl = eng.active_sets()
    op, ol = sim.entries(asz)
    np.testing.assert_array_equal(gl, ol)
    np.testing.assert_array_equal(np.where(gp == 0xFFFFFFFF, 0, gp), np.where(op == 0xFFFFFFFF, 0, op))


@pytest.mark.parametrize("n,asz", [(300, 12), (200, 5), (64, 32), (9, 12), (14, 12)])
def test_init_active_sets_parity(n, asz):
    """gs_init_active_sets == PushActiveSet::rotate from empty entries (incl. N-1 <= size)."""
    eng, sims, _, _ = make_pair(n, [1], asz=asz)
    assert_entries(eng, sims[0], asz)


def run_parity(n, ranks, rounds, *, p, mode, thr=0.15, mi=2, asz=12, fanout=6, fail_at=None, fractions=None,
               full_every=5, extra=None, stakes=None):
    eng, sims, origins, st = make_pair(n, ranks, asz=asz, fanout=fanout, p=p, thr=thr, mi=mi, mode=mode, extra=extra,
                                       stakes=stakes)
    thr_v = np.broadcast_to(np.asarray(thr, dtype=float), (len(ranks),))
    mi_v = np.broadcast_to(np.asarray(mi), (len(ranks),))
    total_prunes = 0
    for r in range(rounds):
        if fail_at is not None and r == fail_at:
            eng.fail_nodes(fractions)
            for s, f in zip(sims, fractions):
                s.fail_nodes(f)
            for k, s in enumerate(sims):
                np.testing.assert_array_equal(eng.failed(k), s.failed())
        eng.run_gossip()
        for k, (s, o) in enumerate(zip(sims, origins)):
            s.run_gossip(o)
            np.testing.assert_array_equal(eng.distances(k), s.distances(), err_msg=f"hops slot {k} round {r}")
            lists = eng.inbound_lists(k)
            for v in range(n):
                want = s.orders(v)
                assert lists[v] == ([] if want is None else want), f"inbound slot {k} node {v} round {r}"
            if r % full_every == 0:  # Cluster::mst (FIFO first discoverers) and Cluster::pushes
                mst, pushes = eng.mst(k), eng.pushes(k)
                for u in range(n):
                    want = s.mst(u)
                    assert mst.get(u) == (sorted(want) if want else None), f"mst slot {k} src {u} round {r}"
                    assert pushes.get(u, []) == sorted(s.pushes(u) or []), f"pushes slot {k} src {u} round {r}"
        eng.consume_messages()
        eng.send_prunes()
        for k, (s, o) in enumerate(zip(sims, origins)):
            s.consume_messages(o)
            s.send_prunes(o, float(thr_v[k]), int(mi_v[k]))
            assert eng.prunes(k) == s.prunes(), f"prunes slot {k} round {r}"
            total_prunes += len(s.prunes())
            if r % full_every == 0 or r == rounds - 1:
                up, ln, keys, sc = eng.caches(k)
                oup, oln, okeys, osc = s.caches(o)
                has = oup != 0xFFFFFFFF
                np.testing.assert_array_equal(up[has], oup[has])
                np.testing.assert_array_equal(up[~has], 0)
                np.testing.assert_array_equal(ln, oln)
                np.testing.assert_array_equal(keys, okeys)
                np.testing.assert_array_equal(sc, osc)
        eng.prune_connections()
        for k, (s, o) in enumerate(zip(sims, origins)):
            s.prune_connections()
            e, i, pr = eng.counters(k)
            oe, oi, op = s.counters()
            np.testing.assert_array_equal(e, np.where(oe == U64MAX, 0, oe))
            np.testing.assert_array_equal(i, np.where(oi == U64MAX, 0, oi))
            np.testing.assert_array_equal(pr, op)
            np.testing.assert_array_equal(eng.pruned_all(k), s.pruned_all(o), err_msg=f"prune state round {r}")
        eng.chance_to_rotate(r)
        for s in sims:
            s.chance_to_rotate(asz, p, r)
        if r % full_every == 0 or r == rounds - 1:
            assert_entries(eng, sims[0], asz)
            for k, (s, o) in enumerate(zip(sims, origins)):
                np.testing.assert_array_equal(eng.pruned_all(k), s.pruned_all(o))
    return total_prunes


@pytest.mark.parametrize("mode", MODES)
def test_round_by_round_parity(mode):
    """Every step of 45 rounds, 5 origins, heavy rotation: state identical to the oracle."""
    total = run_parity(240, [1, 2, 7, 60, 240], 45, p=0.08, mode=mode, full_every=4)
    assert total > 0  # the ~20-round prune waves were exercised


def test_hybrid_bfs_round_by_round_parity():
    """GS_BFS_HYBRID (opt-in push-graph BFS): the 45-round oracle comparison, and
    the same with every level through its grid kernels."""
    assert run_parity(240, [1, 2, 7, 60, 240], 45, p=0.08, mode=gs.GS_BFS_HYBRID, full_every=4) > 0
    assert run_parity(240, [1, 2, 7, 60, 240], 45, p=0.08, mode=gs.GS_BFS_HYBRID, full_every=9,
                      extra=dict(no_small_levels=True)) > 0


@pytest.mark.parametrize("mode,extra", [
    (gs.GS_BFS_MULTI, dict(no_small_levels=True)),      # every level through k_mv_expand / k_mv_apply
    (gs.GS_BFS_BINNED, dict(binned_all_levels=False)),  # k_bin_small + the direct levels (the default hybrid)
    (gs.GS_BFS_BINNED, dict(binned_all_levels=False, no_small_levels=True)),  # every level direct, grid-wide
    (gs.GS_BFS_BINNED, dict(wide_records=True)),        # every level binned, 8-byte records
])
def test_round_by_round_parity_level_kernels(mode, extra):
    """The same 45 rounds with the grid-wide level kernels (or the small-level kernels) that
    the default small-network paths skip, each directly against the oracle."""
    total = run_parity(240, [1, 2, 7, 60, 240], 45, p=0.08, mode=mode, full_every=4, extra=extra)
    assert total > 0


@pytest.mark.parametrize("mode", [gs.GS_BFS_BINNED, gs.GS_BFS_MULTI])
def test_parity_hub_in_degrees_above_64(mode):
    """Fanout = active-set size 32 on 500 nodes whose stakes halve every 8 stake ranks (buckets
    24 down to 0; stake ranks shuffled over the ids), inbound capacity 256: the top-stake nodes sit in most high-bucket
    entries and receive 65-83 pushes a round -- the binned gather's whole-wave rows for
    pairs above G_HEAVY = 64 records, the consume's single-lane path above 64 -- every
    level binned; against the oracle round by round. (The binned gather's fallback for a
    step with more than half its pairs heavy cannot occur: that needs a mean in-degree
    above 32 >= fanout.)"""
    n = 500
    st = np.maximum(2.0 ** (54 - np.arange(n) / 8.0), 1e9).astype(np.uint64)
    st = st[np.random.default_rng(5).permutation(n)]  # hubs spread over the ids (and the multi BFS's fine bins)
    extra = dict(inbound_capacity=256, binned_all_levels=mode == gs.GS_BFS_BINNED)
    eng, sims, origins, _ = make_pair(n, [1], asz=32, fanout=32, p=0.05, mode=mode, extra=extra, stakes=st)
    eng.run_gossip()
    _, ing, _ = eng.counters(0)
    assert int((ing > 64).sum()) >= 5, int(ing.max())
    eng.close()
    run_parity(n, [1, 2, 40], 22, p=0.05, mode=mode, asz=32, fanout=32, full_every=7, extra=extra, stakes=st)


@pytest.mark.parametrize("mode", [gs.GS_BFS_LEVEL, gs.GS_BFS_BINNED, gs.GS_BFS_MULTI])
def test_parity_sweep_params_and_failures(mode):
    """Per-slot thresholds / min-ingress and fail-nodes (failed peers burn fanout slots)."""
    run_parity(180, [1, 3, 5, 9], 42, p=0.03, mode=mode, thr=[0.0, 0.15, 0.4, 1.0], mi=[0, 2, 3, 1],
               fail_at=2, fractions=[0.1, 0.2, 0.3, 0.5], full_every=6)


def test_parity_small_fanout_and_asz():
    run_parity(150, [1, 4], 30, p=0.05, mode=gs.GS_BFS_WORKGROUP, asz=7, fanout=3, full_every=5)


def test_rotation_round_sequence_and_deferred_clear():
    """Rotations at repeated / skipped round indices (the rotation counters alternate by
    round parity), and the one-kernel round's deferred prune-bit clear (applied inside
    the next round kernel, or flushed before a step call or readback): active sets and
    prune state stay identical to the oracle's."""
    n, asz, p = 220, 12, 0.25
    eng, sims, origins, st = make_pair(n, [1, 9, 50], asz=asz, p=p, mode=gs.GS_BFS_WORKGROUP)
    assert eng.info()["fused_round"]

    def oracle_round(r, rotate_round):
        for s, o in zip(sims, origins):
            s.run_gossip(o)
            s.consume_messages(o)
            s.send_prunes(o, 0.15, 2)
            s.prune_connections()
            s.chance_to_rotate(asz, p, rotate_round)

    seq = [0, 1, 1, 4, 5, 5, 6, 9, 10, 11, 12, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26]
    for i, r in enumerate(seq):
        if i % 3 == 2:  # step-wise iteration: flushes the fused round's pending clear first
            eng.run_gossip(); eng.consume_messages(); eng.send_prunes(); eng.prune_connections()
            eng.chance_to_rotate(r)
        else:
            eng.round(r)
        oracle_round(r, r)
        if i % 4 == 3 or i == len(seq) - 1:
            assert_entries(eng, sims[0], asz)
            for k, (s, o) in enumerate(zip(sims, origins)):
                np.testing.assert_array_equal(eng.pruned_all(k), s.pruned_all(o), err_msg=f"iteration {i}")
                np.testing.assert_array_equal(eng.distances(k), s.distances())


@pytest.mark.parametrize("mode,narrow", [(gs.GS_BFS_LEVEL, False), (gs.GS_BFS_BINNED, False),
                                         (gs.GS_BFS_LEVEL, True), (gs.GS_BFS_BINNED, True),
                                         (gs.GS_BFS_MULTI, False), (gs.GS_BFS_MULTI, True)])
def test_fused_round_matches_steps(mode, narrow):
    """gs_round's step-kernel path (consume + prune + apply of gs_consume_g.hip: register,
    wave and serial consume paths, register and wave prune paths) == the step-by-step
    calls (the generic per-pair kernels). thresholds 0 / min-ingress 0 make prunes long."""
    pks, st = eb.synth.network(260)
    a = gs.Engine(st, 4, seed=3, rotation_probability=0.05, narrow_wave_path=narrow, **ekw(mode))
    b = gs.Engine(st, 4, seed=3, rotation_probability=0.05, **ekw(mode))
    for e in (a, b):
        e.set_slots([0, 10, 100, 200], [2, 0, 2, 1], [0.15, 0.0, 0.5, 0.05])
        e.init_active_sets()
    for r in range(30):
        a.round(r, record=r >= 10)
        b.run_gossip(); b.consume_messages(); b.send_prunes(); b.prune_connections(); b.chance_to_rotate(r)
        if r >= 10:
            b.record_round()
    for k in range(4):
        np.testing.assert_array_equal(a.hops(k), b.hops(k))
        np.testing.assert_array_equal(a.pruned_all(k), b.pruned_all(k))
        for x, y in zip(a.caches(k), b.caches(k)):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(a.accumulators(k), b.accumulators(k)):
            np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.summaries(), b.summaries())


def test_rotation_ahead_matches_serial_rotation(monkeypatch):
    """The one-kernel round with its rotation run ahead in the round kernel's workgroup 0 on
    a second row buffer (round 5, the default) == the same engine with GS_ROT_AHEAD=0 (a
    rotation launch after each round), through the state changes the double buffer must
    survive: consecutive rounds, a repeated round parity (serial fallback), step-wise calls
    including a step rotation, an uploaded entry, and ahead rounds again. Rotation
    probability 0.2 so that ~80 of 400 nodes rotate per round."""
    pks, st = eb.synth.network(400)
    engs = []
    for ahead in (True, False):
        if ahead:
            monkeypatch.delenv("GS_ROT_AHEAD", raising=False)
        else:
            monkeypatch.setenv("GS_ROT_AHEAD", "0")
        e = gs.Engine(st, 5, seed=11, rotation_probability=0.2, bfs_mode=gs.GS_BFS_WORKGROUP)
        e.set_slots([0, 3, 50, 150, 399], [2, 0, 2, 1, 2], [0.15, 0.0, 0.5, 0.05, 0.15])
        e.init_active_sets()
        engs.append(e)
    monkeypatch.delenv("GS_ROT_AHEAD", raising=False)

    def both(f):
        for e in engs:
            f(e)

    for r in range(8):
        both(lambda e: e.round(r, record=r >= 2))
    both(lambda e: e.round(9, record=True))   # same parity as round 7: serial fallback
    both(lambda e: e.round(10, record=True))
    both(lambda e: (e.run_gossip(), e.consume_messages(), e.send_prunes(), e.prune_connections(),
                    e.chance_to_rotate(11)))  # step-wise, with an in-place rotation
    for r in range(12, 16):
        both(lambda e: e.round(r, record=True))
    peers = engs[1].get_entry(7, 3)
    both(lambda e: e.set_entry(7, 3, peers[::-1]))  # an uploaded entry (rows change in place)
    for r in range(16, 24):  # through the first prune wave
        both(lambda e: e.round(r, record=True))
    a, b = engs
    pa, la = a.active_sets()
    pb, lb = b.active_sets()
    np.testing.assert_array_equal(la, lb)
    np.testing.assert_array_equal(pa, pb)
    for k in range(5):
        np.testing.assert_array_equal(a.hops(k), b.hops(k))
        np.testing.assert_array_equal(a.pruned_all(k), b.pruned_all(k))
        for x, y in zip(a.caches(k), b.caches(k)):
            np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.summaries(), b.summaries())
    assert a.info()["bfs_mode"] == b.info()["bfs_mode"]


@pytest.mark.parametrize("narrow", [False, True])
def test_multi_fused_gather_consume_matches_steps(narrow, monkeypatch):
    """GS_MV_FUSED=1: the multi-source BFS's gs_round consumes straight from the gather's
    LDS CSR (k_mv_consume: register, wave and serial paths with narrow bounds) -- equal
    to the step-by-step calls, as the default gather + k_cg_consume round is."""
    monkeypatch.setenv("GS_MV_FUSED", "1")
    pks, st = eb.synth.network(260)
    a = gs.Engine(st, 4, seed=3, rotation_probability=0.05, narrow_wave_path=narrow, bfs_mode=gs.GS_BFS_MULTI)
    monkeypatch.delenv("GS_MV_FUSED")
    b = gs.Engine(st, 4, seed=3, rotation_probability=0.05, bfs_mode=gs.GS_BFS_MULTI)
    for e in (a, b):
        e.set_slots([0, 10, 100, 200], [2, 0, 2, 1], [0.15, 0.0, 0.5, 0.05])
        e.init_active_sets()
    for r in range(30):
        a.round(r, record=r >= 10)
        b.run_gossip(); b.consume_messages(); b.send_prunes(); b.prune_connections(); b.chance_to_rotate(r)
        if r >= 10:
            b.record_round()
    for k in range(4):
        np.testing.assert_array_equal(a.hops(k), b.hops(k))
        np.testing.assert_array_equal(a.pruned_all(k), b.pruned_all(k))
        for x, y in zip(a.caches(k), b.caches(k)):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(a.accumulators(k), b.accumulators(k)):
            np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(a.summaries(), b.summaries())


# --------------------------------------------------------- whole simulation ----
F64_NAMES = ["coverage", "rmr", "branching", "hop_mean", "hop_median", "coverage_stats", "rmr_stats",
             "branching_stats", "aggregate_hops", "ldh", "stranded", "stranded_round_mean", "stranded_round_median"]
U64_NAMES = ["origin", "hop_max", "hop_min", "aggregate_hops", "ldh", "stranded", "stranded_times",
             "stranded_round_count", "stranded_round_max", "stranded_round_min", "hops_hist", "stranded_hist",
             "egress_hist", "ingress_hist", "prune_hist", "egress_cpb", "validator_hist", "hist_errors",
             "failed_count"]


def compare_sim(n, *, ranks, iterations, warm, test_type=0, fractions=None, thresholds=None, min_ingress=None, **kw):
    pks, st = eb.synth.network(n)
    res = gs.run_simulations(st, n_sims=len(ranks), origin_ranks=ranks, iterations=iterations, warm_up=warm,
                             test_type=test_type, fractions=fractions, thresholds=thresholds,
                             min_ingress=min_ingress, **kw)
    for k, rank in enumerate(ranks):
        okw = dict(kw)
        if fractions is not None:
            okw["fraction_to_fail"] = fractions[k]
        if thresholds is not None:
            okw["thr"] = thresholds[k]
        if min_ingress is not None:
            okw["min_ingress"] = min_ingress[k]
        okw.pop("bfs_mode", None)
        o = ob.run_simulation(pks, st, origin_rank=rank, iterations=iterations, warm_up=warm, test_type=test_type,
                              **okw)
        for name in F64_NAMES:
            np.testing.assert_array_equal(res.f64(k, name), o.f64(name), err_msg=f"sim {k} {name}")
        for name in U64_NAMES:
            np.testing.assert_array_equal(res.u64(k, name), o.u64(name), err_msg=f"sim {k} {name}")


def test_simulation_stats_parity_origin_rank_sweep():
    compare_sim(300, ranks=[1, 2, 3], iterations=70, warm=20, seed=11, p=0.02)


def test_simulation_stats_parity_fail_nodes():
    compare_sim(250, ranks=[1, 1, 1], iterations=50, warm=10, test_type=5, fractions=[0.1, 0.25, 0.4],
                when_to_fail=5, seed=5, bfs_mode=gs.GS_BFS_LEVEL)


def test_simulation_stats_parity_threshold_sweep():
    compare_sim(220, ranks=[1, 1, 1], iterations=45, warm=5, thresholds=[0.05, 0.2, 0.6], min_ingress=[2, 1, 4],
                seed=9)


# ---------------------------------------------------- size-independent checks ----
def test_large_network_invariants():
    """N = 200k, level-synchronous BFS: properties that hold at any size."""
    n = 200_000
    st = eb.synth.power_law_stakes(n)  # id order is irrelevant to these invariants
    eng = gs.Engine(st, 2, seed=21, bfs_mode=gs.GS_BFS_LEVEL)
    eng.set_slots([0, n // 2])
    eng.init_active_sets()
    for r in range(3):
        eng.round(r, record=True)
    peers, lens = eng.active_sets()
    assert (lens == 12).all()
    srt = np.sort(peers, axis=2)
    assert (np.diff(srt.astype(np.int64), axis=2) != 0).all()  # no duplicate peers in an entry
    assert (peers != np.arange(n, dtype=np.uint32)[:, None, None]).all()  # never yourself
    summ = eng.summaries()
    for k in range(2):
        hops = eng.hops(k)
        off, src, hop = eng.inbound(k, cap=8 * n)
        e, i, _ = eng.counters(k)
        assert int(i.sum()) == int(e.sum()) == int(off[-1]) == int(summ[-1, k]["pushes"])
        assert int((hops != 0xFF).sum()) == int(summ[-1, k]["visited"])
        # BFS: every reached non-origin node has an inbound record from hop-1, each record's hop is src hop + 1
        h = hops.astype(np.int64)
        dest = np.repeat(np.arange(n), np.diff(off).astype(np.int64))
        assert (hop.astype(np.int64)[:off[-1]] == h[src[:off[-1]]] + 1).all()
        first = hop[off[:-1][np.diff(off) > 0]]
        reached = np.diff(off) > 0
        assert (first.astype(np.int64) == h[reached]).all()
        assert (dest >= 0).all()


@pytest.mark.parametrize("all_levels,wide,mispredict", [(False, False, False), (True, False, False),
                                                        (True, True, False), (False, False, True),
                                                        (True, False, True)])
def test_binned_bfs_matches_level_bfs_large(all_levels, wide, mispredict):
    """N = 300k, 3 slots, a fail-nodes fraction: the propagation-blocked BFS (hybrid
    with the direct kernel for small levels, or binned throughout; 4- or 8-byte
    records) gives the level BFS's hops, in-degrees, inbound sets, counters and
    summaries. `mispredict`: the predicted level loop inverts its binned/direct choice
    every other round, so levels of >= 2^17 pairs run direct while the previous round's
    pool runs (Lt) are still in memory -- the gather must take only this round's binned
    levels."""
    n = 300_000
    st = eb.synth.power_law_stakes(n)
    engs = [gs.Engine(st, 3, seed=33, rotation_probability=0.01, bfs_mode=gs.GS_BFS_LEVEL),
            gs.Engine(st, 3, seed=33, rotation_probability=0.01, bfs_mode=gs.GS_BFS_BINNED,
                      binned_all_levels=all_levels, wide_records=wide, mispredict_levels=mispredict)]
    for e in engs:
        e.set_slots([0, 17, n - 1], [2, 1, 3], [0.15, 0.3, 0.05])
        e.init_active_sets()
        e.fail_nodes([0.0, 0.2, 0.1])
    for r in range(6 if mispredict else 4):
        for e in engs:
            e.round(r, record=r >= 1)
        a, b = engs
        for k in range(3):
            np.testing.assert_array_equal(a.hops(k), b.hops(k))
            offa, srca, hopa = a.inbound(k, cap=8 * n)
            offb, srcb, hopb = b.inbound(k, cap=8 * n)
            np.testing.assert_array_equal(offa, offb)
            np.testing.assert_array_equal(srca, srcb)  # lists come back in consume order
            np.testing.assert_array_equal(hopa, hopb)
            for x, y in zip(a.counters(k), b.counters(k)):
                np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(engs[0].summaries(), engs[1].summaries())
    for k in range(3):
        for x, y in zip(engs[0].accumulators(k), engs[1].accumulators(k)):
            np.testing.assert_array_equal(x, y)


def test_binned_bfs_large_bins_matches_level_bfs():
    """More than 2^24 pairs (1.5M nodes x 12 slots): the binned BFS takes bins of 2^12 pairs,
    8-byte records and the 1,024-thread gather with 160 KB of LDS. Equal to the level BFS
    (hops, counters, summaries)."""
    n, S = 1_500_000, 12
    st = eb.synth.power_law_stakes(n)
    origins = [int(x) for x in np.argsort(-st.astype(np.float64), kind="stable")[:S]]
    engs = [gs.Engine(st, S, seed=41, rotation_probability=0.013333, bfs_mode=m)
            for m in (gs.GS_BFS_LEVEL, gs.GS_BFS_BINNED)]
    for e in engs:
        e.set_slots(origins, 2, [0.05 * (1 + k % 6) for k in range(S)])
        e.init_active_sets()
        e.fail_nodes([0.0, 0.1] * (S // 2))
    for r in range(3):
        for e in engs:
            e.round(r, record=True)
    a, b = engs
    np.testing.assert_array_equal(a.summaries(), b.summaries())
    for k in (0, 5, 11):
        np.testing.assert_array_equal(a.hops(k), b.hops(k))
        for x, y in zip(a.counters(k), b.counters(k)):
            np.testing.assert_array_equal(x, y)
    for e in engs:
        e.close()


# ------------------------------------------- one-kernel workgroup round ----
def run_fused_parity(n, S, rounds, *, fanout=6, asz=12, p=0.02, thr=0.15, mi=2, seed=11, check=(0, 1, 2, 3),
                     fail_at=None, fraction=0.0, full_every=5, narrow=False, origins=None, record_from=3):
    """gs_round's one-kernel workgroup round against the oracle, round by round, on
    `check` slots of an S-slot engine (the other slots run alongside)."""
    pks, st = eb.synth.network(n)
    eng = gs.Engine(st, S, fanout=fanout, active_set_size=asz, rotation_probability=p, seed=seed,
                    bfs_mode=gs.GS_BFS_WORKGROUP, narrow_wave_path=narrow)
    assert eng.info()["fused_round"]
    if origins is None:
        origins = [(k * 37 + 1) % n for k in range(S)]
    eng.set_slots(origins, mi, thr)
    eng.init_active_sets()
    sims = {k: ob.Sim(ob.PHILOX, seed, pks, st, fanout) for k in check}
    for s in sims.values():
        s.init_philox(asz)
    total_prunes, max_in = 0, 0
    for r in range(rounds):
        if fail_at is not None and r == fail_at:
            eng.fail_nodes([fraction] * S)
            for s in sims.values():
                s.fail_nodes(fraction)
        eng.round(r, record=r >= record_from)
        for k, s in sims.items():
            o = origins[k]
            s.run_gossip(o)
            s.consume_messages(o)
            s.send_prunes(o, thr, mi)
            np.testing.assert_array_equal(eng.distances(k), s.distances(), err_msg=f"hops slot {k} round {r}")
            assert eng.prunes(k) == s.prunes(), f"prunes slot {k} round {r}"
            total_prunes += len(s.prunes())
            s.prune_connections()
            e, i, pr = eng.counters(k)
            oe, oi, op = s.counters()
            np.testing.assert_array_equal(e, np.where(oe == U64MAX, 0, oe))
            np.testing.assert_array_equal(i, np.where(oi == U64MAX, 0, oi))
            np.testing.assert_array_equal(pr, op)
            max_in = max(max_in, int(i.max()))
            if r % full_every == 0 or r == rounds - 1:
                up, ln, keys, sc = eng.caches(k)
                oup, oln, okeys, osc = s.caches(o)
                has = oup != 0xFFFFFFFF
                np.testing.assert_array_equal(up[has], oup[has])
                np.testing.assert_array_equal(ln, oln)
                np.testing.assert_array_equal(keys, okeys)
                np.testing.assert_array_equal(sc, osc)
            s.chance_to_rotate(asz, p, r)  # the engine's round ends with the rotation
            if r % full_every == 0 or r == rounds - 1:
                np.testing.assert_array_equal(eng.pruned_all(k), s.pruned_all(o), err_msg=f"prune state {r}")
    return eng, total_prunes, max_in


def test_fused_round_parity():
    """C2-shaped (all-origins batch) fused rounds: 45 rounds across two prune waves."""
    eng, total, _ = run_fused_parity(300, 96, 45, check=(0, 5, 50, 95))
    assert total > 0
    with pytest.raises(gs.GsError):  # inbound records stay on-chip in the fused round
        eng.inbound_lists(0)


def test_fused_round_heavy_paths():
    """fanout = active set = 32 on 150 nodes: in-degrees > 16 (wave path) and > 24
    (ordered single-lane path, narrowed from > 64), cache entries > 32 keys (wave
    prune), failures."""
    eng, total, max_in = run_fused_parity(150, 64, 42, fanout=32, asz=32, p=0.05, thr=0.05, mi=1,
                                          check=(0, 7, 33), fail_at=25, fraction=0.2, full_every=3, narrow=True)
    assert total > 0
    assert max_in > 24


def fused_vs_split(n, S, rounds, *, checks, seed=5, origins=None, **kw):
    pks, st = eb.synth.network(n)
    engines = [gs.Engine(st, S, seed=seed, bfs_mode=gs.GS_BFS_WORKGROUP, split_round=f, **kw) for f in (False, True)]
    assert engines[0].info()["fused_round"] and not engines[1].info()["fused_round"]
    for e in engines:
        e.set_slots(origins if origins is not None else [(k * 5) % n for k in range(S)], 2, 0.15)
        e.init_active_sets()
    for r in range(rounds):
        for e in engines:
            e.round(r, record=r >= 5)
    a, b = engines
    np.testing.assert_array_equal(a.summaries(), b.summaries())
    for k in checks:
        np.testing.assert_array_equal(a.hops(k), b.hops(k))
        np.testing.assert_array_equal(a.pruned_all(k), b.pruned_all(k))
        for x, y in zip(a.caches(k), b.caches(k)):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(a.accumulators(k), b.accumulators(k)):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("n,fanout,asz", [
    (3500, 6, 12),  # > 3,072 nodes: the CSR reloads rows instead of staging the push lists
    (600, 8, 8),    # 8 pushes per lane: register-staged CSR at its widest
    (500, 7, 16),   # fanout > 6: push columns = ring slots, CSR from rows
])
def test_fused_round_matches_split_round_shapes(n, fanout, asz):
    """The one-kernel round's push-list / CSR variants == the split kernels, through a prune wave."""
    fused_vs_split(n, 24, 45, checks=(0, 11, 23), fanout=fanout, active_set_size=asz, rotation_probability=0.03)


def test_fused_round_matches_split_round():
    """One-kernel round == split kernels (WG BFS + consume/prune + stats) incl. summaries."""
    pks, st = eb.synth.network(400)
    engines = [gs.Engine(st, 80, seed=5, rotation_probability=0.03, bfs_mode=gs.GS_BFS_WORKGROUP, split_round=f)
               for f in (False, True)]
    assert engines[0].info()["fused_round"] and not engines[1].info()["fused_round"]
    for e in engines:
        e.set_slots([(k * 5) % 400 for k in range(80)], 2, 0.15)
        e.init_active_sets()
    for r in range(50):
        for e in engines:
            e.round(r, record=r >= 5)
    a, b = engines
    np.testing.assert_array_equal(a.summaries(), b.summaries())
    for k in (0, 13, 79):
        np.testing.assert_array_equal(a.hops(k), b.hops(k))
        np.testing.assert_array_equal(a.pruned_all(k), b.pruned_all(k))
        for x, y in zip(a.caches(k), b.caches(k)):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(a.accumulators(k), b.accumulators(k)):
            np.testing.assert_array_equal(x, y)


# ------------------------------------------------------- BASELINE configs at size ----
C2_SEED = 0x5EED0003  # bench.py's simulation seed


def test_fused_round_parity_c2_size():
    """BASELINE C2 at its real size, on bench.py's own engine: N = 3,000 power-law nodes,
    all 3,000 origins batched (origin of slot s = node s), p = 0.01, seed 0x5EED0003.
    Six slots are compared with the oracle every round through the first prune wave
    (hops, prune sets, counters; caches and prune state every 6 rounds). Every node id
    >= 768 is reached and pushes, so k_round_wg's register-staged CSR runs all of its
    CSR_NPT = 4 iterations per thread (gs_round_wg.hip, nodes 768..3071)."""
    n = 3000
    eng, total, max_in = run_fused_parity(n, n, 28, p=0.01, seed=C2_SEED, origins=list(range(n)),
                                          check=(0, 1, 767, 768, 2047, 2999), full_every=6, record_from=20)
    assert total > 0  # the first prune wave (~round 20) was compared
    assert max_in > 6
    summ = eng.summaries()
    assert summ.shape == (8, n) and int(summ["prunes"].sum()) > 0


def test_fused_round_matches_split_round_c2_size():
    """The same C2 engine, all 3,000 slots: the one-kernel round equals the split kernels
    (workgroup BFS + step consume/prune + stats) for every slot's per-round summaries, and
    hops / prune state / caches / accumulators of sampled slots, through a prune wave."""
    n = 3000
    fused_vs_split(n, n, 26, checks=(0, 768, 1500, 2999), seed=C2_SEED, origins=list(range(n)),
                   rotation_probability=0.01)


@pytest.mark.parametrize("mode", MODES)
def test_simulation_parity_c1(mode):
    """BASELINE C1 as configured: ~1,000-node network, push fanout 6, active-set size 12,
    origin rank 1, 200 warm-up + 100 measured iterations (p 0.013333, min-ingress 2,
    threshold 0.15): gs_run_simulations == the oracle's run_simulation for every result
    array (gossip_main.rs:292-647)."""
    compare_sim(1000, ranks=[1], iterations=300, warm=200, seed=C2_SEED, p=0.013333, bfs_mode=mode)


def _invariants(eng, k, n, summ_last, failed=None):
    """Size-independent properties of one slot's last round (gossip.rs:494-615)."""
    hops = eng.hops(k)
    off, src, hop = eng.inbound(k, cap=32 * n)
    e, i, _ = eng.counters(k)
    E = int(off[-1])
    assert int(i.sum()) == int(e.sum()) == E == int(summ_last["pushes"])
    reached = hops != 0xFF
    assert int(reached.sum()) == int(summ_last["visited"])
    h = hops.astype(np.int64)
    assert (hop.astype(np.int64)[:E] == h[src[:E]] + 1).all()  # orders hop = dist[src] + 1
    has = np.diff(off) > 0
    assert (hop[off[:-1][has]].astype(np.int64) == h[has]).all()  # first arrival sets the hop
    assert (reached[has]).all() and int((reached & ~has).sum()) == 1  # only the origin is reached without a push
    if failed is not None:
        f = failed.astype(bool)
        # pushes to failed peers are dropped (gossip.rs:538-541): only a failed origin is reached
        assert int((reached & f & has).sum()) == 0
        assert int(summ_last["stranded"]) == int((~reached & ~f).sum())
    return hops


def test_multi_bfs_many_fine_bins_matches_level():
    """More fine bins than the small-level kernel keeps in LDS (4.2M nodes in 512-node fine
    bins: 8,204 > 8,192): its level-start pool fills live in global memory and its pool
    places are global atomics. Four rounds with failures, three slots, through the
    predicted level loop from round 1: equal to the level BFS (summaries, hops, counters)."""
    n = 4_200_000
    st = eb.synth.power_law_stakes(n)
    m = gs.Engine(st, 3, seed=29, rotation_probability=0.01, bfs_mode=gs.GS_BFS_MULTI)
    lv = gs.Engine(st, 3, seed=29, rotation_probability=0.01, bfs_mode=gs.GS_BFS_LEVEL)
    for e in (m, lv):
        e.set_slots([0, 0, 5], [2, 2, 1], [0.15, 0.3, 0.15])
        e.init_active_sets()
        e.fail_nodes([0.0, 0.2, 0.1])
    for r in range(4):
        for e in (m, lv):
            e.round(r, record=True)
    np.testing.assert_array_equal(m.summaries(), lv.summaries())
    for k in range(3):
        np.testing.assert_array_equal(m.hops(k), lv.hops(k))
        for x, y in zip(m.counters(k), lv.counters(k)):
            np.testing.assert_array_equal(x, y)
    for e in (m, lv):
        e.close()


def test_c4_sweep_slots_1m():
    """BASELINE C4 at size: a 1M-node power-law network, origin rank 1, the fail-nodes sweep
    (f = 0.1..0.5, when-to-fail 0) and the prune-stake-threshold sweep (0.05..0.40) as 13
    slots of one engine, 22 rounds through the first prune wave. The binned BFS equals
    the level BFS bit for bit (summaries of every slot every round; hops, counters and
    accumulators at the end, inbound lists of two slots), and the size-independent
    properties hold on every slot."""
    n = 1_000_000
    st = eb.synth.power_law_stakes(n)
    origin = int(np.argmax(st))  # rank 1: the largest stake, lowest id on ties
    fr = [0.1, 0.2, 0.3, 0.4, 0.5] + [0.0] * 8
    thr = [0.15] * 5 + [0.05 * (j + 1) for j in range(8)]
    S = len(fr)
    engs = [gs.Engine(st, S, seed=C2_SEED, rotation_probability=0.013333, bfs_mode=m)
            for m in (gs.GS_BFS_LEVEL, gs.GS_BFS_BINNED, gs.GS_BFS_MULTI)]
    for e in engs:
        e.set_slots([origin] * S, 2, thr)
        e.init_active_sets()
        e.fail_nodes(fr)
    for r in range(22):
        for e in engs:
            e.round(r, record=True)
    a = engs[0]
    sa = a.summaries()
    for b in engs[1:]:
        np.testing.assert_array_equal(sa, b.summaries())
    for k in range(S):
        fa = a.failed(k)
        assert int(fa.sum()) == int(fr[k] * n)  # floor(f * N) nodes fail (gossip.rs:756-771)
        ha = _invariants(a, k, n, sa[-1, k], failed=fa) if k in (0, 4, 5, 12) else a.hops(k)
        ca, aa = a.counters(k), a.accumulators(k)
        for b in engs[1:]:
            np.testing.assert_array_equal(fa, b.failed(k))
            np.testing.assert_array_equal(ha, b.hops(k))
            for x, y in zip(ca, b.counters(k)):
                np.testing.assert_array_equal(x, y)
            for x, y in zip(aa, b.accumulators(k)):
                np.testing.assert_array_equal(x, y)
    for e in engs:  # gs_round keeps the multi BFS's inbound rows on-chip: materialize the next BFS
        e.run_gossip()
    for k in (0, 12):
        ia = a.inbound(k, cap=32 * n)
        for b in engs[1:]:
            for x, y in zip(ia, b.inbound(k, cap=32 * n)):
                np.testing.assert_array_equal(x, y)
    # the threshold slots share origin, trajectory and caches until they prune: at the
    # first prune round a higher threshold keeps more inbound stake, so prunes do not grow
    pr = sa["prunes"][:, 5:].astype(np.int64)
    first = int(np.nonzero(pr.sum(axis=1))[0][0])
    assert (np.diff(pr[first]) <= 0).all() and pr[first, 0] > pr[first, -1]
    assert (sa["visited"][:, 5:] > 0.9 * n).all()
    # more failures reach fewer nodes
    assert (np.diff(sa["visited"][-1, :5].astype(np.int64)) < 0).all()


def test_c3_widest_rows_100k():
    """C3's widest active sets: 100k nodes at active-set size 27 (ring rows padded to 28
    words), two slots, 4 rounds: binned == level bit for bit and the invariants hold."""
    n = 100_000
    st = eb.synth.power_law_stakes(n)
    engs = [gs.Engine(st, 2, seed=C2_SEED, active_set_size=27, rotation_probability=0.013333, bfs_mode=m)
            for m in (gs.GS_BFS_LEVEL, gs.GS_BFS_BINNED, gs.GS_BFS_MULTI)]
    for e in engs:
        e.set_slots([int(np.argmax(st)), n // 3], 2, 0.15)
        e.init_active_sets()
        for r in range(4):
            e.round(r, record=True)
    a = engs[0]
    peers, lens = a.active_sets()
    assert (lens == 27).all()
    srt = np.sort(peers, axis=2)
    assert (np.diff(srt.astype(np.int64), axis=2) != 0).all()
    sa = a.summaries()
    for b in engs[1:]:
        np.testing.assert_array_equal(peers, b.active_sets()[0])
        np.testing.assert_array_equal(sa, b.summaries())
    for k in range(2):
        ha = _invariants(a, k, n, sa[-1, k])
        for b in engs[1:]:
            np.testing.assert_array_equal(ha, b.hops(k))
    for e in engs:  # gs_round keeps the multi BFS's inbound rows on-chip: materialize the next BFS
        e.run_gossip()
    for k in range(2):
        ia = a.inbound(k, cap=32 * n)
        for b in engs[1:]:
            for x, y in zip(ia, b.inbound(k, cap=32 * n)):
                np.testing.assert_array_equal(x, y)


def test_multi_bfs_groups_and_entries():
    """The multi-source BFS with 70 slots (three slot groups of <= 32) whose origins have
    different buckets (so a node's slots split over several entries k = min(bucket[u],
    bucket[origin])), failures, per-slot thresholds, 30 rounds through a prune wave:
    equal to the level BFS in every summary, hop table, counter, cache and accumulator."""
    n, S = 3000, 70
    pks, st = eb.synth.network(n)
    engs = [gs.Engine(st, S, seed=9, rotation_probability=0.03, bfs_mode=m)
            for m in (gs.GS_BFS_LEVEL, gs.GS_BFS_MULTI)]
    origins = [(k * 131 + 7) % n for k in range(S - 6)] + [5, 5, 5, 77, 77, 77]  # shared origins too
    fr = [0.0, 0.1, 0.0, 0.3] * (S // 4) + [0.0] * (S % 4)
    for e in engs:
        e.set_slots(origins, [k % 4 for k in range(S)], [0.05 * (k % 7) for k in range(S)])
        e.init_active_sets()
        e.fail_nodes(fr)
    for r in range(30):
        for e in engs:
            e.round(r, record=r >= 4)
    a = engs[0]
    assert int(a.summaries()["prunes"].sum()) > 0
    for b in engs[1:]:
        np.testing.assert_array_equal(a.summaries(), b.summaries())
        for k in (0, 17, 31, 32, 50, 63, 64, 66, 69):
            np.testing.assert_array_equal(a.hops(k), b.hops(k))
            np.testing.assert_array_equal(a.pruned_all(k), b.pruned_all(k))
            for x, y in zip(a.counters(k), b.counters(k)):
                np.testing.assert_array_equal(x, y)
            for x, y in zip(a.caches(k), b.caches(k)):
                np.testing.assert_array_equal(x, y)
            for x, y in zip(a.accumulators(k), b.accumulators(k)):
                np.testing.assert_array_equal(x, y)
    for e in engs:
        e.run_gossip()
    for b in engs[1:]:
        for k in (0, 40, 69):
            for x, y in zip(a.inbound(k), b.inbound(k)):
                np.testing.assert_array_equal(x, y)
