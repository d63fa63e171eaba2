"""Pin the CPU oracle against the reference's own unit-test known answers.

Every expected value below is an assertion from the reference's inline tests
(file:line cited per test). Pubkeys come from Pubkey::new_unique() (a BE
counter starting at 1, each test alone in a fresh process), RNG streams from
ChaChaRng::from_seed([189;32]) / ([147;32]) exactly as the reference tests.
test_rmr (gossip_stats.rs:2074-2157) is stale (SURVEY.md header) and not used.
"""

import pytest

import oracle_bind as ob
from oracle_bind import counter_pubkey as cpk, b58decode

LAMPORTS = 1_000_000_000
MAX_STAKE = (1 << 20) * LAMPORTS


def test_chacha_keystream_zero_key():
    # djb ChaCha20, zero key / zero nonce, block 0 (the classic keystream vector).
    r = ob.Rng.chacha(bytes(32))
    words = [r.next_u64() for _ in range(4)]
    raw = b"".join(w.to_bytes(8, "little") for w in words)
    assert raw.hex() == "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"


def test_philox_random123_kat():
    assert ob.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert ob.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert ob.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_base58_roundtrip_and_counter_keys():
    # gossip_stats.rs tests decode to new_unique counters.
    assert b58decode("11111113pNDtm61yGF8j2ycAwLEPsuWQXobye5qDR") == cpk(7)
    assert ob.base58(cpk(1)) == "1111111QLbz7JHiBTspS962RLKV8GndWFwiEaqKM"
    for i in (1, 2, 3, 17, 40, 1 << 40):
        assert ob.b58decode(ob.base58(cpk(i))) == cpk(i)
        assert ob.b58encode(cpk(i)) == ob.base58(cpk(i))


def test_get_stake_bucket():
    # push_active_set.rs:205-226
    assert ob.lib.or_stake_bucket(0, 0) == 0
    buckets = [0, 1, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 4, 5, 5]
    for k, b in enumerate(buckets):
        assert ob.lib.or_stake_bucket(k * LAMPORTS, 1) == b
    for stake, b in [(4_194_303, 22), (4_194_304, 23), (8_388_607, 23), (8_388_608, 24)]:
        assert ob.lib.or_stake_bucket(stake * LAMPORTS, 1) == b
    assert ob.lib.or_stake_bucket(2**64 - 1, 1) == 24


def test_push_active_set_entry():
    # push_active_set.rs:341-400
    rng = ob.Rng.chacha(bytes([147] * 32))
    nodes = [cpk(i) for i in range(1, 21)]
    weights = [rng.gen_range(1, 1000) for _ in range(20)]
    e = ob.Entry()
    e.rotate(rng, 5, nodes, weights)
    keys = [nodes[i] for i in (16, 11, 17, 14, 5)]
    assert e.keys() == keys
    for origin in nodes:
        if origin not in keys:
            assert e.get_nodes(origin, False) == keys
        else:
            assert e.get_nodes(origin, True) == keys
            assert e.get_nodes(origin, False) == [k for k in keys if k != origin]
    for node in keys:
        assert e.filter_contains(node, node) == 1
    origin = nodes[3]
    e.prune(nodes[11], origin)
    e.prune(nodes[14], origin)
    e.prune(nodes[19], origin)
    assert e.get_nodes(origin, True) == keys
    assert e.get_nodes(origin, False) == [k for k in keys if k not in (nodes[11], nodes[14])]
    e.rotate(rng, 5, nodes, weights)
    assert e.keys() == [nodes[i] for i in (11, 17, 14, 5, 7)]
    e.rotate(rng, 6, nodes, weights)
    assert e.keys() == [nodes[i] for i in (17, 14, 5, 7, 1, 13)]
    e.rotate(rng, 4, nodes, weights)
    assert e.keys() == [nodes[i] for i in (5, 7, 1, 13)]


def test_push_active_set():
    # push_active_set.rs:228-339
    rng = ob.Rng.chacha(bytes([189] * 32))
    pubkey = cpk(1)
    nodes = [cpk(i) for i in range(2, 22)]
    stakes = {n: rng.gen_range(1, MAX_STAKE) for n in nodes}
    stakes[pubkey] = rng.gen_range(1, MAX_STAKE)
    st = ob.Stakes(stakes)
    pas = ob.PushActiveSet()
    pas.rotate(rng, 5, nodes, st)
    for k in range(25):
        ks = pas.entry_keys(k)
        assert len(ks) == 5
        for n in ks:
            assert pas.filter_contains(k, n, n) == 1
    other, origin = nodes[5], nodes[17]
    sel = lambda idx: [nodes[i] for i in idx]  # noqa: E731
    assert pas.get_nodes(pubkey, origin, st) == sel([13, 5, 18, 16, 0])
    assert pas.get_nodes(pubkey, other, st) == sel([13, 18, 16, 0])
    pas.prune(pubkey, nodes[5], [origin], st)
    pas.prune(pubkey, nodes[3], [origin], st)
    pas.prune(pubkey, nodes[16], [origin], st)
    assert pas.get_nodes(pubkey, origin, st) == sel([13, 18, 0])
    assert pas.get_nodes(pubkey, other, st) == sel([13, 18, 16, 0])
    pas.rotate(rng, 7, nodes, st)
    for k in range(25):
        assert len(pas.entry_keys(k)) == 7
    assert pas.get_nodes(pubkey, origin, st) == sel([18, 0, 7, 15, 11])
    assert pas.get_nodes(pubkey, other, st) == sel([18, 16, 0, 7, 15, 11])
    for n in (18, 0, 15):
        pas.prune(pubkey, nodes[n], [origin, other], st)
    assert pas.get_nodes(pubkey, origin, st) == sel([7, 11])
    assert pas.get_nodes(pubkey, other, st) == sel([16, 7, 11])


def test_received_cache():
    # received_cache.rs:141-200
    cache = ob.ReceivedCache()
    pubkey, origin = cpk(1), cpk(2)
    records = [[3, 1, 7, 5], [7, 6, 5, 2], [2, 0, 0, 2], [3, 5, 0, 6], [6, 2, 6, 2]]
    nodes = [cpk(i) for i in range(3, 8)]
    for node, rec in zip(nodes, records):
        for num_dups, k in enumerate(rec):
            for _ in range(k):
                cache.record(origin, node, num_dups)
    up, scores = cache.entry(origin)
    assert up == 21
    assert scores == {nodes[0]: 4, nodes[1]: 13, nodes[2]: 2, nodes[3]: 8, nodes[4]: 8}
    stakes = ob.Stakes({nodes[0]: 6, nodes[1]: 1, nodes[2]: 5, nodes[3]: 3, nodes[4]: 7, pubkey: 9, origin: 9})
    assert set(cache.clone().prune(pubkey, origin, 0.5, 2, stakes)) == {nodes[0], nodes[2], nodes[3]}
    assert set(cache.prune(pubkey, origin, 1.0, 0, stakes)) == {nodes[0], nodes[2]}
    # the entry was taken (std::mem::take) by the prune
    up, scores = cache.entry(origin)
    assert up == 0 and scores == {}


def six_node_cluster():
    """The 5+1 node cluster of test_mst / test_pruning / test_rmr (gossip.rs:1041-1067)."""
    rng = ob.Rng.chacha(bytes([189] * 32))
    nodes = [cpk(i) for i in range(1, 6)]
    pubkey = cpk(6)
    stakes = [rng.gen_range(1, MAX_STAKE) for _ in range(5)]
    stakes.append(rng.gen_range(1, MAX_STAKE))
    pks = nodes + [pubkey]  # sorted by Pubkey == nodes.sort_by_key(pubkey)
    sim = ob.Sim(ob.COMPAT, 0, pks, stakes, 2)
    sim.init_compat(rng, 12)
    return sim, pks, stakes, rng


def test_mst():
    # gossip.rs:1040-1163
    sim, pks, stakes, _ = six_node_cluster()
    buckets = sorted(ob.lib.or_stake_bucket(s, 1) for s in stakes)
    assert buckets == [15, 16, 19, 19, 20, 20]
    origin = 5
    sim.run_gossip(origin)
    assert sim.visited_len() == 6
    assert list(sim.distances()) == [2, 3, 1, 2, 1, 0]
    inbound = {d: dict(sim.orders(d)) for d in range(5)}
    assert [len(inbound[d]) for d in range(5)] == [3, 1, 3, 2, 3]
    assert inbound[0][1] == 4 and inbound[0][4] == 2
    assert inbound[1][0] == 3
    assert inbound[2][0] == 3 and inbound[2][3] == 3 and inbound[2][5] == 1
    assert inbound[4][2] == 2 and inbound[4][3] == 3 and inbound[4][5] == 1
    assert sim.orders(5) is None
    assert sim.coverage() == (1.0, 0)
    assert sim.mst(5) == [2, 4]
    assert sim.mst(4) == [0, 3]
    assert sim.mst(0) == [1]
    assert sim.mst(1) is None and sim.mst(3) is None


def test_pruning():
    # gossip_main.rs:1071-1163
    sim, pks, stakes, rng = six_node_cluster()
    origin = 5
    for i in range(21):
        sim.run_gossip(origin)
        assert sim.visited_len() == 6
        sim.consume_messages(origin)
        sim.send_prunes(origin, 0.15, 2)
        assert sim.prunes_len() == 6
        prunes = sim.prunes()
        if i <= 18:
            assert prunes == []
        for pruner, prunee in prunes:
            expect = {2: 0, 0: 1, 4: 3}
            if pruner in expect:
                assert prunee == expect[pruner]
        if i == 19:
            assert sorted(prunes) == [(0, 1), (2, 0), (4, 3)]
        sim.prune_connections()
        sim.chance_to_rotate(12, 0.2, i, rng)  # rotation is a no-op on 6 nodes (entries hold all 5 peers)


def test_nth_largest():
    # gossip_main.rs:1056-1069
    stakes = [10, 123, 67, 18, 29, 567, 12, 5, 875, 234, 12, 5, 76, 0, 12354, 985]
    ranks = [5, 10, 12, 1, 6, 2, 9, 16]
    res = [234, 18, 12, 12354, 123, 985, 29, 0]
    pks = [cpk(i) for i in range(1, 17)]
    sim = ob.Sim(ob.PHILOX, 0, pks, stakes, 6)
    for r, want in zip(ranks, res):
        assert stakes[sim.find_nth_largest(r)] == want


def ten_node_stakes():
    rng = ob.Rng.chacha(bytes([189] * 32))
    keys = [cpk(i) for i in range(1, 11)]
    vals = [rng.gen_range(1, MAX_STAKE) for _ in range(10)]
    return dict(zip(keys, vals))


def test_stranded():
    # gossip_stats.rs:2007-2072
    stakes = ob.Stakes(ten_node_stakes())
    s = ob.Stats()
    k = lambda x: b58decode(x)  # noqa: E731
    stranded = [k("11111113pNDtm61yGF8j2ycAwLEPsuWQXobye5qDR"), k("11111114DhpssPJgSi1YU7hCMfYt1BJ334YgsffXm"),
                k("11111114d3RrygbPdAtMuFnDmzsN8T5fYKVQ7FVr7"), k("111111152P2r5yt6odmBLPsFCLBrFisJ3aS7LqLAT")]
    s.insert_stranded(stranded, stakes)
    s.calculate()
    f, u = s.f64("stranded"), s.u64("stranded")
    assert u[0] == 4
    assert list(f[:4]) == [0.4, 4.0, 1.0, 1.0]
    assert f[4] == 645017127080371.25 and f[5] == 724161057685112.0
    assert u[2] == 1017190976849038 and u[3] == 114555416102223
    assert f[6] == 645017127080371.25 and f[7] == 724161057685112.0
    for _ in range(4):
        stranded += [k("11111113R2cuenjG5nFubqX9Wzuukdin2YfGQVzu5"), k("11111112D1oxKts8YPdTJRG5FzxTNpMtWmq8hkVx3"),
                     k("111111131h1vYVSYuKP6AhS86fbRdMw9XHiZAvAaj"), k("1111111QLbz7JHiBTspS962RLKV8GndWFwiEaqKM")]
    for _ in range(7):
        stranded += [k("11111113R2cuenjG5nFubqX9Wzuukdin2YfGQVzu5"), k("111111152P2r5yt6odmBLPsFCLBrFisJ3aS7LqLAT"),
                     k("1111111QLbz7JHiBTspS962RLKV8GndWFwiEaqKM"), k("11111114DhpssPJgSi1YU7hCMfYt1BJ334YgsffXm")]
    s.insert_stranded(stranded, stakes)
    s.calculate()
    f, u = s.f64("stranded"), s.u64("stranded")
    assert u[0] == 52
    assert list(f[:4]) == [5.2, 26.0, 6.50, 6.50]
    assert f[4] == 617812196595019.00 and f[5] == 623567922929968.5
    assert u[2] == 1017190976849038 and u[3] == 114555416102223
    assert f[6] == 615709255382738.9 and f[7] == 585038762479069.0


def test_hops():
    # gossip_stats.rs:2159-2259 (only the distances' values matter)
    M = 2**64 - 1
    s = ob.Stats()
    s.insert_hops([M, M, M, M, 0, 1, 1, 2, 2, 3])
    s.insert_hops([M, M, M, M, M, M, 0, 1, 1, 2])
    s.insert_hops([M, M, M, M, M, M, M, 0, 1, 6])
    mean, median = s.f64("hop_mean"), s.f64("hop_median")
    mx, mn = s.u64("hop_max"), s.u64("hop_min")
    assert (mean[0], median[0], mx[0], mn[0]) == (1.8, 2.0, 3, 1)
    assert (mean[1], median[1], mx[1], mn[1]) == (1.3333333333333333, 1.0, 2, 1)
    assert (mean[2], median[2], mx[2], mn[2]) == (3.5, 3.5, 6, 1)
    s.calculate()
    assert list(s.f64("aggregate_hops")) == [2.0, 1.5] and list(s.u64("aggregate_hops")) == [6, 1]
    assert list(s.f64("ldh")) == [3.6666666666666665, 3.0] and list(s.u64("ldh")) == [6, 2]


def test_coverage():
    # gossip_stats.rs:2261-2359
    s = ob.Stats()
    for visited, want in [(6, (0.6, 0.6, 0.6, 0.6)), (4, (0.5, 0.5, 0.6, 0.4)),
                          (2, (0.4000000000000001, 0.4, 0.6, 0.2))]:
        s.insert_coverage(visited / 10)
        s.calculate()
        assert tuple(s.f64("coverage_stats")) == want


def test_branching_factors():
    # gossip_stats.rs:2361-2428
    s = ob.Stats()
    s.branching([3, 2, 1, 1, 1, 0, 1, 1])
    assert s.f64("branching")[0] == 1.25


@pytest.mark.parametrize("seed", [1, 7])
def test_weighted_shuffle_prefix_semantics(seed):
    """WeightedShuffle: smallest index whose remaining-prefix exceeds the draw."""
    rng = ob.Rng.chacha(bytes([seed] * 32))
    nodes = [cpk(i) for i in range(1, 41)]
    weights = [((i * 7) % 25 + 1) ** 2 for i in range(40)]
    e = ob.Entry()
    e.rotate(rng, 39, nodes, weights)  # len 39 < 40 candidates: keeps draws 2..40
    got = e.keys()
    # replay with a Python restatement of the same draws
    rng2 = ob.Rng.chacha(bytes([seed] * 32))
    w = list(weights)
    order = []
    while sum(w):
        v = rng2.gen_range(0, sum(w))
        acc = 0
        for i, x in enumerate(w):
            acc += x
            if acc > v:
                order.append(i)
                w[i] = 0
                break
    assert got == [nodes[i] for i in order[1:40]]
