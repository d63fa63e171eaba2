"""CPU checks of the oracle helpers the large-N GPU parity tests rely on
(tests/test_oracle_scale.py): the stand-in pubkeys keep base58 order = id order, the
one-node active-set replay equals the oracle's own initialize_gossip + chance_to_rotate,
and the bulk entry upload / orders export are consistent with the per-node calls."""
import numpy as np

import oracle_bind as ob


def stand_in_pubkeys(n):
    """0xA5 || 0^23 || id big-endian: every key encodes to 44 base58 characters, so
    base58 (= node id) order is id order."""
    return [b"\xa5" + bytes(23) + i.to_bytes(8, "big") for i in range(n)]


def test_stand_in_pubkeys_order_is_id_order():
    pks = stand_in_pubkeys(1000) + [b"\xa5" + bytes(23) + (10**7 - 1).to_bytes(8, "big")]
    strs = [ob.base58(p) for p in pks]
    assert all(len(s) == 44 for s in strs)
    assert strs == sorted(strs)


def power_law(n):
    i = np.arange(n, dtype=np.uint64)
    return np.maximum(np.uint64(15_000_000_000_000_000) // (i + np.uint64(1)) + (i * np.uint64(7919)) %
                      np.uint64(1_000_000_000), np.uint64(1_000_000_000))


def test_replay_node_entries_equals_sim():
    n, asz, seed, p = 300, 12, 0x5EED0003, 0.1
    st = power_law(n)
    sim = ob.Sim(ob.PHILOX, seed, stand_in_pubkeys(n), st, 6)
    sim.init_philox(asz)
    nodes = [0, 1, 2, 57, 150, 299]
    peers, lens = sim.entries(asz)
    for v in nodes:
        rp, rl, rot = ob.replay_node_entries(seed, st, v, asz, p, 0)
        assert rot == 0
        np.testing.assert_array_equal(rl, lens[v])
        np.testing.assert_array_equal(rp, peers[v])
    for r in range(20):
        sim.chance_to_rotate(asz, p, r)
    peers, lens = sim.entries(asz)
    rots = 0
    for v in nodes:
        rp, rl, rot = ob.replay_node_entries(seed, st, v, asz, p, 20)
        rots += rot
        np.testing.assert_array_equal(rl, lens[v])
        np.testing.assert_array_equal(rp, peers[v])
    assert rots > 0


def test_set_entries_and_orders_all():
    n, asz, seed = 200, 8, 11
    st = power_law(n)
    a = ob.Sim(ob.PHILOX, seed, stand_in_pubkeys(n), st, 6)
    a.init_philox(asz)
    peers, lens = a.entries(asz)
    b = ob.Sim(ob.PHILOX, seed, stand_in_pubkeys(n), st, 6)
    b.set_entries(np.where(peers == 0xFFFFFFFF, 0, peers), lens)
    p2, l2 = b.entries(asz)
    np.testing.assert_array_equal(l2, lens)
    np.testing.assert_array_equal(p2, peers)
    origin = a.find_nth_largest(1)
    pruned = 0
    for r in range(22):  # both through a prune wave: the uploaded entries behave as the initialised ones
        for s in (a, b):
            s.run_gossip(origin)
            s.consume_messages(origin)
            s.send_prunes(origin, 0.15, 2)
            s.prune_connections()
        assert a.prunes() == b.prunes()
        pruned += len(a.prunes())
        np.testing.assert_array_equal(a.pruned_all(origin), b.pruned_all(origin))
    off, src, hop = b.orders_all(64 * n)
    for v in range(n):
        want = b.orders(v) or []
        assert list(zip(src[off[v]:off[v + 1]].tolist(), hop[off[v]:off[v + 1]].tolist())) == want
    assert pruned > 0
