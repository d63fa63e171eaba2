"""ctypes binding to oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference's push path (see
oracle/oracle_core.h). Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, always as the checker.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58decode(s: str) -> bytes:
    n = 0
    for ch in s:
        n = n * 58 + B58.index(ch)
    body = n.to_bytes((n.bit_length() + 7) // 8, "big") if n else b""
    lead = len(s) - len(s.lstrip("1"))
    out = b"\x00" * lead + body
    assert len(out) == 32, (s, len(out))
    return out


def b58encode(b: bytes) -> str:
    n = int.from_bytes(b, "big")
    s = ""
    while n:
        n, r = divmod(n, 58)
        s = B58[r] + s
    lead = len(b) - len(b.lstrip(b"\x00"))
    return "1" * lead + s


def counter_pubkey(i: int) -> bytes:
    """solana_sdk Pubkey::new_unique(): big-endian counter in bytes 0..8."""
    return i.to_bytes(8, "big") + b"\x00" * 24


def _load():
    if not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    lib = C.CDLL(LIB_PATH)
    P, U64, U32, SZ, D, I = C.c_void_p, C.c_uint64, C.c_uint32, C.c_size_t, C.c_double, C.c_int
    BP = C.c_char_p
    sig = {
        "or_last_error": (BP, []),
        "or_chacha_new": (P, [BP]),
        "or_philox_stream_new": (P, [U64, U32, U32, U32]),
        "or_rng_free": (None, [P]),
        "or_rng_next_u64": (U64, [P]),
        "or_gen_range": (U64, [P, U64, U64]),
        "or_gen_f64": (D, [P]),
        "or_philox": (None, [P, P, P]),
        "or_base58": (I, [BP, BP]),
        "or_pubkey_from_counter": (None, [U64, BP]),
        "or_stake_bucket": (I, [U64, I]),
        "or_stakes_new": (P, [BP, P, SZ]),
        "or_stakes_free": (None, [P]),
        "or_entry_new": (P, []),
        "or_entry_free": (None, [P]),
        "or_entry_rotate": (None, [P, P, SZ, BP, P, SZ]),
        "or_entry_keys": (SZ, [P, BP, SZ]),
        "or_entry_get_nodes": (SZ, [P, BP, I, BP, SZ]),
        "or_entry_prune": (None, [P, BP, BP]),
        "or_entry_filter_contains": (I, [P, BP, BP]),
        "or_pas_new": (P, []),
        "or_pas_free": (None, [P]),
        "or_pas_rotate": (None, [P, P, SZ, BP, SZ, P]),
        "or_pas_get_nodes": (SZ, [P, BP, BP, P, BP, SZ]),
        "or_pas_prune": (None, [P, BP, BP, BP, SZ, P]),
        "or_pas_entry_keys": (SZ, [P, I, BP, SZ]),
        "or_pas_filter_contains": (I, [P, I, BP, BP]),
        "or_rc_new": (P, []),
        "or_rc_free": (None, [P]),
        "or_rc_clone": (P, [P]),
        "or_rc_record": (None, [P, BP, BP, SZ]),
        "or_rc_entry": (C.c_long, [P, BP, P, BP, P, SZ]),
        "or_rc_prune": (SZ, [P, BP, BP, D, SZ, P, BP, SZ]),
        "or_sim_new": (P, [I, U64, BP, P, SZ, SZ]),
        "or_sim_free": (None, [P]),
        "or_sim_init_compat": (None, [P, P, SZ]),
        "or_sim_init_philox": (None, [P, SZ]),
        "or_sim_run_gossip": (None, [P, SZ]),
        "or_sim_consume": (None, [P, SZ]),
        "or_sim_send_prunes": (None, [P, SZ, D, SZ]),
        "or_sim_prune_connections": (None, [P]),
        "or_sim_chance_to_rotate": (None, [P, SZ, D, U32, P]),
        "or_sim_fail_nodes": (C.c_long, [P, D]),
        "or_sim_find_nth_largest": (SZ, [P, SZ]),
        "or_sim_rank": (SZ, [P, SZ]),
        "or_sim_round": (U64, [P, SZ, D, SZ, SZ, D, U32]),
        "or_sim_visited_len": (SZ, [P]),
        "or_sim_distances": (None, [P, P]),
        "or_sim_orders": (C.c_long, [P, SZ, P, P, SZ]),
        "or_sim_pushes": (C.c_long, [P, SZ, P, SZ]),
        "or_sim_mst": (C.c_long, [P, SZ, P, SZ]),
        "or_sim_prunes_len": (SZ, [P]),
        "or_sim_prunes": (SZ, [P, P, P, SZ]),
        "or_sim_counters": (None, [P, P, P, P]),
        "or_sim_rmr": (I, [P, P, P, P]),
        "or_sim_rmr_m": (U64, [P]),
        "or_sim_rmr_n": (U64, [P]),
        "or_sim_coverage": (D, [P, P]),
        "or_sim_stranded": (SZ, [P, P, SZ]),
        "or_sim_entry": (C.c_long, [P, SZ, I, P, SZ]),
        "or_sim_entry_pruned": (I, [P, SZ, I, SZ, SZ]),
        "or_sim_entries": (None, [P, P, P, SZ]),
        "or_sim_pruned_all": (None, [P, SZ, P]),
        "or_sim_caches": (None, [P, SZ, P, P, P, P, SZ]),
        "or_sim_cache": (C.c_long, [P, SZ, SZ, P, P, P, SZ]),
        "or_sim_failed": (None, [P, P]),
        "or_sim_total_prunes": (SZ, [P]),
        "or_sim_set_entries": (I, [P, P, P, SZ]),
        "or_sim_orders_all": (C.c_long, [P, P, P, P, SZ]),
        "or_replay_node_entries": (C.c_long, [U64, P, SZ, SZ, SZ, D, U32, P, P, SZ]),
        "or_stats_new": (P, []),
        "or_stats_free": (None, [P]),
        "or_stats_insert_hops": (None, [P, P, SZ]),
        "or_stats_insert_coverage": (None, [P, D]),
        "or_stats_insert_rmr": (None, [P, D]),
        "or_stats_insert_stranded": (None, [P, BP, SZ, P]),
        "or_stats_branching": (None, [P, P, SZ]),
        "or_stats_calculate": (None, [P]),
        "or_run_simulation": (P, [BP, P, SZ, SZ, SZ, SZ, SZ, D, D, SZ, U64, U64, U64, D, SZ, I, SZ, U64]),
        "or_res_f64": (SZ, [P, BP, P, SZ]),
        "or_res_u64": (SZ, [P, BP, P, SZ]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def pk_blob(pks):
    return b"".join(pks)


def split_pks(buf, n):
    return [bytes(buf[32 * i:32 * i + 32]) for i in range(n)]


class Rng:
    def __init__(self, handle):
        self.h = handle

    @classmethod
    def chacha(cls, seed: bytes):
        return cls(lib.or_chacha_new(seed))

    @classmethod
    def philox(cls, seed, purpose, a, b):
        return cls(lib.or_philox_stream_new(seed, purpose, a, b))

    def next_u64(self):
        return lib.or_rng_next_u64(self.h)

    def gen_range(self, lo, hi):
        return lib.or_gen_range(self.h, lo, hi)

    def gen_f64(self):
        return lib.or_gen_f64(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_rng_free(self.h)


def philox(ctr, key):
    c = np.array(ctr, dtype=np.uint32)
    k = np.array(key, dtype=np.uint32)
    o = np.zeros(4, dtype=np.uint32)
    lib.or_philox(_ptr(c), _ptr(k), _ptr(o))
    return [int(x) for x in o]


def base58(pk: bytes) -> str:
    buf = C.create_string_buffer(64)
    n = lib.or_base58(pk, buf)
    return buf.value[:n].decode()


class Stakes:
    def __init__(self, mapping):
        keys = list(mapping.keys())
        vals = np.array([mapping[k] for k in keys], dtype=np.uint64)
        self.h = lib.or_stakes_new(pk_blob(keys), _ptr(vals), len(keys))

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_stakes_free(self.h)


class Entry:
    def __init__(self):
        self.h = lib.or_entry_new()

    def rotate(self, rng, size, nodes, weights):
        w = np.array(weights, dtype=np.uint64)
        lib.or_entry_rotate(self.h, rng.h, size, pk_blob(nodes), _ptr(w), len(nodes))

    def keys(self):
        buf = C.create_string_buffer(32 * 64)
        n = lib.or_entry_keys(self.h, buf, 64)
        return split_pks(buf.raw, n)

    def get_nodes(self, origin, force):
        buf = C.create_string_buffer(32 * 64)
        n = lib.or_entry_get_nodes(self.h, origin, 1 if force else 0, buf, 64)
        return split_pks(buf.raw, n)

    def prune(self, node, origin):
        lib.or_entry_prune(self.h, node, origin)

    def filter_contains(self, node, key):
        return lib.or_entry_filter_contains(self.h, node, key)

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_entry_free(self.h)


class PushActiveSet:
    def __init__(self):
        self.h = lib.or_pas_new()

    def rotate(self, rng, size, nodes, stakes):
        lib.or_pas_rotate(self.h, rng.h, size, pk_blob(nodes), len(nodes), stakes.h)

    def get_nodes(self, pubkey, origin, stakes):
        buf = C.create_string_buffer(32 * 64)
        n = lib.or_pas_get_nodes(self.h, pubkey, origin, stakes.h, buf, 64)
        return split_pks(buf.raw, n)

    def prune(self, pubkey, node, origins, stakes):
        lib.or_pas_prune(self.h, pubkey, node, pk_blob(origins), len(origins), stakes.h)

    def entry_keys(self, k):
        buf = C.create_string_buffer(32 * 64)
        n = lib.or_pas_entry_keys(self.h, k, buf, 64)
        return split_pks(buf.raw, n)

    def filter_contains(self, k, node, key):
        return lib.or_pas_filter_contains(self.h, k, node, key)

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_pas_free(self.h)


class ReceivedCache:
    def __init__(self, h=None):
        self.h = h or lib.or_rc_new()

    def record(self, origin, node, num_dups):
        lib.or_rc_record(self.h, origin, node, num_dups)

    def entry(self, origin):
        up = np.zeros(1, dtype=np.uint64)
        buf = C.create_string_buffer(32 * 128)
        sc = np.zeros(128, dtype=np.uint64)
        n = lib.or_rc_entry(self.h, origin, _ptr(up), buf, _ptr(sc), 128)
        if n < 0:
            return None
        return int(up[0]), dict(zip(split_pks(buf.raw, n), [int(x) for x in sc[:n]]))

    def clone(self):
        return ReceivedCache(lib.or_rc_clone(self.h))

    def prune(self, pubkey, origin, thr, min_ingress, stakes):
        buf = C.create_string_buffer(32 * 128)
        n = lib.or_rc_prune(self.h, pubkey, origin, thr, min_ingress, stakes.h, buf, 128)
        return split_pks(buf.raw, n)

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_rc_free(self.h)


COMPAT, PHILOX = 0, 1


class Sim:
    """One reference simulation (one origin): Cluster + nodes, restated."""

    def __init__(self, mode, seed, pks, stakes, fanout):
        self.n = len(pks)
        self.pks = list(pks)
        st = np.array(stakes, dtype=np.uint64)
        self.h = lib.or_sim_new(mode, seed, pk_blob(pks), _ptr(st), self.n, fanout)

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_sim_free(self.h)

    def init_compat(self, rng, asz):
        lib.or_sim_init_compat(self.h, rng.h, asz)

    def init_philox(self, asz):
        lib.or_sim_init_philox(self.h, asz)

    def run_gossip(self, origin):
        lib.or_sim_run_gossip(self.h, origin)

    def consume_messages(self, origin):
        lib.or_sim_consume(self.h, origin)

    def send_prunes(self, origin, thr, min_ingress):
        lib.or_sim_send_prunes(self.h, origin, thr, min_ingress)

    def prune_connections(self):
        lib.or_sim_prune_connections(self.h)

    def chance_to_rotate(self, asz, p, rnd, compat_rng=None):
        lib.or_sim_chance_to_rotate(self.h, asz, p, rnd, compat_rng.h if compat_rng else None)

    def fail_nodes(self, f):
        r = lib.or_sim_fail_nodes(self.h, f)
        if r < 0:
            raise RuntimeError(lib.or_last_error().decode())
        return r

    def find_nth_largest(self, n):
        return lib.or_sim_find_nth_largest(self.h, n)

    def round(self, origin, thr, min_ingress, asz, p, rnd):
        return lib.or_sim_round(self.h, origin, thr, min_ingress, asz, p, rnd)

    def rank(self, i):
        return lib.or_sim_rank(self.h, i)

    def visited_len(self):
        return lib.or_sim_visited_len(self.h)

    def distances(self):
        out = np.zeros(self.n, dtype=np.uint64)
        lib.or_sim_distances(self.h, _ptr(out))
        return out

    def orders(self, dest):
        src = np.zeros(self.n, dtype=np.uint32)
        hops = np.zeros(self.n, dtype=np.uint64)
        c = lib.or_sim_orders(self.h, dest, _ptr(src), _ptr(hops), self.n)
        if c < 0:
            return None
        return [(int(s), int(h)) for s, h in zip(src[:c], hops[:c])]

    def pushes(self, src):
        out = np.zeros(self.n, dtype=np.uint32)
        c = lib.or_sim_pushes(self.h, src, _ptr(out), self.n)
        return None if c < 0 else [int(x) for x in out[:c]]

    def mst(self, src):
        out = np.zeros(self.n, dtype=np.uint32)
        c = lib.or_sim_mst(self.h, src, _ptr(out), self.n)
        return None if c < 0 else [int(x) for x in out[:c]]

    def prunes_len(self):
        return lib.or_sim_prunes_len(self.h)

    def prunes(self):
        cap = 64 * self.n + 64
        a = np.zeros(cap, dtype=np.uint32)
        b = np.zeros(cap, dtype=np.uint32)
        c = lib.or_sim_prunes(self.h, _ptr(a), _ptr(b), cap)
        return [(int(x), int(y)) for x, y in zip(a[:c], b[:c])]

    def counters(self):
        e = np.zeros(self.n, dtype=np.uint64)
        i = np.zeros(self.n, dtype=np.uint64)
        p = np.zeros(self.n, dtype=np.uint64)
        lib.or_sim_counters(self.h, _ptr(e), _ptr(i), _ptr(p))
        return e, i, p

    def rmr(self):
        r = np.zeros(1, dtype=np.float64)
        m = np.zeros(1, dtype=np.uint64)
        n = np.zeros(1, dtype=np.uint64)
        st = lib.or_sim_rmr(self.h, _ptr(r), _ptr(m), _ptr(n))
        return None if st else (float(r[0]), int(m[0]), int(n[0]))

    def rmr_mn(self):
        return lib.or_sim_rmr_m(self.h), lib.or_sim_rmr_n(self.h)

    def coverage(self):
        left = np.zeros(1, dtype=np.uint64)
        c = lib.or_sim_coverage(self.h, _ptr(left))
        return c, int(left[0])

    def stranded(self):
        out = np.zeros(self.n, dtype=np.uint32)
        c = lib.or_sim_stranded(self.h, _ptr(out), self.n)
        return [int(x) for x in out[:c]]

    def entry(self, node, k):
        out = np.zeros(64, dtype=np.uint32)
        c = lib.or_sim_entry(self.h, node, k, _ptr(out), 64)
        return [int(x) for x in out[:c]]

    def entries(self, cap):
        peers = np.zeros(self.n * 25 * cap, dtype=np.uint32)
        lens = np.zeros(self.n * 25, dtype=np.uint8)
        lib.or_sim_entries(self.h, _ptr(peers), _ptr(lens), cap)
        return peers.reshape(self.n, 25, cap), lens.reshape(self.n, 25)

    def pruned_all(self, origin):
        out = np.zeros(self.n, dtype=np.uint32)
        lib.or_sim_pruned_all(self.h, origin, _ptr(out))
        return out

    def caches(self, origin, cap=96):
        up = np.zeros(self.n, dtype=np.uint32)
        ln = np.zeros(self.n, dtype=np.uint32)
        k = np.zeros(self.n * cap, dtype=np.uint32)
        s = np.zeros(self.n * cap, dtype=np.uint32)
        lib.or_sim_caches(self.h, origin, _ptr(up), _ptr(ln), _ptr(k), _ptr(s), cap)
        return up, ln, k.reshape(self.n, cap), s.reshape(self.n, cap)

    def entry_pruned(self, node, k, peer, origin):
        return lib.or_sim_entry_pruned(self.h, node, k, peer, origin)

    def cache(self, node, origin):
        up = np.zeros(1, dtype=np.uint64)
        keys = np.zeros(256, dtype=np.uint32)
        sc = np.zeros(256, dtype=np.uint64)
        c = lib.or_sim_cache(self.h, node, origin, _ptr(up), _ptr(keys), _ptr(sc), 256)
        if c < 0:
            return None
        return int(up[0]), {int(k): int(s) for k, s in zip(keys[:c], sc[:c])}

    def failed(self):
        out = np.zeros(self.n, dtype=np.uint8)
        lib.or_sim_failed(self.h, _ptr(out))
        return out

    def total_prunes(self):
        return lib.or_sim_total_prunes(self.h)

    def set_entries(self, peers, lens):
        """Every node's entries at once (peers [n, 25, cap] in FIFO order, lens [n, 25])."""
        p = np.ascontiguousarray(peers, dtype=np.uint32)
        ln = np.ascontiguousarray(lens, dtype=np.uint8)
        if lib.or_sim_set_entries(self.h, _ptr(p), _ptr(ln), p.shape[2]) != 0:
            raise ValueError(lib.or_last_error().decode())

    def orders_all(self, cap):
        """Every destination's orders as CSR (off [n+1], src, hop), lists in consume order."""
        off = np.zeros(self.n + 1, dtype=np.uint32)
        src = np.zeros(cap, dtype=np.uint32)
        hop = np.zeros(cap, dtype=np.uint8)
        c = lib.or_sim_orders_all(self.h, _ptr(off), _ptr(src), _ptr(hop), cap)
        if c < 0:
            raise ValueError("orders exceed cap")
        return off, src[:c], hop[:c]


def replay_node_entries(seed, stakes, node, asz, p, rounds):
    """One node's entries after init + `rounds` rotation rounds (PHILOX), replayed alone:
    (peers [25, asz] ids in FIFO order, lens [25], rotations made)."""
    st = np.ascontiguousarray(stakes, dtype=np.uint64)
    peers = np.zeros(25 * asz, dtype=np.uint32)
    lens = np.zeros(25, dtype=np.uint8)
    rot = lib.or_replay_node_entries(seed, _ptr(st), len(st), node, asz, p, rounds, _ptr(peers), _ptr(lens), asz)
    if rot < 0:
        raise ValueError(lib.or_last_error().decode())
    return peers.reshape(25, asz), lens, rot


class Stats:
    def __init__(self, h=None):
        self.h = h or lib.or_stats_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib.or_stats_free(self.h)

    def insert_hops(self, values):
        a = np.array(values, dtype=np.uint64)
        lib.or_stats_insert_hops(self.h, _ptr(a), len(a))

    def insert_coverage(self, v):
        lib.or_stats_insert_coverage(self.h, v)

    def insert_rmr(self, v):
        lib.or_stats_insert_rmr(self.h, v)

    def insert_stranded(self, pks, stakes):
        lib.or_stats_insert_stranded(self.h, pk_blob(pks), len(pks), stakes.h)

    def branching(self, set_sizes):
        a = np.array(set_sizes, dtype=np.uint64)
        lib.or_stats_branching(self.h, _ptr(a), len(a))

    def calculate(self):
        lib.or_stats_calculate(self.h)

    def f64(self, name, cap=1 << 16):
        out = np.zeros(cap, dtype=np.float64)
        n = lib.or_res_f64(self.h, name.encode(), _ptr(out), cap)
        assert n != C.c_size_t(-1).value, name
        return out[:n].copy()

    def u64(self, name, cap=1 << 20):
        out = np.zeros(cap, dtype=np.uint64)
        n = lib.or_res_u64(self.h, name.encode(), _ptr(out), cap)
        assert n != C.c_size_t(-1).value, name
        return out[:n].copy()


def run_simulation(pks, stakes, *, fanout=6, asz=12, iterations=1, origin_rank=1, p=0.013333, thr=0.15,
                   min_ingress=2, nb_stranded=10, nb_message=5, nb_hops=15, fraction_to_fail=0.1,
                   when_to_fail=0, test_type=0, warm_up=200, seed=0):
    st = np.array(stakes, dtype=np.uint64)
    h = lib.or_run_simulation(pk_blob(pks), _ptr(st), len(pks), fanout, asz, iterations, origin_rank, p, thr,
                              min_ingress, nb_stranded, nb_message, nb_hops, fraction_to_fail, when_to_fail,
                              test_type, warm_up, seed)
    if not h:
        raise RuntimeError(lib.or_last_error().decode())
    return Stats(h)
