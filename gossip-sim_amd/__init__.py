"""gossip-sim_amd -- MI355X-native push-propagation engine for gossip-sim.

Python side of the C ABI in include/gossip_hip.h (ctypes, no torch types). The
engine itself is libgossip_hip.so (HIP kernels for gfx950, built in-tree by
`make -C gossip-sim_amd`). There is no CPU fallback: constructing an Engine
without the library or without a visible GPU raises.

The Engine methods mirror the reference's Cluster API (src/gossip.rs):
run_gossip / consume_messages / send_prunes / prune_connections /
chance_to_rotate / fail_nodes, applied to every slot (= independent sim) at once.
"""
import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libgossip_hip.so")
if os.environ.get("GS_LIB_VARIANT"):  # A/B builds of the same sources (scripts/), never a fallback
    LIB_PATH = os.path.join(PKG_DIR, "variants", os.environ["GS_LIB_VARIANT"], "libgossip_hip.so")

GS_BFS_AUTO, GS_BFS_WORKGROUP, GS_BFS_LEVEL, GS_BFS_BINNED, GS_BFS_MULTI, GS_BFS_HYBRID = 0, 1, 2, 3, 4, 5
GS_FLAG_PROFILE = 1
GS_FLAG_SPLIT_ROUND = 2
GS_FLAG_NARROW_WAVE_PATH = 4
GS_FLAG_BINNED_ALL_LEVELS = 8
GS_FLAG_WIDE_RECORDS = 16
GS_FLAG_NO_SMALL_LEVELS = 32
GS_FLAG_MISPREDICT_LEVELS = 64
GS_FLAG_FRONTIER_EXCHANGE = 128
HOP_UNREACHED = 0xFF
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


class GsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"gossip_hip error {code}: {msg}")
        self.code = code


class Params(C.Structure):
    _fields_ = [("push_fanout", C.c_uint32), ("active_set_size", C.c_uint32), ("rotation_probability", C.c_double),
                ("seed", C.c_uint64), ("device", C.c_int32), ("bfs_mode", C.c_uint32),
                ("inbound_capacity", C.c_uint32), ("flags", C.c_uint32)]


class Slot(C.Structure):
    _fields_ = [("origin", C.c_uint32), ("min_ingress_nodes", C.c_uint32), ("prune_stake_threshold", C.c_double)]


class RoundSummary(C.Structure):
    _fields_ = [("visited", C.c_uint32), ("pushes", C.c_uint32), ("prunes", C.c_uint32), ("stranded", C.c_uint32),
                ("hop_sum", C.c_uint64), ("hop_count", C.c_uint32), ("hop_min", C.c_uint32),
                ("hop_max", C.c_uint32), ("hop_med_lo", C.c_uint32), ("hop_med_hi", C.c_uint32),
                ("pad0", C.c_uint32), ("stranded_stake_sum", C.c_uint64), ("stranded_stake_min", C.c_uint64),
                ("stranded_stake_max", C.c_uint64), ("stranded_med_lo", C.c_uint64),
                ("stranded_med_hi", C.c_uint64)]


SUMMARY_DTYPE = np.dtype([(n, np.uint32 if t is C.c_uint32 else np.uint64) for n, t in RoundSummary._fields_])
assert SUMMARY_DTYPE.itemsize == C.sizeof(RoundSummary)


class SimConfig(C.Structure):
    _fields_ = [("push_fanout", C.c_uint32), ("active_set_size", C.c_uint32), ("iterations", C.c_uint32),
                ("warm_up_rounds", C.c_uint32), ("min_ingress_nodes", C.c_uint32), ("when_to_fail", C.c_uint32),
                ("rotation_probability", C.c_double), ("prune_stake_threshold", C.c_double),
                ("fraction_to_fail", C.c_double), ("num_buckets_stranded", C.c_uint64),
                ("num_buckets_message", C.c_uint64), ("num_buckets_hops", C.c_uint64), ("test_type", C.c_int32),
                ("seed", C.c_uint64), ("device", C.c_int32), ("bfs_mode", C.c_uint32)]


EXPORTS = {
    # name: (restype, argtypes)
    "gs_last_error": (C.c_char_p, []),
    "gs_kernel_hash": (C.c_char_p, []),
    "gs_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "gs_read_mst": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "gs_create_part": (C.c_int, [C.POINTER(Params), C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                 C.POINTER(C.c_void_p)]),
    "gs_part_sizes": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "gs_part_round": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]),
    "gs_part_prunes_out": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "gs_part_prunes_in": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]),
    "gs_part_exchange_sizes": (C.c_int, [C.c_void_p, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "gs_part_prunes_dense_out": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "gs_part_prunes_dense_in": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "gs_part_xbfs_groups": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "gs_part_xbfs_begin": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "gs_part_xbfs_expand": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "gs_part_xbfs_send": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "gs_part_xbfs_apply": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int,
                                     C.POINTER(C.c_uint32)]),
    "gs_part_xbfs_end": (C.c_int, [C.c_void_p, C.c_int]),
    "gs_part_xbfs_expand_async": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, C.c_void_p]),
    "gs_part_xbfs_apply_async": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]),
    "gs_part_xbfs_async_status": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_void_p,
                                            C.c_size_t]),
    "gs_stream": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "gs_part_xround_finish": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int, C.POINTER(C.c_uint32)]),
    "gs_part_stats_out": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "gs_part_stats_in": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "gs_create": (C.c_int, [C.POINTER(Params), C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_void_p)]),
    "gs_destroy": (None, [C.c_void_p]),
    "gs_set_slots": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "gs_sync": (C.c_int, [C.c_void_p]),
    "gs_init_active_sets": (C.c_int, [C.c_void_p]),
    "gs_set_active_set_entry": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32]),
    "gs_get_active_set_entry": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint32,
                                          C.POINTER(C.c_uint32)]),
    "gs_fail_nodes": (C.c_int, [C.c_void_p, C.c_void_p]),
    "gs_run_gossip": (C.c_int, [C.c_void_p]),
    "gs_consume_messages": (C.c_int, [C.c_void_p]),
    "gs_send_prunes": (C.c_int, [C.c_void_p]),
    "gs_prune_connections": (C.c_int, [C.c_void_p]),
    "gs_chance_to_rotate": (C.c_int, [C.c_void_p, C.c_uint32]),
    "gs_record_round": (C.c_int, [C.c_void_p]),
    "gs_round": (C.c_int, [C.c_void_p, C.c_uint32, C.c_int]),
    "gs_read_hops": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "gs_read_inbound": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "gs_read_prunes": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_size_t,
                                 C.POINTER(C.c_size_t)]),
    "gs_read_cache": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32), C.c_void_p, C.c_void_p,
                                C.c_uint32, C.POINTER(C.c_uint32)]),
    "gs_read_pruned": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]),
    "gs_read_counters": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_read_active_sets": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_read_caches": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "gs_read_pruned_all": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "gs_read_round_summaries": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "gs_read_accumulators": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
    "gs_read_failed": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "gs_kernel_time": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "gs_kernel_time_reset": (C.c_int, [C.c_void_p]),
    "gs_engine_round_kind": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "gs_engine_bfs_geometry": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    "gs_engine_memory": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "gs_engine_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint64)]),
    "gs_hops_stat_new": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p]),
    "gs_stat_collection_calculate": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p]),
    "gs_run_simulations": (C.c_int, [C.POINTER(SimConfig), C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p)]),
    "gs_result_free": (None, [C.c_void_p]),
    "gs_result_f64": (C.c_size_t, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_void_p, C.c_size_t]),
    "gs_result_u64": (C.c_size_t, [C.c_void_p, C.c_uint32, C.c_char_p, C.c_void_p, C.c_size_t]),
}

_lib = None


def source_hash():
    """sha256 (16 hex digits) of the device sources on disk (csrc/*.hip, csrc/*.h), hashed
    as gen_khash.py hashes them when the library is built."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(PKG_DIR, "csrc")
    for name in sorted(os.listdir(d)):
        if name.endswith((".hip", ".h")):
            h.update(name.encode() + b"\0")
            with open(os.path.join(d, name), "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]


def kernel_hash():
    """The kernel hash compiled into the LOADED libgossip_hip.so (gs_kernel_hash), when it
    equals the sources on disk; None under GS_LIB_VARIANT (an A/B build) or when the library
    is out of date with its sources. Profiles under profiles/ carry the hash of the kernels
    they measured; bench.py reports a profile's figures only when it equals this one."""
    if os.environ.get("GS_LIB_VARIANT"):
        return None
    built = lib().gs_kernel_hash().decode()
    return built if built == source_hash() else None


def build(quiet=True):
    """Compile libgossip_hip.so (and the gossip-sim CLI) for gfx950 in-tree."""
    cmd = ["make", "-C", PKG_DIR, "-j8"]
    subprocess.check_call(cmd, stdout=subprocess.DEVNULL if quiet else None)


def lib():
    """Load the engine library; raises if it is missing (no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise GsError(-2, f"{LIB_PATH} is missing: run `make -C gossip-sim_amd` (no CPU fallback exists)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in EXPORTS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def _check(rc):
    if rc != 0:
        raise GsError(rc, lib().gs_last_error().decode())


def b58encode(b: bytes) -> str:
    n = int.from_bytes(b, "big")
    s = ""
    while n:
        n, r = divmod(n, 58)
        s = B58[r] + s
    return "1" * (len(b) - len(b.lstrip(b"\x00"))) + s


def ids_from_pubkeys(pubkeys):
    """Node id = rank of the base58 string (the consume tie-break order, gossip.rs:639-645)."""
    strs = [b58encode(p) for p in pubkeys]
    order = sorted(range(len(strs)), key=lambda i: strs[i])
    ids = [0] * len(strs)
    for r, i in enumerate(order):
        ids[i] = r
    return ids


class Engine:
    """One engine = one device + one shared active-set trajectory + n_slots sims."""

    def __init__(self, stakes, n_slots, *, fanout=6, active_set_size=12, rotation_probability=0.013333, seed=0,
                 device=0, bfs_mode=GS_BFS_AUTO, inbound_capacity=0, profile=False, split_round=False,
                 narrow_wave_path=False, binned_all_levels=False, wide_records=False, no_small_levels=False,
                 mispredict_levels=False, frontier_exchange=False, part=None):
        L = lib()
        self.stakes = np.ascontiguousarray(stakes, dtype=np.uint64)
        self.n = len(self.stakes)
        self.n_slots = n_slots
        self.active_set_size = active_set_size
        p = Params(fanout, active_set_size, rotation_probability, seed, device, bfs_mode, inbound_capacity,
                   (GS_FLAG_PROFILE if profile else 0) | (GS_FLAG_SPLIT_ROUND if split_round else 0) |
                   (GS_FLAG_NARROW_WAVE_PATH if narrow_wave_path else 0) |
                   (GS_FLAG_BINNED_ALL_LEVELS if binned_all_levels else 0) |
                   (GS_FLAG_WIDE_RECORDS if wide_records else 0) | (GS_FLAG_NO_SMALL_LEVELS if no_small_levels else 0) |
                   (GS_FLAG_MISPREDICT_LEVELS if mispredict_levels else 0) |
                   (GS_FLAG_FRONTIER_EXCHANGE if frontier_exchange else 0))
        h = C.c_void_p()
        if part is None:
            _check(L.gs_create(C.byref(p), _ptr(self.stakes), self.n, n_slots, C.byref(h)))
        else:  # (rank, nranks): one rank of a node-range partition (gossip_sim_amd.partition)
            _check(L.gs_create_part(C.byref(p), _ptr(self.stakes), self.n, n_slots, part[0], part[1], C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().gs_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def info(self):
        n, s, m, b = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint64()
        _check(lib().gs_engine_info(self.h, C.byref(n), C.byref(s), C.byref(m), C.byref(b)))
        f = C.c_uint32()
        _check(lib().gs_engine_round_kind(self.h, C.byref(f)))
        pb, ob = C.c_uint64(), C.c_uint64()
        _check(lib().gs_engine_memory(self.h, C.byref(pb), C.byref(ob)))
        return {"n_nodes": n.value, "n_slots": s.value, "bfs_mode": m.value, "device_bytes": b.value,
                "pair_bytes": pb.value, "other_bytes": ob.value, "fused_round": bool(f.value),
                "bfs_persistent": bool(self.bfs_geometry()["persistent_wgs"])}

    def bfs_geometry(self):
        """Multi / hybrid BFS geometry (diagnostics): expand slice, coarse and fine bins, group width, groups."""
        out = np.zeros(6, dtype=np.uint32)
        _check(lib().gs_engine_bfs_geometry(self.h, _ptr(out), 6))
        return dict(zip(["expand_slice", "coarse_bins", "fine_bins", "group_width", "groups", "persistent_wgs"],
                        out.tolist()))

    def set_slots(self, origins, min_ingress=2, thresholds=0.15):
        S = self.n_slots
        mi = np.broadcast_to(np.asarray(min_ingress), (S,))
        th = np.broadcast_to(np.asarray(thresholds, dtype=np.float64), (S,))
        arr = (Slot * S)(*[Slot(int(o), int(m), float(t)) for o, m, t in zip(origins, mi, th)])
        _check(lib().gs_set_slots(self.h, C.cast(arr, C.c_void_p), S))

    def init_active_sets(self):
        _check(lib().gs_init_active_sets(self.h))

    def set_entry(self, node, bucket, peers):
        a = np.ascontiguousarray(peers, dtype=np.uint32)
        _check(lib().gs_set_active_set_entry(self.h, node, bucket, _ptr(a), len(a)))

    def get_entry(self, node, bucket):
        out = np.zeros(64, dtype=np.uint32)
        ln = C.c_uint32()
        _check(lib().gs_get_active_set_entry(self.h, node, bucket, _ptr(out), 64, C.byref(ln)))
        return [int(x) for x in out[:ln.value]]

    def fail_nodes(self, fractions):
        f = np.ascontiguousarray(np.broadcast_to(np.asarray(fractions, dtype=np.float64), (self.n_slots,)))
        _check(lib().gs_fail_nodes(self.h, _ptr(f)))

    # --- Cluster steps -------------------------------------------------------
    def run_gossip(self):
        _check(lib().gs_run_gossip(self.h))

    def consume_messages(self):
        _check(lib().gs_consume_messages(self.h))

    def send_prunes(self):
        _check(lib().gs_send_prunes(self.h))

    def prune_connections(self):
        _check(lib().gs_prune_connections(self.h))

    def chance_to_rotate(self, round_index):
        _check(lib().gs_chance_to_rotate(self.h, round_index))

    def record_round(self):
        _check(lib().gs_record_round(self.h))

    def round(self, round_index, record=False):
        _check(lib().gs_round(self.h, round_index, 1 if record else 0))

    def sync(self):
        _check(lib().gs_sync(self.h))

    # --- readbacks -----------------------------------------------------------
    def hops(self, slot):
        out = np.zeros(self.n, dtype=np.uint8)
        _check(lib().gs_read_hops(self.h, slot, _ptr(out)))
        return out

    def distances(self, slot):
        h = self.hops(slot).astype(np.uint64)
        h[h == HOP_UNREACHED] = np.uint64(2**64 - 1)
        return h

    def inbound(self, slot, cap=None):
        cap = cap or 64 * self.n
        off = np.zeros(self.n + 1, dtype=np.uint32)
        src = np.zeros(cap, dtype=np.uint32)
        hop = np.zeros(cap, dtype=np.uint8)
        _check(lib().gs_read_inbound(self.h, slot, _ptr(off), _ptr(src), _ptr(hop), cap))
        return off, src, hop

    def inbound_lists(self, slot):
        off, src, hop = self.inbound(slot)
        return [list(zip(src[off[v]:off[v + 1]].tolist(), hop[off[v]:off[v + 1]].tolist())) for v in range(self.n)]

    def prunes(self, slot):
        cap = 96 * self.n
        a = np.zeros(cap, dtype=np.uint32)
        b = np.zeros(cap, dtype=np.uint32)
        cnt = C.c_size_t()
        _check(lib().gs_read_prunes(self.h, slot, _ptr(a), _ptr(b), cap, C.byref(cnt)))
        return list(zip(a[:cnt.value].tolist(), b[:cnt.value].tolist()))

    def cache(self, slot, node):
        up, ln = C.c_uint32(), C.c_uint32()
        k = np.zeros(128, dtype=np.uint32)
        s = np.zeros(128, dtype=np.uint32)
        _check(lib().gs_read_cache(self.h, slot, node, C.byref(up), _ptr(k), _ptr(s), 128, C.byref(ln)))
        return up.value, dict(zip(k[:ln.value].tolist(), s[:ln.value].tolist()))

    def pruned(self, slot, node):
        m = C.c_uint32()
        _check(lib().gs_read_pruned(self.h, slot, node, C.byref(m)))
        return m.value

    def active_sets(self):
        """(peers[n, 25, asz] FIFO order, lens[n, 25])."""
        asz = self.active_set_size
        peers = np.zeros(self.n * 25 * asz, dtype=np.uint32)
        lens = np.zeros(self.n * 25, dtype=np.uint8)
        _check(lib().gs_read_active_sets(self.h, _ptr(peers), _ptr(lens)))
        return peers.reshape(self.n, 25, asz), lens.reshape(self.n, 25)

    def caches(self, slot):
        """(upserts[n], lens[n], keys[n, 96], scores[n, 96]); keys sorted per node."""
        up = np.zeros(self.n, dtype=np.uint32)
        ln = np.zeros(self.n, dtype=np.uint32)
        k = np.zeros(self.n * 96, dtype=np.uint32)
        s = np.zeros(self.n * 96, dtype=np.uint32)
        _check(lib().gs_read_caches(self.h, slot, _ptr(up), _ptr(ln), _ptr(k), _ptr(s)))
        return up, ln, k.reshape(self.n, 96), s.reshape(self.n, 96)

    def pruned_all(self, slot):
        out = np.zeros(self.n, dtype=np.uint32)
        _check(lib().gs_read_pruned_all(self.h, slot, _ptr(out)))
        return out

    def counters(self, slot):
        e = np.zeros(self.n, dtype=np.uint32)
        i = np.zeros(self.n, dtype=np.uint32)
        p = np.zeros(self.n, dtype=np.uint32)
        _check(lib().gs_read_counters(self.h, slot, _ptr(e), _ptr(i), _ptr(p)))
        return e, i, p

    def summaries(self):
        cap = 1 << 16
        while True:
            out = np.zeros(cap, dtype=SUMMARY_DTYPE)
            cnt = C.c_size_t()
            rc = lib().gs_read_round_summaries(self.h, _ptr(out), cap, C.byref(cnt))
            if rc == -4 and cnt.value > cap:
                cap = cnt.value
                continue
            _check(rc)
            return out[:cnt.value].reshape(-1, self.n_slots)

    def mst(self, slot):
        """Cluster::mst (gossip.rs:580-591): {discoverer: sorted nodes it first discovered}."""
        parent = np.zeros(self.n, dtype=np.uint32)
        _check(lib().gs_read_mst(self.h, slot, _ptr(parent)))
        out = {}
        for v in np.nonzero(parent != 0xFFFFFFFF)[0]:
            out.setdefault(int(parent[v]), []).append(int(v))
        return out

    def pushes(self, slot):
        """Cluster::pushes (gossip.rs:566-573): {src: sorted peers it pushed to}."""
        off, src, _ = self.inbound(slot)
        out = {}
        for v in range(self.n):
            for s in src[off[v]:off[v + 1]].tolist():
                out.setdefault(int(s), []).append(v)
        return {k: sorted(v) for k, v in out.items()}

    def accumulators(self, slot):
        e = np.zeros(self.n, dtype=np.uint64)
        i = np.zeros(self.n, dtype=np.uint64)
        p = np.zeros(self.n, dtype=np.uint64)
        st = np.zeros(self.n, dtype=np.uint32)
        hh = np.zeros(256, dtype=np.uint64)
        _check(lib().gs_read_accumulators(self.h, slot, _ptr(e), _ptr(i), _ptr(p), _ptr(st), _ptr(hh)))
        return e, i, p, st, hh

    def failed(self, slot):
        out = np.zeros(self.n, dtype=np.uint8)
        _check(lib().gs_read_failed(self.h, slot, _ptr(out)))
        return out

    def kernel_time(self, family):
        ms, n = C.c_double(), C.c_uint64()
        _check(lib().gs_kernel_time(self.h, family.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def kernel_time_reset(self):
        _check(lib().gs_kernel_time_reset(self.h))


class HopsStatOut(C.Structure):
    _fields_ = [("mean", C.c_double), ("median", C.c_double), ("max", C.c_uint64), ("min", C.c_uint64)]


def hops_stat(values):
    """HopsStat::new (gossip_stats.rs:47-98) over raw distances (u64::MAX = unreached)."""
    a = np.ascontiguousarray(values, dtype=np.uint64)
    out = HopsStatOut()
    _check(lib().gs_hops_stat_new(_ptr(a), len(a), C.byref(out)))
    return out.mean, out.median, out.max, out.min


def stat_collection(values):
    a = np.ascontiguousarray(values, dtype=np.float64)
    out = np.zeros(4, dtype=np.float64)
    _check(lib().gs_stat_collection_calculate(_ptr(a), len(a), _ptr(out)))
    return tuple(float(x) for x in out)


class SimResult:
    def __init__(self, h, n_sims):
        self.h = h
        self.n_sims = n_sims

    def __del__(self):
        if getattr(self, "h", None):
            lib().gs_result_free(self.h)

    def f64(self, sim, name, cap=1 << 16):
        out = np.zeros(cap, dtype=np.float64)
        n = lib().gs_result_f64(self.h, sim, name.encode(), _ptr(out), cap)
        if n == C.c_size_t(-1).value:
            raise KeyError(name)
        return out[:n].copy()

    def u64(self, sim, name, cap=1 << 20):
        out = np.zeros(cap, dtype=np.uint64)
        n = lib().gs_result_u64(self.h, sim, name.encode(), _ptr(out), cap)
        if n == C.c_size_t(-1).value:
            raise KeyError(name)
        return out[:n].copy()


def run_simulations(stakes, *, n_sims=1, origin_ranks=None, min_ingress=None, thresholds=None, fractions=None,
                    fanout=6, asz=12, iterations=1, warm_up=200, p=0.013333, thr=0.15, min_ingress_nodes=2,
                    fraction_to_fail=0.1, when_to_fail=0, nb_stranded=10, nb_message=5, nb_hops=15, test_type=0,
                    seed=0, device=0, bfs_mode=GS_BFS_AUTO):
    """gossip_main.rs run_simulation for n_sims sims sharing one trajectory (one engine)."""
    st = np.ascontiguousarray(stakes, dtype=np.uint64)
    cfg = SimConfig(fanout, asz, iterations, warm_up, min_ingress_nodes, when_to_fail, p, thr, fraction_to_fail,
                    nb_stranded, nb_message, nb_hops, test_type, seed, device, bfs_mode)

    def arr(x, dt):
        return None if x is None else np.ascontiguousarray(x, dtype=dt)

    r, mi, th, fr = arr(origin_ranks, np.uint32), arr(min_ingress, np.uint32), arr(thresholds, np.float64), \
        arr(fractions, np.float64)
    h = C.c_void_p()
    _check(lib().gs_run_simulations(C.byref(cfg), _ptr(st), len(st), n_sims,
                                    None if r is None else _ptr(r), None if mi is None else _ptr(mi),
                                    None if th is None else _ptr(th), None if fr is None else _ptr(fr), C.byref(h)))
    return SimResult(h, n_sims)
