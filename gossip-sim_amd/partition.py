"""Node-range partition of a simulation batch over ranks.

One process per GPU. Every rank creates its engine with gs_create_part on the same
stakes, slots and seed: it owns the node ids [node_lo, node_hi) and keeps per-(slot,
node) state -- hops, in-degrees, received caches, counters, accumulators -- for those
nodes only. Active-set rows, prune masks and failed flags are replicated. A round is the
call sequence of include/gossip_hip.h gs_part_*; this class runs it and does the
exchanges with torch.distributed:

  after consume   all-gather of the ranks' prune-record counts; then, the same choice
                  on every rank, either an all-gather of the records (padded to the
                  largest count; every rank applies every record) or -- when a rank's
                  records overflow its preallocated buffer or the dense form is smaller,
                  as in a prune wave -- a SUM all-reduce of dense [N][S] ring-slot bit
                  words (bit-disjoint across ranks, so SUM = OR). Either way this is
                  prune_connections on the replicated masks. Nothing is exchanged per BFS
                  level: each rank runs the whole BFS over its replicated rows.
  recorded round  SUM of the statistics partials (u64 words).

With the "nccl" backend (RCCL over xGMI) the exchange buffers are torch tensors on the
rank's GPU and the engine copies device to device; with "gloo" they are host tensors.
Results on owned nodes, and every summary, are bit-identical to one engine over all
nodes (tests/test_partition.py).
"""
import ctypes as C
import os
import time

import numpy as np

from . import GS_BFS_MULTI, Engine, _check, lib


def coarse_bin_nodes(n):
    """Nodes per coarse destination bin of the multi-source BFS for an n-node graph (the
    rule of gs_bfs_multi.hip mv_geometry: about 256 bins, 2^6 .. 2^13 nodes each)."""
    ub = max(1, (n - 1).bit_length())
    return 1 << min(13, max(6, ub - 8 if ub > 8 else 0))


def partition_unit(n, frontier=False):
    """Node ids per partition unit: 1,024; a frontier-exchange partition owns whole coarse
    bins as well (each level's records for a bin go to one rank)."""
    return max(1024, coarse_bin_nodes(n)) if frontier else 1024


def partition_ranges(n, world, frontier=False):
    """The node ranges gs_create_part gives ranks 0..world-1: contiguous, whole units
    (partition_unit) of ceil(n / world) rounded up. Raises ValueError when a trailing rank
    would own no node (e.g. n = 3,000 over 4 ranks) -- identically on every rank, before any
    engine or collective exists, so no rank is left waiting in a collective."""
    unit = partition_unit(n, frontier)
    c = -(-(-(-n // world)) // unit) * unit
    out = [(min(n, r * c), min(n, r * c + c)) for r in range(world)]
    if any(lo >= hi for lo, hi in out):
        raise ValueError(f"a node-range partition of {n} nodes over {world} ranks leaves a rank without nodes "
                         f"(ranges are whole {unit}-id units of {c}); use at most {-(-n // c)} ranks")
    return out


class PartitionedEngine:
    def __init__(self, stakes, n_slots, *, group=None, device=0, exchange="auto", bfs="replicated",
                 profile=False, serialize=False, async_levels=True, **engine_kw):
        import torch
        import torch.distributed as tdist
        self.torch, self.tdist, self.group = torch, tdist, group
        self.rank = tdist.get_rank(group)
        self.world = tdist.get_world_size(group)
        engine_kw["bfs_mode"] = GS_BFS_MULTI
        if bfs not in ("replicated", "frontier"):
            raise ValueError("bfs must be replicated or frontier")
        self.frontier = bfs == "frontier"
        ranges = partition_ranges(len(stakes), self.world, self.frontier)  # (raises the same on every rank)
        self.eng = Engine(stakes, n_slots, device=device, part=(self.rank, self.world),
                          frontier_exchange=self.frontier, **engine_kw)
        sw = C.c_size_t()
        lo, hi = C.c_uint32(), C.c_uint32()
        _check(lib().gs_part_sizes(self.eng.h, C.byref(sw), C.byref(lo), C.byref(hi)))
        self.node_lo, self.node_hi = lo.value, hi.value
        assert (self.node_lo, self.node_hi) == ranges[self.rank], (self.node_lo, self.node_hi, ranges)
        self.levels = 0         # BFS levels of the last round (frontier exchange)
        self.level_bytes = 0    # frontier-exchange bytes this rank received over all rounds
        self.on_device = tdist.get_backend(group) == "nccl"
        if self.on_device:
            torch.cuda.set_device(device)
        self.dev = torch.device("cuda", device) if self.on_device else torch.device("cpu")
        self.stats = torch.zeros(sw.value, dtype=torch.int64, device=self.dev)
        rc, dw = C.c_size_t(), C.c_size_t()
        _check(lib().gs_part_exchange_sizes(self.eng.h, C.byref(rc), C.byref(dw)))
        self.record_cap, self.dense_words = rc.value, dw.value
        if exchange not in ("auto", "records", "dense"):
            raise ValueError("exchange must be auto, records or dense")
        self.exchange = exchange
        # [N * S] int32 dense exchange buffer (4 * S * N bytes: 640 MB at C5's 10M x 16):
        # allocated here for exchange="dense"; for "auto" only in the first round that goes
        # dense, after every rank has agreed that its allocation succeeded (_dense_buffer), so
        # a rank that runs out of memory fails with the others instead of leaving them waiting
        # in the all-reduce
        self.dense = None
        if exchange == "dense":
            self.dense = torch.zeros(self.dense_words, dtype=torch.int32, device=self.dev)
        self.records = 0       # prune records of the last round (all ranks)
        self.last_mode = None  # "records" / "dense" / None (no prunes)
        self.bytes_in = 0      # exchange bytes this rank received over all rounds (collective payload)
        # profile=True: seconds per phase of this rank (device-synchronised wall time around
        # each engine call; "exchange" = the collectives). serialize=True runs the ranks' engine
        # calls one rank at a time (barriers in between), so ranks sharing one GPU time their
        # own kernels alone: the per-rank share of a K-GPU run, measured on one device.
        self.prof = {} if profile else None
        self.serialize = serialize
        # frontier exchange: after a round of the synchronous level loop, the next rounds run
        # their levels without a host wait (fixed-capacity message slots sized from the last
        # round, _async_levels); async_levels=False keeps the per-level size exchange
        # (not with serialize over several ranks: the loop's collectives cannot take turns)
        self.async_levels = async_levels and self.frontier and not (serialize and self.world > 1)
        self.pred = {}          # slot group -> message slot words per level (agreed by every rank)
        self.async_rounds = 0   # groups run by the asynchronous loop / redone after an overflow
        self.async_redo = 0
        self._ext = None
        if self.async_levels and self.on_device:
            sp = C.c_void_p()
            _check(lib().gs_stream(self.eng.h, C.byref(sp)))
            self._ext = torch.cuda.ExternalStream(sp.value, device=self.dev)
        bsc = coarse_bin_nodes(len(stakes))
        self._hdr = max(-(-(hi - lo) // bsc) + 2 for lo, hi in ranges)  # bin headers per message, at most

    # the Engine's other calls (set_slots, init_active_sets, fail_nodes, readbacks) are
    # replicated or rank-local and need no exchange
    def __getattr__(self, name):
        return getattr(self.eng, name)

    def _ptr(self, t):
        return C.c_void_p(t.data_ptr())

    def _dense_buffer(self):
        """The dense exchange buffer, allocated on first use with a MIN all-reduce of an ok
        flag: every rank raises if any rank's allocation failed."""
        if self.dense is not None:
            return self.dense
        torch = self.torch
        buf, err = None, None
        try:
            buf = torch.zeros(self.dense_words, dtype=torch.int32, device=self.dev)
        except RuntimeError as ex:  # (torch.cuda.OutOfMemoryError is a RuntimeError)
            err = ex
        ok = torch.tensor([0 if buf is None else 1], dtype=torch.int64, device=self.dev)
        self.tdist.all_reduce(ok, op=self.tdist.ReduceOp.MIN, group=self.group)
        if int(ok.item()) == 0:
            raise RuntimeError(f"dense prune exchange: a rank could not allocate {4 * self.dense_words} bytes"
                               + (f" (this rank: {err})" if err else ""))
        self.dense = buf
        return buf

    def _timed(self, name, fn):
        """fn() on this rank, timed into prof[name] when profiling (one rank at a time when
        serialize)."""
        if self.prof is None:
            return fn()
        out = None
        for r in range(self.world if self.serialize else 1):
            if self.serialize:
                self.tdist.barrier(group=self.group)
            if not self.serialize or r == self.rank:
                self.eng.sync()
                t0 = time.perf_counter()
                out = fn()
                self.eng.sync()
                self.prof[name] = self.prof.get(name, 0.0) + time.perf_counter() - t0
        if self.serialize:
            self.tdist.barrier(group=self.group)
        return out

    def _xchg(self, fn):
        """A collective step, timed into prof["exchange"] when profiling."""
        if self.prof is None:
            return fn()
        t0 = time.perf_counter()
        out = fn()
        self._done()
        self.prof["exchange"] = self.prof.get("exchange", 0.0) + time.perf_counter() - t0
        return out

    def _done(self):
        # the engine reads the buffers on its own stream: torch's collective must be complete
        if self.on_device:
            self.torch.cuda.synchronize()

    def _async_levels_run(self, caps):
        """Levels 0 .. len(caps) - 1 of the begun group without a host wait: every rank packs
        its message to rank q into slot q of a K x cap buffer (gs_part_xbfs_expand_async),
        the all-to-all moves equal slots (RCCL: enqueued on the engine's stream, so it
        orders with the kernels), the apply reads the slots' headers. One status read at the
        end: (overflow on any rank, next-level entries on any rank, this rank's words log)."""
        torch, tdist, L, h, K = self.torch, self.tdist, lib(), self.eng.h, self.world
        cmax = max(caps)
        dev = torch.device("cuda", torch.cuda.current_device()) if not self.on_device else self.dev
        send = torch.empty(K * cmax, dtype=torch.int64, device=dev)
        recv = torch.empty(K * cmax, dtype=torch.int64, device=dev)
        self.eng.sync()  # (the buffers exist before the engine's stream uses them)
        for d, cap in enumerate(caps):
            _check(L.gs_part_xbfs_expand_async(h, d, cap, self._ptr(send)))
            if self.on_device:
                with torch.cuda.stream(self._ext):
                    tdist.all_to_all_single(recv[:K * cap], send[:K * cap], group=self.group)
            else:  # gloo: the slots through host memory
                self.eng.sync()
                hs = send[:K * cap].cpu()
                hr = torch.empty_like(hs)
                tdist.all_to_all_single(hr, hs, group=self.group)
                recv[:K * cap].copy_(hr)
                torch.cuda.synchronize()
            _check(L.gs_part_xbfs_apply_async(h, d, self._ptr(recv), cap))
            self.level_bytes += 8 * K * cap
        n, ov = C.c_uint32(), C.c_uint32()
        log = np.zeros((len(caps), K), dtype=np.uint64)
        _check(L.gs_part_xbfs_async_status(h, C.byref(n), C.byref(ov), log.ctypes.data_as(C.c_void_p), len(caps)))
        flags = torch.tensor([ov.value, n.value], dtype=torch.int64, device=self.dev)
        tdist.all_reduce(flags, op=tdist.ReduceOp.MAX, group=self.group)
        del send, recv
        return int(flags[0].item()), int(flags[1].item()), n.value, log

    def _predict(self, g, words):
        """The next round's slot words per level (every rank the same): the largest message of
        each level over ranks and destinations, +25 % and 1,024 words of headroom."""
        torch, tdist = self.torch, self.tdist
        w = torch.zeros(256, dtype=torch.int64, device=self.dev)
        w[:len(words)] = torch.tensor([int(x) for x in words], dtype=torch.int64)
        nl = torch.tensor([len(words)], dtype=torch.int64, device=self.dev)
        tdist.all_reduce(w, op=tdist.ReduceOp.MAX, group=self.group)
        tdist.all_reduce(nl, op=tdist.ReduceOp.MAX, group=self.group)
        w = w.cpu().numpy()[:int(nl.item())]
        force = int(os.environ.get("GS_XBFS_SLOT_WORDS", "0"))  # (tests: slots too small -> overflow -> redo)
        self.pred[g] = [max(force if force else int(x * 1.25) + 1024, self._hdr) for x in w]

    def _frontier_bfs(self, record):
        """Cluster::run_gossip (gossip.rs:494-615) over the partition with a frontier exchange
        per level: each rank expands only its own frontier entries; the level's push records
        go to the ranks owning their destinations (two all-to-alls: the counts, then the
        messages), which apply them; the BFS ends when no rank has a next-level entry. Each
        group's own nodes are then gathered and consumed (consume_messages, gossip.rs:618-653)."""
        torch, tdist, L, h, dev = self.torch, self.tdist, lib(), self.eng.h, int(self.on_device)
        K = self.world
        ng = C.c_uint32()
        _check(L.gs_part_xbfs_groups(h, C.byref(ng)))
        n = C.c_uint32()
        wto = np.zeros(K, dtype=np.uint64)
        wfrom = np.zeros(K, dtype=np.uint64)
        levels = 0
        T, X = self._timed, self._xchg
        for g in range(ng.value):
            T("begin", lambda: _check(L.gs_part_xbfs_begin(h, g, C.byref(n))))
            words = []  # this rank's largest message per level (the next round's slot sizes)
            d = 0
            caps = self.pred.get(g) if self.async_levels else None
            if caps:
                over, more, nloc, log = T("async_levels", lambda: self._async_levels_run(caps))
                self.async_rounds += 1
                if over:  # a message outgrew its slot somewhere: redo the group, sizes exchanged per level
                    self.async_redo += 1
                    T("begin", lambda: _check(L.gs_part_xbfs_begin(h, g, C.byref(n))))
                else:
                    words = [int(x) for x in log.max(axis=1)]
                    d = len(caps)
                    n.value = nloc  # (the sync loop below continues when the BFS went deeper)
            tot = torch.tensor([n.value], dtype=torch.int64, device=self.dev)
            X(lambda: tdist.all_reduce(tot, group=self.group))
            while int(tot.item()) > 0:
                T("expand", lambda: _check(L.gs_part_xbfs_expand(h, d, wto.ctypes.data_as(C.c_void_p))))
                if d < len(words):
                    words[d] = max(words[d], int(wto.max()))
                else:
                    words.append(int(wto.max()))
                cto = torch.tensor(wto.astype(np.int64), device=self.dev)
                cfrom = torch.zeros(K, dtype=torch.int64, device=self.dev)
                X(lambda: tdist.all_to_all_single(cfrom, cto, group=self.group))
                wfrom[:] = cfrom.cpu().numpy().astype(np.uint64)
                send = torch.empty(int(wto.sum()), dtype=torch.int64, device=self.dev)
                T("send", lambda: _check(L.gs_part_xbfs_send(h, self._ptr(send), dev)))
                recv = torch.empty(int(wfrom.sum()), dtype=torch.int64, device=self.dev)
                X(lambda: tdist.all_to_all_single(recv, send, output_split_sizes=[int(x) for x in wfrom],
                                                  input_split_sizes=[int(x) for x in wto], group=self.group))
                self._done()
                T("apply", lambda: _check(L.gs_part_xbfs_apply(h, d, self._ptr(recv), wfrom.ctypes.data_as(C.c_void_p),
                                                               dev, C.byref(n))))
                self.level_bytes += 8 * int(wfrom.sum())
                tot = torch.tensor([n.value], dtype=torch.int64, device=self.dev)
                X(lambda: tdist.all_reduce(tot, group=self.group))
                d += 1
            T("gather_consume", lambda: _check(L.gs_part_xbfs_end(h, int(bool(record)))))
            if self.async_levels:
                # (levels past the BFS's end in the async run sent nothing: trimmed)
                while len(words) > 1 and words[-1] <= self._hdr:
                    words.pop()
                self._predict(g, words)
            levels = max(levels, d)
        self.levels = levels

    def round(self, round_index, record=False):
        """One iteration of gossip_main.rs:449-564 over the partition."""
        torch, tdist, L, h, dev = self.torch, self.tdist, lib(), self.eng.h, int(self.on_device)
        n = C.c_uint32()
        T = self._timed
        if self.frontier:
            self._frontier_bfs(record)
            T("prune", lambda: _check(L.gs_part_xround_finish(h, round_index, int(bool(record)), C.byref(n))))
        else:
            T("round", lambda: _check(L.gs_part_round(h, round_index, int(bool(record)), C.byref(n))))
        counts = [torch.zeros(1, dtype=torch.int64, device=self.dev) for _ in range(self.world)]
        tdist.all_gather(counts, torch.tensor([n.value], dtype=torch.int64, device=self.dev), group=self.group)
        counts = [int(c.item()) for c in counts]
        m = max(counts)
        self.last_mode = None
        if m:
            # records: every rank receives world * m padded records (8 B); dense: a ring
            # all-reduce moves ~2 x the S * N words (4 B) through every rank
            rec_bytes, dense_bytes = 8 * m * self.world, 8 * self.dense_words
            dense = self.exchange == "dense" or (self.exchange == "auto" and
                                                 (m > self.record_cap or rec_bytes > dense_bytes))
            if not dense and m > self.record_cap:
                raise RuntimeError(f"{m} prune records exceed the record buffer ({self.record_cap}); "
                                   "use exchange='auto' or 'dense'")
            if dense:
                self._dense_buffer()
                T("prunes_out", lambda: _check(L.gs_part_prunes_dense_out(h, self._ptr(self.dense), dev)))
                self._xchg(lambda: tdist.all_reduce(self.dense, group=self.group))
                self._done()
                T("prunes_in", lambda: _check(L.gs_part_prunes_dense_in(h, self._ptr(self.dense), dev)))
                self.bytes_in += dense_bytes
                self.last_mode = "dense"
            else:
                mine = torch.zeros(2 * m, dtype=torch.int32, device=self.dev)
                if n.value:
                    T("prunes_out", lambda: _check(L.gs_part_prunes_out(h, self._ptr(mine), dev)))
                parts = [torch.zeros(2 * m, dtype=torch.int32, device=self.dev) for _ in range(self.world)]
                self._xchg(lambda: tdist.all_gather(parts, mine, group=self.group))
                recs = torch.cat([p[:2 * c] for p, c in zip(parts, counts)])
                self._done()
                T("prunes_in", lambda: _check(L.gs_part_prunes_in(h, self._ptr(recs), sum(counts), dev)))
                self.bytes_in += rec_bytes
                self.last_mode = "records"
        self.records = sum(counts)
        T("rotate", lambda: self.eng.chance_to_rotate(round_index))
        if record:
            T("stats", lambda: _check(L.gs_part_stats_out(h, self._ptr(self.stats), dev)))
            self._xchg(lambda: tdist.all_reduce(self.stats, group=self.group))
            self._done()
            T("stats_in", lambda: _check(L.gs_part_stats_in(h, self._ptr(self.stats), dev)))

    def owned(self, arr):
        """The owned slice of a per-node array."""
        return np.asarray(arr)[self.node_lo:self.node_hi]
