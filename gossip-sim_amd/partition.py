"""Node-range partition of a simulation batch over ranks.

One process per GPU. Every rank creates its engine with gs_create_part on the same
stakes, slots and seed: it owns the node ids [node_lo, node_hi) and keeps per-(slot,
node) state -- hops, in-degrees, received caches, counters, accumulators -- for those
nodes only. Active-set rows, prune masks and failed flags are replicated. A round is the
call sequence of include/gossip_hip.h gs_part_*; this class runs it and does the
exchanges with torch.distributed:

  after consume   all-gather of the ranks' prune-record counts, then of the records
                  (padded to the largest count); every rank applies every record
                  (prune_connections on the replicated masks). Nothing is exchanged
                  per BFS level: each rank runs the whole BFS over its replicated rows.
  recorded round  SUM of the statistics partials (u64 words).

With the "nccl" backend (RCCL over xGMI) the exchange buffers are torch tensors on the
rank's GPU and the engine copies device to device; with "gloo" they are host tensors.
Results on owned nodes, and every summary, are bit-identical to one engine over all
nodes (tests/test_partition.py).
"""
import ctypes as C

import numpy as np

from . import GS_BFS_MULTI, Engine, _check, lib


class PartitionedEngine:
    def __init__(self, stakes, n_slots, *, group=None, device=0, **engine_kw):
        import torch
        import torch.distributed as tdist
        self.torch, self.tdist, self.group = torch, tdist, group
        self.rank = tdist.get_rank(group)
        self.world = tdist.get_world_size(group)
        engine_kw["bfs_mode"] = GS_BFS_MULTI
        self.eng = Engine(stakes, n_slots, device=device, part=(self.rank, self.world), **engine_kw)
        sw = C.c_size_t()
        lo, hi = C.c_uint32(), C.c_uint32()
        _check(lib().gs_part_sizes(self.eng.h, C.byref(sw), C.byref(lo), C.byref(hi)))
        self.node_lo, self.node_hi = lo.value, hi.value
        self.on_device = tdist.get_backend(group) == "nccl"
        if self.on_device:
            torch.cuda.set_device(device)
        self.dev = torch.device("cuda", device) if self.on_device else torch.device("cpu")
        self.stats = torch.zeros(sw.value, dtype=torch.int64, device=self.dev)
        self.records = 0  # prune records exchanged in the last round (all ranks)

    # the Engine's other calls (set_slots, init_active_sets, fail_nodes, readbacks) are
    # replicated or rank-local and need no exchange
    def __getattr__(self, name):
        return getattr(self.eng, name)

    def _ptr(self, t):
        return C.c_void_p(t.data_ptr())

    def _done(self):
        # the engine reads the buffers on its own stream: torch's collective must be complete
        if self.on_device:
            self.torch.cuda.synchronize()

    def round(self, round_index, record=False):
        """One iteration of gossip_main.rs:449-564 over the partition."""
        torch, tdist, L, h, dev = self.torch, self.tdist, lib(), self.eng.h, int(self.on_device)
        n = C.c_uint32()
        _check(L.gs_part_round(h, round_index, int(bool(record)), C.byref(n)))
        counts = [torch.zeros(1, dtype=torch.int64, device=self.dev) for _ in range(self.world)]
        tdist.all_gather(counts, torch.tensor([n.value], dtype=torch.int64, device=self.dev), group=self.group)
        counts = [int(c.item()) for c in counts]
        m = max(counts)
        if m:
            mine = torch.zeros(2 * m, dtype=torch.int32, device=self.dev)
            if n.value:
                _check(L.gs_part_prunes_out(h, self._ptr(mine), dev))
            parts = [torch.zeros(2 * m, dtype=torch.int32, device=self.dev) for _ in range(self.world)]
            tdist.all_gather(parts, mine, group=self.group)
            recs = torch.cat([p[:2 * c] for p, c in zip(parts, counts)])
            self._done()
            _check(L.gs_part_prunes_in(h, self._ptr(recs), sum(counts), dev))
        self.records = sum(counts)
        self.eng.chance_to_rotate(round_index)
        if record:
            _check(L.gs_part_stats_out(h, self._ptr(self.stats), dev))
            tdist.all_reduce(self.stats, group=self.group)
            self._done()
            _check(L.gs_part_stats_in(h, self._ptr(self.stats), dev))

    def owned(self, arr):
        """The owned slice of a per-node array."""
        return np.asarray(arr)[self.node_lo:self.node_hi]
