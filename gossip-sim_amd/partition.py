"""Node-range partition of a simulation batch over ranks.

One process per GPU. Every rank builds the same engine (stakes, slots, seed) and
attaches to the partition (gs_part_attach): it owns the node ids
[rank*C, min((rank+1)*C, n)). A round is the call sequence of include/gossip_hip.h
gs_part_*; this class runs it and does the exchanges with torch.distributed:

  per BFS level   SUM of the new-node counts (stop at 0), all-gather of the
                  frontier bitsets (u32 words, rank-major);
  after consume   SUM of the prune counts; when > 0, SUM of the prune-mask deltas
                  (= their OR: a bit belongs to one pruner, owned by one rank);
  recorded round  SUM of the statistics partials (u64 words).

With the "nccl" backend (RCCL over xGMI) the exchange buffers are torch tensors on
the rank's GPU and the engine copies device to device; with "gloo" they are host
tensors. Results are bit-identical to one engine over all nodes (tests/test_partition.py).
"""
import ctypes as C

import numpy as np

from . import GS_BFS_LEVEL, Engine, _check, lib


class PartitionedEngine:
    def __init__(self, stakes, n_slots, *, group=None, device=0, **engine_kw):
        import torch
        import torch.distributed as tdist
        self.torch, self.tdist, self.group = torch, tdist, group
        self.rank = tdist.get_rank(group)
        self.world = tdist.get_world_size(group)
        engine_kw["bfs_mode"] = GS_BFS_LEVEL
        self.eng = Engine(stakes, n_slots, device=device, **engine_kw)
        L = lib()
        _check(L.gs_part_attach(self.eng.h, self.rank, self.world))
        fw, dw, sw = C.c_size_t(), C.c_size_t(), C.c_size_t()
        lo, hi = C.c_uint32(), C.c_uint32()
        _check(L.gs_part_sizes(self.eng.h, C.byref(fw), C.byref(dw), C.byref(sw), C.byref(lo), C.byref(hi)))
        self.node_lo, self.node_hi = lo.value, hi.value
        self.on_device = tdist.get_backend(group) == "nccl"
        if self.on_device:
            torch.cuda.set_device(device)
        dev = torch.device("cuda", device) if self.on_device else torch.device("cpu")
        self.fr_own = torch.zeros(fw.value, dtype=torch.int32, device=dev)
        self.fr_all = [torch.zeros(fw.value, dtype=torch.int32, device=dev) for _ in range(self.world)]
        self.fr_cat = torch.zeros(fw.value * self.world, dtype=torch.int32, device=dev)
        self.delta = torch.zeros(dw.value, dtype=torch.int32, device=dev)
        self.stats = torch.zeros(sw.value, dtype=torch.int64, device=dev)
        self.levels = 0

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

    def _sum(self, x):
        t = self.torch.tensor([int(x)], dtype=self.torch.int64, device=self.fr_own.device)
        self.tdist.all_reduce(t, group=self.group)
        return int(t.item())

    def round(self, round_index, record=False):
        """One iteration of gossip_main.rs:449-564 over the partition."""
        L, h, dev = lib(), self.eng.h, int(self.on_device)
        _check(L.gs_part_begin(h))
        new = C.c_uint32()
        for d in range(254):
            _check(L.gs_part_level(h, d, C.byref(new)))
            if self._sum(new.value) == 0:
                self.levels = d + 1
                break
            _check(L.gs_part_frontier_out(h, self._ptr(self.fr_own), dev))
            self.tdist.all_gather(self.fr_all, self.fr_own, group=self.group)
            self.torch.cat(self.fr_all, out=self.fr_cat)
            self._done()
            _check(L.gs_part_frontier_in(h, self._ptr(self.fr_cat), dev))
        pr = C.c_uint32()
        _check(L.gs_part_consume(h, C.byref(pr)))
        if self._sum(pr.value) > 0:
            _check(L.gs_part_delta_out(h, self._ptr(self.delta), dev))
            self.tdist.all_reduce(self.delta, group=self.group)
            self._done()
            _check(L.gs_part_delta_in(h, self._ptr(self.delta), dev))
        self.eng.chance_to_rotate(round_index)
        if record:
            _check(L.gs_part_stats_out(h, self._ptr(self.stats), dev))
            self.tdist.all_reduce(self.stats, group=self.group)
            self._done()
            _check(L.gs_part_stats_in(h, self._ptr(self.stats), dev))

    def owned(self, arr):
        """The owned slice of a per-node array."""
        return np.asarray(arr)[self.node_lo:self.node_hi]
