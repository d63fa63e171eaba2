"""Sweeps sharded over GPUs: one process per GPU, sims dealt round-robin.

SURVEY.md 8(e): the simulations of a sweep (gossip_main.rs:774-951: origin-rank,
active-set-size, min-ingress, push-fanout, prune-threshold, fail-nodes,
rotation-probability test types) are independent units. Every rank runs its
share of them as slots of ONE engine on its own GPU (run_simulations); the
Philox contract makes a sim's result independent of which rank ran it and of
which other sims shared its engine. There is no data-path collective: after the
sims finish, each rank packs its sims' result arrays (integer histograms,
counters and the f64 statistics, the latter as their IEEE bit patterns) into one
zero-padded int64 buffer and a single all-reduce(SUM) assembles every sim on
every rank. Adding zeros to bit patterns is exact, so the assembled results are
bit-identical to a one-GPU run. With the "nccl" backend (RCCL over xGMI on ROCm)
the buffer lives on the rank's GPU; with "gloo" it stays on the host.

Test types whose parameter changes the engine itself (active-set-size,
push-fanout, rotation-probability) give each value its own engine; `run_sweep`
takes the values and deals them out the same way.
"""
import numpy as np

from . import run_simulations

F64_NAMES = ["coverage", "rmr", "branching", "hop_mean", "hop_median", "coverage_stats", "rmr_stats",
             "branching_stats", "aggregate_hops", "ldh", "stranded", "stranded_round_mean",
             "stranded_round_median"]
U64_NAMES = ["origin", "hop_max", "hop_min", "aggregate_hops", "ldh", "stranded", "stranded_times",
             "stranded_round_count", "stranded_round_max", "stranded_round_min", "hops_hist", "stranded_hist",
             "egress_hist", "ingress_hist", "prune_hist", "egress_cpb", "validator_hist", "hist_errors",
             "failed_count"]
NAMES = [("f", n) for n in F64_NAMES] + [("u", n) for n in U64_NAMES]


def shard(n_units, rank, world):
    """Units owned by `rank`: round-robin, so a sweep of k*world units is balanced."""
    return list(range(rank, n_units, world))


def shard_range(n_units, rank, world):
    """Contiguous units [lo, hi) owned by `rank` (origin sharding of one network)."""
    return n_units * rank // world, n_units * (rank + 1) // world


def gather_rows(dist, local, n_units, world, *, row_bytes, group=None):
    """local: [rows, n_local * row_bytes] uint8 of this rank's contiguous units
    (shard_range). Returns [rows, n_units * row_bytes] with every rank's columns,
    assembled by one all-reduce(SUM) of a zero-padded int64 buffer (exact: each byte
    has one owner). On the "nccl" backend (RCCL over xGMI) the buffer lives on the
    rank's current GPU."""
    torch, tdist = dist
    rank = tdist.get_rank(group)
    lo, hi = shard_range(n_units, rank, world)
    rows = local.shape[0]
    full = np.zeros((rows, n_units * row_bytes), dtype=np.uint8)
    full[:, lo * row_bytes:hi * row_bytes] = local
    assert (n_units * row_bytes) % 8 == 0
    t = torch.from_numpy(full.view(np.int64).copy())
    if tdist.get_backend(group) == "nccl":
        t = t.to(f"cuda:{torch.cuda.current_device()}")
    tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=group)
    return t.cpu().numpy().view(np.uint8).reshape(rows, -1)


def _dist_info(group):
    try:
        import torch.distributed as tdist
    except ImportError:
        return None, 0, 1
    if not tdist.is_available() or not tdist.is_initialized():
        return None, 0, 1
    return tdist, tdist.get_rank(group), tdist.get_world_size(group)


def _as_bits(kind, a):
    a = np.ascontiguousarray(a, dtype=np.float64 if kind == "f" else np.uint64)
    return a.view(np.int64)


def _from_bits(kind, a):
    return np.ascontiguousarray(a, dtype=np.int64).view(np.float64 if kind == "f" else np.uint64).copy()


class SweepResult:
    """Per-sim result arrays by name, the same names as SimResult.f64/u64."""

    def __init__(self, per_sim):
        self.per_sim = per_sim  # list of {(kind, name): ndarray}
        self.n_sims = len(per_sim)

    def f64(self, sim, name):
        return self.per_sim[sim][("f", name)]

    def u64(self, sim, name):
        return self.per_sim[sim][("u", name)]


def allreduce_results(local, n_sims, *, group=None, device=None):
    """local: {sim index: {(kind, name): ndarray}} for this rank's sims. Returns a
    SweepResult holding every sim, assembled with one all-reduce of lengths and
    one all-reduce of the packed int64 bit patterns."""
    tdist, rank, world = _dist_info(group)
    nn = len(NAMES)
    lens = np.zeros((n_sims, nn), dtype=np.int64)
    for i, arrs in local.items():
        for j, key in enumerate(NAMES):
            lens[i, j] = len(arrs[key])
    if tdist is not None:  # (a one-rank group still runs the collective: RCCL is exercised)
        import torch
        t = torch.from_numpy(lens).to(device) if device is not None else torch.from_numpy(lens)
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=group)
        lens = t.cpu().numpy()
    offs = np.zeros(n_sims * nn + 1, dtype=np.int64)
    np.cumsum(lens.reshape(-1), out=offs[1:])
    buf = np.zeros(int(offs[-1]), dtype=np.int64)
    for i, arrs in local.items():
        for j, (kind, name) in enumerate(NAMES):
            k = i * nn + j
            buf[offs[k]:offs[k + 1]] = _as_bits(kind, arrs[(kind, name)])
    if tdist is not None:  # (a one-rank group still runs the collective: RCCL is exercised)
        import torch
        t = torch.from_numpy(buf).to(device) if device is not None else torch.from_numpy(buf)
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM, group=group)
        buf = t.cpu().numpy()
    per_sim = []
    for i in range(n_sims):
        d = {}
        for j, (kind, name) in enumerate(NAMES):
            k = i * nn + j
            d[(kind, name)] = _from_bits(kind, buf[offs[k]:offs[k + 1]])
        per_sim.append(d)
    return SweepResult(per_sim)


def run_sharded(stakes, *, n_sims, origin_ranks=None, min_ingress=None, thresholds=None, fractions=None,
                group=None, device=None, comm_device=None, runner=None, **cfg):
    """run_simulations for n_sims sims dealt over the ranks of `group`.

    device: the HIP device of this rank's engine (default: LOCAL_RANK via cfg or 0).
    comm_device: where the all-reduce buffer lives ("cuda:<i>" for RCCL, None for gloo).
    runner: the per-rank sim runner (default: the HIP engine's run_simulations).
    """
    tdist, rank, world = _dist_info(group)
    runner = runner or run_simulations
    mine = shard(n_sims, rank, world)

    def sub(x):
        return None if x is None else [x[i] for i in mine]

    local = {}
    if mine:
        kw = dict(cfg)
        if device is not None:
            kw["device"] = device
        res = runner(stakes, n_sims=len(mine), origin_ranks=sub(origin_ranks), min_ingress=sub(min_ingress),
                     thresholds=sub(thresholds), fractions=sub(fractions), **kw)
        for j, i in enumerate(mine):
            local[i] = {(kind, name): (res.f64(j, name) if kind == "f" else res.u64(j, name))
                        for kind, name in NAMES}
    return allreduce_results(local, n_sims, group=group, device=comm_device)


def run_sweep(stakes, values, make_cfg, *, group=None, device=None, comm_device=None, runner=None):
    """Engine-changing test types (active-set-size, push-fanout, rotation-probability):
    one single-sim engine per value, values dealt round-robin over the ranks.
    make_cfg(value) -> kwargs of run_simulations for that value."""
    tdist, rank, world = _dist_info(group)
    runner = runner or run_simulations
    local = {}
    for i in shard(len(values), rank, world):
        kw = dict(make_cfg(values[i]))
        if device is not None:
            kw["device"] = device
        res = runner(stakes, n_sims=1, **kw)
        local[i] = {(kind, name): (res.f64(0, name) if kind == "f" else res.u64(0, name)) for kind, name in NAMES}
    return allreduce_results(local, len(values), group=group, device=comm_device)
