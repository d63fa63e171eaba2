"""Sweeps sharded over ranks (gossip-sim_amd/sweep.py).

CPU: world_size 2 over gloo, each rank's sims run by the oracle (test-only
runner): the assembled results on every rank must equal a one-process run,
bit for bit. GPU: the same with the HIP engine, two ranks sharing cuda:0.
"""
import os
import socket
import tempfile

import numpy as np
import pytest

import engine_bind as eb

gs = eb.gs
import gossip_sim_amd.sweep as sweep  # noqa: E402

N, ITERS, WARM = 90, 26, 6
CFG = dict(fanout=6, asz=12, iterations=ITERS, warm_up=WARM, p=0.05, thr=0.15, min_ingress_nodes=2,
           fraction_to_fail=0.1, when_to_fail=4, test_type=5, seed=7)
FRACTIONS = [0.1, 0.2, 0.3, 0.45, 0.05]
RANKS = [1, 1, 2, 1, 3]


class _OracleResult:
    def __init__(self, stats):
        self.stats = stats

    def f64(self, j, name):
        return self.stats[j].f64(name)

    def u64(self, j, name):
        return self.stats[j].u64(name)


def oracle_runner(stakes, *, n_sims, origin_ranks=None, min_ingress=None, thresholds=None, fractions=None,
                  device=None, bfs_mode=None, **kw):
    """Test-only runner with run_simulations' signature, backed by the CPU oracle."""
    import oracle_bind as ob
    pks, _ = eb.synth.network(len(stakes))
    out = []
    for j in range(n_sims):
        out.append(ob.run_simulation(
            pks, stakes, fanout=kw["fanout"], asz=kw["asz"], iterations=kw["iterations"],
            origin_rank=origin_ranks[j] if origin_ranks else 1, p=kw["p"],
            thr=thresholds[j] if thresholds else kw["thr"],
            min_ingress=min_ingress[j] if min_ingress else kw["min_ingress_nodes"],
            fraction_to_fail=fractions[j] if fractions else kw["fraction_to_fail"],
            when_to_fail=kw["when_to_fail"], test_type=kw["test_type"], warm_up=kw["warm_up"], seed=kw["seed"]))
    return _OracleResult(out)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _save(res, path):
    arrs = {}
    for i in range(res.n_sims):
        for kind, name in sweep.NAMES:
            a = res.f64(i, name) if kind == "f" else res.u64(i, name)
            arrs[f"{kind}:{name}:{i}"] = a
    np.savez(path, **arrs)


def _worker(rank, world, port, outdir, use_gpu):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as tdist
    import engine_bind  # noqa: F401  (registers gossip_sim_amd)
    import gossip_sim_amd.sweep as sw
    from test_sweep_dist import oracle_runner, FRACTIONS, RANKS, CFG, N
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    _, st = engine_bind.synth.network(N)
    res = sw.run_sharded(st, n_sims=len(FRACTIONS), origin_ranks=RANKS, fractions=FRACTIONS,
                         runner=None if use_gpu else oracle_runner, device=0 if use_gpu else None, **CFG)
    _save(res, os.path.join(outdir, f"rank{rank}.npz"))
    tdist.barrier()
    tdist.destroy_process_group()


def _run_world(world, use_gpu):
    import torch.multiprocessing as mp
    d = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), d, use_gpu), nprocs=world, join=True)
    return [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]


def _reference(use_gpu):
    _, st = eb.synth.network(N)
    if use_gpu:
        res = gs.run_simulations(st, n_sims=len(FRACTIONS), origin_ranks=RANKS, fractions=FRACTIONS, **CFG)
    else:
        res = oracle_runner(st, n_sims=len(FRACTIONS), origin_ranks=RANKS, fractions=FRACTIONS, **CFG)
    out = {}
    for i in range(len(FRACTIONS)):
        for kind, name in sweep.NAMES:
            out[f"{kind}:{name}:{i}"] = res.f64(i, name) if kind == "f" else res.u64(i, name)
    return out


def _check(got, want):
    assert set(got) == set(want)
    for k in want:
        g, w = got[k], want[k]
        assert g.dtype == w.dtype and g.shape == w.shape, k
        assert g.tobytes() == w.tobytes(), k  # bit-exact, f64 included


def test_shard_partitions_units():
    for n in (0, 1, 5, 13, 16):
        for world in (1, 2, 3, 8):
            owned = sorted(i for r in range(world) for i in sweep.shard(n, r, world))
            assert owned == list(range(n))
            sizes = [len(sweep.shard(n, r, world)) for r in range(world)]
            assert max(sizes) - min(sizes) <= 1


def test_allreduce_single_process_roundtrip():
    rng = np.random.default_rng(3)
    local = {}
    for i in range(3):
        local[i] = {(k, nm): (rng.standard_normal(i + 2) if k == "f" else rng.integers(0, 2**63, i + 1,
                                                                                        dtype=np.uint64))
                    for k, nm in sweep.NAMES}
    local[1][("f", "coverage")] = np.array([-0.0, np.nan, np.inf])
    res = sweep.allreduce_results(local, 3)
    for i in range(3):
        for k, nm in sweep.NAMES:
            a = res.f64(i, nm) if k == "f" else res.u64(i, nm)
            assert a.tobytes() == local[i][(k, nm)].tobytes()


def test_sharded_sweep_gloo_world2_matches_one_process():
    want = _reference(use_gpu=False)
    outs = _run_world(2, use_gpu=False)
    for got in outs:  # every rank holds every sim after the all-reduce
        _check(got, want)


@pytest.mark.gpu
def test_sharded_sweep_gpu_world2_matches_one_process():
    want = _reference(use_gpu=True)
    outs = _run_world(2, use_gpu=True)
    for got in outs:
        _check(got, want)


def _pbfs_worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as tdist
    import engine_bind
    g = engine_bind.gs
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    _, st = engine_bind.synth.network(20_000)
    eng = g.Engine(st, 2, rotation_probability=0.01, seed=5, device=0, bfs_mode=g.GS_BFS_MULTI)
    eng.set_slots([1, 2])
    eng.init_active_sets()
    tdist.barrier()  # both processes hold an engine on the card
    pers = bool(eng.info()["bfs_persistent"])
    for r in range(6):
        eng.round(r, record=True)
    sm = eng.summaries()
    eng.close()
    np.savez(os.path.join(outdir, f"pb{rank}.npz"), pers=np.array([pers]), summ=sm.view(np.uint8))
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.gpu
def test_two_processes_on_one_device_one_persistent_bfs():
    """Two processes (gloo ranks) with one multi-BFS engine each on cuda:0: the persistent BFS
    needs all its workgroups co-resident, so at most one process on a card may run it (a
    lock named after the device's PCI bus id, gs_bfs_pers.hip); the other runs the launched
    level loop. Exactly one of them reports the persistent path, and both runs' summaries are
    equal (the two paths are bit-identical)."""
    import torch.multiprocessing as mp
    d = tempfile.mkdtemp()
    mp.spawn(_pbfs_worker, args=(2, _free_port(), d), nprocs=2, join=True)
    outs = [np.load(os.path.join(d, f"pb{r}.npz")) for r in range(2)]
    assert sum(bool(o["pers"][0]) for o in outs) == 1, [bool(o["pers"][0]) for o in outs]
    assert outs[0]["summ"].tobytes() == outs[1]["summ"].tobytes()


# ---- origin sharding of ONE network (bench.py --shard-origins, strong scaling) ----
SH_N, SH_ORIGINS, SH_ROUNDS = 120, 7, 24


def _origin_rows(origins):
    """Per round, per origin: (pushes, nodes reached) of the oracle's Cluster run over the
    shared seed -- 8 bytes per origin, the unit that bench.py's shard check reassembles."""
    import oracle_bind as ob
    pks, st = eb.synth.network(SH_N)
    rows = np.zeros((SH_ROUNDS, len(origins), 2), dtype=np.uint32)
    for j, o in enumerate(origins):
        sim = ob.Sim(ob.PHILOX, 7, pks, st, 6)
        sim.init_philox(12)
        for r in range(SH_ROUNDS):
            rows[r, j, 0] = sim.round(o, 0.15, 2, 12, 0.05, r)
            rows[r, j, 1] = int((sim.distances() != np.iinfo(np.uint64).max).sum())
    return rows.view(np.uint8).reshape(SH_ROUNDS, -1)


def _shard_worker(rank, world, port, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as tdist
    import engine_bind  # noqa: F401
    import gossip_sim_amd.sweep as sw
    from test_sweep_dist import SH_ORIGINS, _origin_rows
    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = sw.shard_range(SH_ORIGINS, rank, world)
    local = _origin_rows(list(range(lo, hi)))
    full = sw.gather_rows((torch, tdist), local, SH_ORIGINS, world, row_bytes=8)
    np.save(os.path.join(outdir, f"rank{rank}.npy"), full)
    tdist.barrier()
    tdist.destroy_process_group()


def test_origin_shard_reassembly_gloo_world2():
    """--shard-origins: each rank runs a contiguous share of the origins of one network
    (shard_range; the same seed, so the same active-set trajectory), and gather_rows
    reassembles every origin's per-round rows on every rank, bit-identical to one
    process running all origins."""
    import torch.multiprocessing as mp
    for n in (0, 1, 7, 3000):
        for world in (1, 2, 3, 8):
            spans = [sweep.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    want = _origin_rows(list(range(SH_ORIGINS)))
    d = tempfile.mkdtemp()
    mp.spawn(_shard_worker, args=(2, _free_port(), d), nprocs=2, join=True)
    for r in range(2):
        got = np.load(os.path.join(d, f"rank{r}.npy"))
        assert got.tobytes() == want.tobytes()
