"""Node-range partition: two ranks, each owning a contiguous half
of the node ids (whole 1,024-id bins), keep per-(slot, node) state for their own nodes
only, run the whole multi-source BFS over replicated rows, exchange prune records and
statistics partials through torch.distributed, and must reproduce one engine over all
nodes bit for bit: per-round summaries, hop-histogram accumulators, replicated prune
masks, and -- on each rank's own nodes -- hops, message accumulators and caches. Each
rank's device memory is its half of the per-pair state plus the replicated tables.

Both ranks run on the one GPU of the box (two engines on device 0): gloo exchanges host
buffers; nccl (RCCL) exchanges device buffers when RCCL accepts two ranks on one GPU
(otherwise the case is skipped with that reason)."""
import os
import pickle
import socket
import subprocess
import sys

import numpy as np
import pytest

import engine_bind as eb
from partition_case import CASES, cache_rows, run_case, stakes_of

HERE = os.path.dirname(os.path.abspath(__file__))
RCCL_REFUSED = 77


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(tmp_path, case, backend, world=2, exchange="auto", extra_env=None, bfs="replicated"):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GS_PART_OUT=str(tmp_path / f"rank{r}.npz"), GS_PART_CASE=case,
                   GS_PART_BACKEND=backend, GS_PART_EXCHANGE=exchange, GS_PART_BFS=bfs, **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "partition_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    try:
        logs = [p.communicate(timeout=400)[0] for p in procs]
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        for p in procs:
            p.communicate()
        raise
    if backend == "nccl" and any(p.returncode == RCCL_REFUSED for p in procs):
        pytest.skip("RCCL refused two ranks on the box's one GPU: " + " | ".join(l.strip()[-300:] for l in logs))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
        print(log.strip()[-2000:])
    parts = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    caches = []
    for r in range(world):
        with open(tmp_path / f"rank{r}.npz.caches", "rb") as f:
            caches.append(pickle.load(f))
    return parts, caches


def test_partition_ranges_refuse_empty_ranks():
    import gossip_sim_amd.partition as gp
    assert gp.partition_ranges(3000, 2) == [(0, 2048), (2048, 3000)]
    assert gp.partition_ranges(10_000_000, 8)[-1][1] == 10_000_000
    with pytest.raises(ValueError, match="without nodes"):
        gp.partition_ranges(3000, 4)  # ranges of 1,024: the fourth rank would start at 3,072


def test_partition_ranges_frontier_units():
    """A frontier-exchange partition owns whole coarse bins of the multi BFS (mv_geometry's
    ~256 bins of 2^6 .. 2^13 nodes), at least 1,024 ids."""
    import gossip_sim_amd.partition as gp
    assert gp.coarse_bin_nodes(3000) == 64 and gp.coarse_bin_nodes(1_000_000) == 4096
    assert gp.coarse_bin_nodes(10_000_000) == 8192
    assert gp.partition_ranges(3000, 2, frontier=True) == [(0, 2048), (2048, 3000)]
    assert gp.partition_ranges(1_000_000, 2, frontier=True) == [(0, 503808), (503808, 1_000_000)]
    assert all(lo % 8192 == 0 for lo, _ in gp.partition_ranges(10_000_000, 8, frontier=True))


@pytest.mark.gpu
@pytest.mark.parametrize("case,backend,exchange,bfs", [
    ("small", "gloo", "auto", "replicated"), ("small", "gloo", "dense", "replicated"),
    ("small", "nccl", "auto", "replicated"), ("large", "gloo", "auto", "replicated"),
    ("large", "gloo", "records", "replicated"),
    ("small", "gloo", "auto", "frontier"), ("large", "gloo", "auto", "frontier"),
    ("small", "gloo", "auto", "frontier-redo")])
def test_partition_two_ranks_matches_one_engine(tmp_path, case, backend, exchange, bfs):
    """(exchange: the prune exchange -- auto = records outside prune waves, dense in them;
    records / dense forced. bfs: replicated = every rank runs the whole BFS; frontier = each
    rank expands its own frontier and the level's push records go to their owners -- the
    first round with a size exchange per level, the later ones without a host wait per level
    (fixed message slots from the last round's sizes); frontier-redo: slots forced too small,
    so a round's message overflows its slot and the group is redone with exact sizes.)"""
    extra = {"GS_PART_RECORD_CAP": str(1 << 25)} if exchange == "records" else {}
    if bfs == "frontier-redo":
        extra["GS_XBFS_SLOT_WORDS"] = "40"
        bfs = "frontier"
        redo = True
    else:
        redo = False
    parts, caches = run_ranks(tmp_path, case, backend, exchange=exchange, extra_env=extra, bfs=bfs)
    if bfs == "frontier":
        assert all(int(p["levels"][0]) >= 3 and int(p["levels"][1]) > 0 for p in parts), [p["levels"] for p in parts]
        asy = [tuple(int(x) for x in p["async"]) for p in parts]
        assert all(a > 0 for a, _ in asy), asy  # rounds after the first ran the asynchronous level loop
        assert all((r > 0) == redo for _, r in asy), asy
    modes = set(str(m) for m in parts[0]["xmodes"] if str(m))
    if exchange != "auto":
        assert modes == {exchange}, modes
    elif case == "large":
        assert "dense" in modes, modes  # the prune wave outgrows the record buffer
    c = CASES[case]
    st = stakes_of(case, eb.synth)
    S = len(c["mi"])
    one = eb.gs.Engine(st, S, bfs_mode=eb.gs.GS_BFS_LEVEL, seed=c["seed"], rotation_probability=c["p"])
    want = run_case(one, case, st)
    want_caches = {k: cache_rows(one, case, k) for k in range(S)}
    one.close()
    assert sum(int(p["hi"][0]) - int(p["lo"][0]) for p in parts) == c["n"]
    assert want["summaries"]["prunes"].sum() > 0 and want["summaries"]["stranded"].sum() > 0
    for p in parts:
        np.testing.assert_array_equal(p["summaries"], want["summaries"])
    for k in range(S):
        np.testing.assert_array_equal(sum(p[f"acc{k}"] for p in parts), want[f"acc{k}"], err_msg=f"slot {k}")
        for r, p in enumerate(parts):
            lo, hi = int(p["lo"][0]), int(p["hi"][0])
            np.testing.assert_array_equal(p[f"hist{k}"], want[f"hist{k}"])
            np.testing.assert_array_equal(p[f"pruned{k}"], want[f"pruned{k}"], err_msg=f"masks slot {k}")
            np.testing.assert_array_equal(p[f"hops{k}"][lo:hi], want[f"hops{k}"][lo:hi])
            if f"cache{k}" in want:
                np.testing.assert_array_equal(p[f"cache{k}"][lo:hi], want[f"cache{k}"][lo:hi], err_msg=f"cache {k}")
            for v, row in caches[r][k].items():
                assert row == want_caches[k][v], f"cache slot {k} node {v}"
    if case == "large" and exchange == "auto" and bfs == "replicated":
        # device memory per rank: its share of the per-(slot, node) state + the replicated tables
        # (the forced-records run enlarges the record buffer by GS_PART_RECORD_CAP: not compared)
        # (the reference engine without the persistent BFS's level buffers: a partition rank
        # runs the launched level loop and allocates none)
        os.environ["GS_MV_PBFS"] = "0"
        try:
            full = eb.gs.Engine(st, S, bfs_mode=eb.gs.GS_BFS_MULTI, seed=c["seed"], rotation_probability=c["p"])
        finally:
            os.environ.pop("GS_MV_PBFS", None)
        fi = full.info()
        full.close()
        for p in parts:
            dev, pair, other = (int(x) for x in p["bytes"])
            share = (int(p["hi"][0]) - int(p["lo"][0])) / c["n"]
            assert abs(pair - share * fi["pair_bytes"]) <= 0.01 * fi["pair_bytes"] + (64 << 20), (pair, fi)
            assert abs(other - fi["other_bytes"]) <= 0.02 * fi["other_bytes"], (other, fi)
            assert dev < 0.8 * fi["device_bytes"], (dev, fi)


@pytest.mark.gpu
@pytest.mark.parametrize("bfs", ["replicated", "frontier"])
def test_partition_c5_as_configured(tmp_path, bfs):
    """BASELINE C5 as configured on the box's one GPU: 10M nodes, origin ranks 1..16 as 16
    slots, node-range partitioned over two gloo ranks (two engines on device 0), 22 rounds
    through the first prune wave (records exchanged in ordinary rounds, dense words in the
    wave). Equals one unpartitioned engine (the level-synchronous BFS) bit for bit: every
    per-round summary and hop histogram, per-rank digests of owned hops and accumulators,
    the replicated prune state, sampled caches; and the size-independent BFS properties
    hold on the unpartitioned run. bfs="frontier": each rank expands only its own frontier and
    the levels' push records go to their owners (the north star's frontier exchange)."""
    from test_gpu_parity import _invariants
    parts, caches = run_ranks(tmp_path, "c5", "gloo", bfs=bfs)
    c = CASES["c5"]
    n, S = c["n"], len(c["mi"])
    ranges = [(int(p["lo"][0]), int(p["hi"][0])) for p in parts]
    assert ranges[0][0] == 0 and ranges[0][1] == ranges[1][0] and ranges[1][1] == n
    modes = [str(m) for m in parts[0]["xmodes"]]
    assert "dense" in modes and "records" in modes, modes  # the prune wave went dense
    st = stakes_of("c5", eb.synth)
    one = eb.gs.Engine(st, S, bfs_mode=eb.gs.GS_BFS_LEVEL, seed=c["seed"], rotation_probability=c["p"])
    want = run_case(one, "c5", st, ranges=ranges)
    want_caches = {k: cache_rows(one, "c5", k) for k in range(S)}
    summ = want["summaries"]
    assert summ["prunes"].sum() > 0 and (summ["visited"] > 0.9 * n).all()
    for k in (0, S - 1):
        _invariants(one, k, n, summ[-1, k])
    one.close()
    for r, p in enumerate(parts):
        np.testing.assert_array_equal(p["summaries"], summ)
        for k in range(S):
            np.testing.assert_array_equal(p[f"hist{k}"], want[f"hist{k}"])
            assert p[f"pruned{k}"][0] == want[f"pruned{k}"][0], f"prune state slot {k}"
            assert list(p[f"dig{k}"][0]) == list(want[f"dig{k}"][r]), f"rank {r} slot {k}"
            for v, row in caches[r][k].items():
                assert row == want_caches[k][v], f"cache slot {k} node {v}"
