"""RCCL executed: every torch.distributed exchange of the multi-GPU paths
run over the "nccl" backend (RCCL on ROCm) on the box's one GPU, as a world-size-1 process
group, and compared bit for bit with the same run over gloo and with one plain engine.

RCCL refuses two ranks on one GPU (tests/test_partition.py skips its nccl case for that),
but a one-rank communicator runs every collective for real on device buffers: the node
partition's prune-record all-gather and dense-word all-reduce read and written by
gs_part_prunes_out/_in and gs_part_prunes_dense_out/_in with dev = 1, the frontier-exchange
BFS's two all-to-alls per level (gs_part_xbfs_send / _apply with dev = 1), its statistics
all-reduce (gs_part_stats_out/_in), the sweep assembly (sweep.allreduce_results on
cuda:0) and the origin-shard reassembly (sweep.gather_rows). The reference's finalize
step these replace: gossip_main.rs:567-646."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import engine_bind as eb
from partition_case import CASES, run_case, stakes_of

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, backend):
    out = tmp_path / f"{backend}.npz"
    env = dict(os.environ, GS_RCCL_BACKEND=backend, GS_RCCL_PORT=str(_port()), GS_RCCL_OUT=str(out),
               MASTER_ADDR="127.0.0.1", GS_PART_RECORD_CAP=str(1 << 22))  # (records forced through the prune wave)
    p = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_worker.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    return dict(np.load(out))


@pytest.mark.gpu
def test_rccl_world1_exchanges_match_gloo_and_one_engine(tmp_path):
    nccl = _run(tmp_path, "nccl")
    gloo = _run(tmp_path, "gloo")
    assert str(nccl["backend"][0]) == "nccl" and str(gloo["backend"][0]) == "gloo"
    assert set(nccl) == set(gloo)
    for k in nccl:
        if k != "backend":
            assert nccl[k].tobytes() == gloo[k].tobytes(), k
    # the frontier exchange ran its levels without host waits after the first round (slots from
    # the last round's sizes), the collective enqueued on the engine's stream
    assert int(nccl["part_frontier_async"][0]) > 0, nccl["part_frontier_async"]
    for ex in ("records", "dense"):  # each exchange form really ran, in the prune wave too
        modes = set(str(m) for m in nccl[f"part_{ex}_modes"] if str(m))
        assert modes == {ex}, (ex, modes)
    c = CASES["small"]
    st = stakes_of("small", eb.synth)
    one = eb.gs.Engine(st, len(c["mi"]), bfs_mode=eb.gs.GS_BFS_LEVEL, seed=c["seed"], rotation_probability=c["p"])
    want = run_case(one, "small", st)
    one.close()
    assert want["summaries"]["prunes"].sum() > 0
    for ex in ("records", "dense", "frontier"):
        for k, v in want.items():
            got = nccl[f"part_{ex}_{k}"]
            assert got.tobytes() == np.asarray(v).tobytes(), (ex, k)
    _, st90 = eb.synth.network(90)
    res = eb.gs.run_simulations(st90, n_sims=3, origin_ranks=[1, 2, 1], fractions=[0.1, 0.0, 0.3], fanout=6, asz=12,
                                iterations=24, warm_up=4, p=0.05, thr=0.15, min_ingress_nodes=2, fraction_to_fail=0.1,
                                when_to_fail=3, test_type=5, seed=7)
    import gossip_sim_amd.sweep as sw
    for i in range(3):
        for kind, name in sw.NAMES:
            w = res.f64(i, name) if kind == "f" else res.u64(i, name)
            assert nccl[f"sweep_{kind}:{name}:{i}"].tobytes() == np.asarray(w).tobytes(), (i, name)
    np.testing.assert_array_equal(nccl["rows"], np.arange(240, dtype=np.uint8).reshape(5, 48))
