"""Node-range partition: two ranks, each owning half of the node
ids, exchange frontier bitsets per BFS level, prune-mask deltas and statistics partials
through torch.distributed (gloo, host buffers) and must reproduce one engine over all
nodes bit for bit: per-round summaries, hop-histogram accumulators, replicated prune
masks, and -- on each rank's own nodes -- hops, message accumulators and caches.

Both ranks run on the one GPU of the box (two engines on device 0); the RCCL path is
the same call sequence with device buffers.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import engine_bind as eb
from partition_case import CASE, run_case

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_partition_two_ranks_matches_one_engine(tmp_path):
    world, port = 2, free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GS_PART_OUT=str(tmp_path / f"rank{r}.npz"))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "partition_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = [p.communicate(timeout=240)[0] for p in procs]
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]

    st = eb.synth.network(CASE["n"])[1]
    one = eb.gs.Engine(st, len(CASE["origins"]), bfs_mode=eb.gs.GS_BFS_LEVEL, seed=CASE["seed"],
                       rotation_probability=CASE["p"])
    want = run_case(one)
    parts = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    assert sum(int(p["hi"][0]) - int(p["lo"][0]) for p in parts) == CASE["n"]
    assert want["summaries"]["prunes"].sum() > 0 and want["summaries"]["stranded"].sum() > 0
    for p in parts:
        np.testing.assert_array_equal(p["summaries"], want["summaries"])
    for k in range(len(CASE["origins"])):
        np.testing.assert_array_equal(sum(p[f"acc{k}"] for p in parts), want[f"acc{k}"], err_msg=f"slot {k}")
        for p in parts:
            lo, hi = int(p["lo"][0]), int(p["hi"][0])
            np.testing.assert_array_equal(p[f"hist{k}"], want[f"hist{k}"])
            np.testing.assert_array_equal(p[f"pruned{k}"], want[f"pruned{k}"], err_msg=f"masks slot {k}")
            np.testing.assert_array_equal(p[f"hops{k}"][lo:hi], want[f"hops{k}"][lo:hi])
            np.testing.assert_array_equal(p[f"cache{k}"][lo:hi], want[f"cache{k}"][lo:hi], err_msg=f"cache {k}")
