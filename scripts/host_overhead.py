#!/usr/bin/env python3
"""Host enqueue time vs wall time of gs_round on the C2 workload (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

gs = bench.load_pkg()
import gossip_sim_amd.synth as synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
S = int(sys.argv[2]) if len(sys.argv) > 2 else n
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 0
st = synth.power_law_stakes(n) if n > 100000 else synth.network(n)[1]
eng = gs.Engine(st, S, rotation_probability=0.01, seed=0x5EED0003, profile=False, bfs_mode=mode)
eng.set_slots([s % n for s in range(S)], 2, 0.15)
eng.init_active_sets()
for r in range(20):
    eng.round(r, record=False)
eng.sync()
for rep in range(3):
    t0 = time.perf_counter()
    ts = []
    K = 60 if n <= 100000 else 10
    for r in range(20 + K * rep, 20 + K * (rep + 1)):
        eng.round(r, record=True)
        ts.append(time.perf_counter())
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    d = [(b - a) * 1e6 for a, b in zip([t0] + ts[:-1], ts)]
    print(f"rep {rep}: enqueue {1e6 * (t1 - t0) / K:.1f} us/round (max {max(d):.0f}), wall {1e6 * (t2 - t0) / K:.1f} us/round")
