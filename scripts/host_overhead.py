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
pks, st = synth.network(n)
eng = gs.Engine(st, n, rotation_probability=0.01, seed=0x5EED0003, profile=False)
eng.set_slots([s % n for s in range(n)], 2, 0.15)
eng.init_active_sets()
for r in range(20):
    eng.round(r, record=False)
eng.sync()
for rep in range(3):
    t0 = time.perf_counter()
    ts = []
    for r in range(20 + 60 * rep, 80 + 60 * rep):
        eng.round(r, record=True)
        ts.append(time.perf_counter())
    t1 = time.perf_counter()
    eng.sync()
    t2 = time.perf_counter()
    d = [(b - a) * 1e6 for a, b in zip([t0] + ts[:-1], ts)]
    print(f"rep {rep}: enqueue {1e6 * (t1 - t0) / 60:.1f} us/round (max {max(d):.0f}), wall {1e6 * (t2 - t0) / 60:.1f} us/round")
