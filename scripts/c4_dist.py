#!/usr/bin/env python3
"""C4 diagnostics: distribution of received-cache lengths and per-slot in-degrees after a
few rounds, and their per-wave (64 consecutive nodes) maxima -- what the consume's lane
path iterates over."""
import importlib.util, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
gs = bench.load_pkg()
import gossip_sim_amd.synth as synth
st = synth.power_law_stakes(1_000_000)
org = int(np.argmax(st))
fr = [0.1, 0.2, 0.3, 0.4, 0.5] + [0.0] * 8
thr = [0.15] * 5 + [round(0.05 * (j + 1), 2) for j in range(8)]
eng = gs.Engine(st, 13, rotation_probability=0.013333, seed=0x5EED0003, device=0)
eng.set_slots([org] * 13, 2, thr)
eng.init_active_sets()
eng.fail_nodes(fr)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 15):
    eng.round(r)
eng.sync()
for slot in (0, 7):
    up, ln, _, _ = eng.caches(slot)
    off, _, _ = eng.inbound(slot)
    deg = np.diff(off.astype(np.int64))
    w = (len(ln) // 64) * 64
    lw = ln[:w].reshape(-1, 64).max(axis=1)
    dw = deg[:w].reshape(-1, 64).max(axis=1)
    q = lambda a: np.percentile(a, [50, 90, 99, 100]).tolist()
    print(f"slot {slot}: len mean {ln.mean():.1f} pct50/90/99/max {q(ln)}; wave-max len mean {lw.mean():.1f}; "
          f"in-degree mean {deg.mean():.2f} pct {q(deg)}; wave-max deg mean {dw.mean():.1f}; "
          f"len>32 {np.mean(ln > 32):.3f} len>16 {np.mean(ln > 16):.3f} deg>16 {np.mean(deg > 16):.4f}")
eng.close()
