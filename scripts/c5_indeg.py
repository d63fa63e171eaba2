#!/usr/bin/env python3
"""Round 4 diagnostic: the per-(slot, node) in-degree distribution of the C5 leg's
configuration (10M-node power-law network, origin ranks 1..16 as slots), from one
recorded round's ingress accumulators, and the share of consume's lane / wave / serial
paths (in-degree <= 16 / <= 64 / more)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

gs = bench.load_pkg()
from importlib import import_module  # noqa: E402
synth = import_module(gs.__name__ + ".synth")

n = int(os.environ.get("N", 10_000_000))
S = 16
st = synth.power_law_stakes(n)
order = np.lexsort((np.arange(n), -st.astype(np.float64)))
eng = gs.Engine(st, S, seed=0, rotation_probability=0.013333, device=0, bfs_mode=gs.GS_BFS_MULTI)
eng.set_slots([int(x) for x in order[:S]], 2, 0.15)
eng.init_active_sets()
print("init done", flush=True)
R = int(os.environ.get("ROUNDS", 6))
for r in range(R):
    eng.round(r, record=(r == R - 1))
    eng.sync()
    print("round", r, flush=True)
out = {"nodes": n, "slots": S, "round": R - 1}
tot = {"pairs": 0, "lane": 0, "wave": 0, "serial": 0, "rec_lane": 0, "rec_wave": 0, "rec_serial": 0}
for k in range(S):
    _, ing, _ = eng.counters(k)
    print("slot", k, flush=True)
    c = ing.astype(np.int64)
    tot["pairs"] += n
    lane, wave, ser = c <= 16, (c > 16) & (c <= 64), c > 64
    tot["lane"] += int(lane.sum()); tot["wave"] += int(wave.sum()); tot["serial"] += int(ser.sum())
    tot["rec_lane"] += int(c[lane].sum()); tot["rec_wave"] += int(c[wave].sum()); tot["rec_serial"] += int(c[ser].sum())
    if k in (0, 15):
        h = np.bincount(np.minimum(c, 200))
        out[f"slot{k}_hist_0_200"] = h.tolist()
        out[f"slot{k}_max"] = int(c.max())
        # waves of 64 consecutive nodes: mean of the wave max over the wave mean
        w = c[: (n // 64) * 64].reshape(-1, 64)
        out[f"slot{k}_wave_max_mean"] = float(w.max(axis=1).mean())
        out[f"slot{k}_wave_mean"] = float(w.mean())
        out[f"slot{k}_heavy_lanes_per_wave_mean"] = float((w > 16).sum(axis=1).mean())
out["totals"] = tot
eng.close()
with open(os.environ.get("OUT", "/dev/stdout"), "w") as f:
    f.write(json.dumps(out))
