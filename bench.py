#!/usr/bin/env python3
"""bench.py -- push-propagation edges/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], "C2"): a ~3,000-node synthetic power-law
stake network, ALL 3,000 origins batched as independent sims (slots) of one
engine, rotation probability 0.01, push fanout 6, active-set size 12. A step is
one full gossip iteration for every slot (gossip_main.rs:449-564: run_gossip ->
consume -> send_prunes -> prune_connections -> chance_to_rotate -> the
measured-round statistics), with all inputs resident in HBM.

value = pushes to non-failed peers over all slots and ranks / wall time of the
K timed steps (max over ranks). Multi-GPU: one process per GPU; each rank runs
its own 3,000 origin-sims with seed + rank (independent sims, no data-path
collective) => "scaling": "weak". torch.distributed (gloo) is used only for the
barrier and the max/sum of the timing scalars.

roofline: the propagation kernel (BFS) with SURVEY.md 8(d) algorithmic bytes
B_prop = V*(4*ASZ + 5) + 8*E per origin-round, divided by that kernel's summed
duration measured with hipEvents on the engine stream over the timed steps.
cpu_baseline: the oracle (reference-structure C++ restatement: maps keyed by
32-byte pubkeys, one origin at a time, single core) timed on this host on a
bounded sample of the same workload.
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "gossip-sim_amd")
METRIC = "push-propagation edges/sec (origin-BFS rounds/sec) at 1/2/4/8 MI355X, %HBM BW"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def load_pkg():
    spec = importlib.util.spec_from_file_location("gossip_sim_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["gossip_sim_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pmc_traffic(kernel, nodes, slots):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary of
    this same workload (scripts/pmc.sh + scripts/pmc_summary.py), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{kernel}_{nodes}x{slots}.json")),
                       reverse=True):
        with open(path) as f:
            d = json.load(f)
        return d["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(pks, stakes, args, budget_s):
    """Oracle (port of the reference path) on host cores: one origin-sim, rounds until the budget."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob  # test infrastructure: used only as the baseline/checker here
    sim = ob.Sim(ob.PHILOX, args.seed, pks, stakes, args.fanout)
    t0 = time.perf_counter()
    sim.init_philox(args.active_set_size)
    t_init = time.perf_counter() - t0
    origin = sim.find_nth_largest(1)
    edges, rounds = 0, 0
    t0 = time.perf_counter()
    while True:
        edges += sim.round(origin, args.threshold, args.min_ingress, args.active_set_size, args.rotation_probability,
                           rounds)
        rounds += 1
        el = time.perf_counter() - t0
        if (el >= budget_s and rounds >= 3) or rounds >= args.warmup + args.steps:
            break
    return {"value": edges / el, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"1 origin-sim (origin rank 1) of the same {len(pks)}-node network, rounds 0..{rounds - 1} "
                      f"({edges} pushes in {el:.2f} s; active-set init {t_init:.2f} s untimed); oracle/ "
                      f"reference-structure C++ restatement, single thread",
            "origin_rounds_per_s": rounds / el}


def large_leg(gs, synth, args, nodes=1_000_000, slots=8, warmup=5, steps=20):
    """SURVEY 8(d) C4-shaped secondary measurement (1 GPU): a 1M-node network, 8 origin
    slots (independent sims, origins = node ids 0..7), the step-kernel round with the binned BFS. Reports the propagation path's
    B_prop fraction of HBM peak (north-star target) and the whole round's rate."""
    pks, stakes = synth.network(nodes)
    eng = gs.Engine(stakes, slots, fanout=args.fanout, active_set_size=args.active_set_size,
                    rotation_probability=args.rotation_probability, seed=args.seed, device=0, profile=True)
    eng.set_slots(list(range(slots)), args.min_ingress, args.threshold)
    eng.init_active_sets()
    for r in range(warmup):
        eng.round(r, record=False)
    eng.sync()
    eng.kernel_time_reset()
    t0 = time.perf_counter()
    for r in range(warmup, warmup + steps):
        eng.round(r, record=True)
    eng.sync()
    dt = time.perf_counter() - t0
    summ = eng.summaries()
    E = float(summ["pushes"].astype("float64").sum())
    V = float(summ["visited"].astype("float64").sum())
    b_ms, _ = eng.kernel_time("bfs")
    info = eng.info()
    eng.close()
    b_prop = V * (4 * args.active_set_size + 5) + 8 * E
    ach = b_prop / (b_ms * 1e-3) / 1e9 if b_ms > 0 else None
    return {"workload": f"C4-shaped: {nodes}-node power-law network, {slots} origin slots, step-kernel round",
            "bfs_mode": info["bfs_mode"], "steps": steps, "warmup": warmup,
            "ms_per_step": dt / steps * 1e3, "edges_per_s": E / dt,
            "bfs_us_per_round": b_ms * 1e3 / steps,
            "bfs_roofline": {"bound": "hbm", "achieved": round(ach, 2) if ach else None, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                             "bytes_model": "B_prop (SURVEY 8d)",
                             "kernels": "k_bin_direct/k_bin_expand/k_bin_apply per level + k_bin_gather"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nodes", type=int, default=3000)
    ap.add_argument("--slots", type=int, default=0, help="origin slots per GPU (default: all nodes)")
    ap.add_argument("--fanout", type=int, default=6)
    ap.add_argument("--active-set-size", type=int, default=12)
    ap.add_argument("--rotation-probability", type=float, default=0.01)
    ap.add_argument("--threshold", type=float, default=0.15)
    ap.add_argument("--min-ingress", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0x5EED0003)
    ap.add_argument("--bfs-mode", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--split-round", action="store_true", help="step kernels instead of the one-kernel round")
    ap.add_argument("--no-large", action="store_true", help="skip the 1M-node secondary leg")
    args = ap.parse_args()

    gs = load_pkg()          # loads libgossip_hip.so (and its HIP runtime) before torch, if torch is used at all
    gs.lib()
    import gossip_sim_amd.synth as synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = (torch, tdist)

    def barrier():
        if dist:
            dist[1].barrier()

    def reduce(x, op):
        if not dist:
            return x
        t = dist[0].tensor([x], dtype=dist[0].float64)
        dist[1].all_reduce(t, op=op(dist[1]))
        return float(t.item())

    pks, stakes = synth.network(args.nodes)
    S = args.slots or args.nodes
    eng = gs.Engine(stakes, S, fanout=args.fanout, active_set_size=args.active_set_size,
                    rotation_probability=args.rotation_probability, seed=args.seed + rank, device=local_rank,
                    bfs_mode=args.bfs_mode, profile=not args.no_profile, split_round=args.split_round)
    origins = [s % args.nodes for s in range(S)]
    eng.set_slots(origins, args.min_ingress, args.threshold)
    eng.init_active_sets()
    for r in range(args.warmup):
        eng.round(r, record=False)
    eng.sync()
    eng.kernel_time_reset()
    barrier()
    eng.sync()
    t0 = time.perf_counter()
    for r in range(args.warmup, args.warmup + args.steps):
        eng.round(r, record=True)
    eng.sync()
    barrier()
    dt_local = time.perf_counter() - t0
    summ = eng.summaries()  # [steps, S]
    assert summ.shape[0] == args.steps
    E = float(summ["pushes"].astype("float64").sum())
    V = float(summ["visited"].astype("float64").sum())
    fused = eng.info()["fused_round"]
    k_ms, k_n = eng.kernel_time("round" if fused else "bfs")
    dt = reduce(dt_local, lambda d: d.ReduceOp.MAX)
    E_all = reduce(E, lambda d: d.ReduceOp.SUM)
    asz = args.active_set_size
    # SURVEY.md 8(d) algorithmic bytes of this rank's timed steps:
    #   propagation  B_prop    = V*(4*ASZ + 5) + 8*E
    #   consume      B_consume = 5*E + 16*R        (R = receiving pairs = V - origins)
    #   statistics   B_stats   = 8 per (origin, node)
    b_prop = V * (4 * asz + 5) + 8 * E
    R = V - S * args.steps
    b_round = b_prop + 5 * E + 16 * R + 8.0 * args.nodes * S * args.steps
    b_kernel = b_round if fused else b_prop
    roof = None
    if k_ms > 0:
        achieved = b_kernel / (k_ms * 1e-3) / 1e9
        kname = "k_round_wg" if fused else {gs.GS_BFS_WORKGROUP: "k_bfs_wg", gs.GS_BFS_LEVEL: "k_bfs_level",
                                            gs.GS_BFS_BINNED: "k_bin_expand+k_bin_apply"}[eng.info()["bfs_mode"]]
        traffic, tsrc = pmc_traffic(kname, args.nodes, S)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                "kernel": kname,
                "bytes_model": "B_prop+B_consume+B_stats (SURVEY 8d)" if fused else "B_prop (SURVEY 8d)",
                "bytes_per_launch": round(b_kernel / max(k_n, 1)), "avg_launch_us": round(k_ms * 1e3 / max(k_n, 1), 2),
                "launches": k_n}
    phases = None
    if os.environ.get("GS_PHASE_PROFILE") == "1" and fused:  # workgroup-ms per k_round_wg phase
        names = ["init", "bfs", "csr_stats", "consume_prune", "heavy", "summary"]
        phases = {nm: round(eng.kernel_time("phase." + chr(65 + i))[0], 2) for i, nm in enumerate(names)}
        phases["bfs_levels_per_slot_round"] = round(eng.kernel_time("phase.H")[0] * 1e5 / (S * args.steps), 2)
        lv = eng.kernel_time("phase.H")[0] * 1e5
        for i, nm in enumerate(["lvl_row_load_cyc", "lvl_push_cyc", "lvl_rest_iters_cyc", "lvl_barriers_cyc"]):
            phases[nm] = round(eng.kernel_time("phase." + chr(73 + i))[0] * 1e5 / max(lv, 1), 1)  # per level
    out = {
        "metric": METRIC,
        "value": E_all / dt,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (deterministic Philox power-law stakes, SURVEY.md 8(d))",
        "config": {"workload": "C2: ~3,000-node power-law network, all origins batched, rotation-probability 0.01",
                   "nodes": args.nodes, "origin_slots_per_gpu": S, "push_fanout": args.fanout,
                   "active_set_size": asz, "rotation_probability": args.rotation_probability,
                   "prune_stake_threshold": args.threshold, "min_ingress_nodes": args.min_ingress,
                   "bfs_mode": eng.info()["bfs_mode"], "fused_round": fused,
                   "parallelism": f"origin-sharded x{world}"},
        "origin_rounds_per_s": S * args.steps * world / dt,
        "roofline": roof,
        **({"phases_wg_ms": phases} if phases else {}),
        "cpu_baseline": None,
    }
    eng.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pks, stakes, args, args.cpu_budget)
    if rank == 0 and world == 1 and not args.no_large and args.nodes < 1_000_000:
        out["large_1m"] = large_leg(gs, synth, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist[1].destroy_process_group()


if __name__ == "__main__":
    main()
