"""Per-rank shares of a node-range-partitioned C5 run, measured on ONE GPU.

Launched as K ranks over gloo, all on device 0 (torch.distributed.run --nproc-per-node K
--master-addr 127.0.0.1 scripts/part_share.py --bfs frontier|replicated). The ranks' engine calls
take turns (PartitionedEngine(profile=True, serialize=True)): each rank's kernels run alone on
the device, so a rank's phase times are its share of a K-GPU run, without the interconnect.
The collectives ("exchange") run over gloo through host memory here and are reported with
their payload bytes only; their xGMI cost is modelled in DESIGN.md §7.
Rank 0 prints one JSON line per rank: ms per round per phase, BFS levels, frontier bytes
received per round, prune-exchange bytes per round."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bfs", default="frontier", choices=["frontier", "replicated"])
    ap.add_argument("--nodes", type=int, default=10_000_000)
    ap.add_argument("--slots", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"],
                    help="nccl: records and prune words stay on the device (one rank per GPU: world 1 here)")
    args = ap.parse_args()
    import torch.distributed as tdist
    if args.backend == "nccl":
        import torch
        torch.cuda.set_device(0)
    tdist.init_process_group(args.backend)
    rank, world = tdist.get_rank(), tdist.get_world_size()
    import importlib.util
    spec = importlib.util.spec_from_file_location("gossip_sim_amd", os.path.join(ROOT, "gossip-sim_amd", "__init__.py"),
                                                  submodule_search_locations=[os.path.join(ROOT, "gossip-sim_amd")])
    gs = importlib.util.module_from_spec(spec)
    sys.modules["gossip_sim_amd"] = gs
    spec.loader.exec_module(gs)
    import gossip_sim_amd.partition as gp
    import gossip_sim_amd.synth as synth
    n = args.nodes
    stakes = synth.power_law_stakes(n)
    order = np.lexsort((np.arange(n), -stakes.astype(np.float64)))
    origins = [int(x) for x in order[:args.slots]]
    t0 = time.perf_counter()
    pe = gp.PartitionedEngine(stakes, args.slots, device=0, seed=0x5EED0003, rotation_probability=0.013333,
                              bfs=args.bfs, profile=True, serialize=True)
    pe.set_slots(origins, [2] * args.slots, [0.15] * args.slots)
    pe.init_active_sets()
    t_init = time.perf_counter() - t0
    for r in range(args.warmup):
        pe.round(r, record=False)
    pe.prof.clear()
    lb0, xb0 = pe.level_bytes, pe.bytes_in
    tdist.barrier()
    t1 = time.perf_counter()
    levels = []
    for r in range(args.warmup, args.warmup + args.steps):
        pe.round(r, record=True)
        levels.append(pe.levels)
    pe.sync()
    tdist.barrier()
    wall = (time.perf_counter() - t1) / args.steps
    K = args.steps
    row = {"rank": rank, "world": world, "bfs": args.bfs, "nodes": [pe.node_lo, pe.node_hi],
           "ms_per_round": {k: round(v / K * 1e3, 3) for k, v in sorted(pe.prof.items())},
           "engine_ms_per_round": round(sum(v for k, v in pe.prof.items() if k != "exchange") / K * 1e3, 3),
           "levels": levels, "frontier_bytes_in_per_round": (pe.level_bytes - lb0) / K,
           "prune_bytes_in_per_round": (pe.bytes_in - xb0) / K, "wall_ms_per_round_serialized": round(wall * 1e3, 2),
           "device_bytes": pe.info()["device_bytes"], "setup_s": round(t_init, 1),
           "rounds": [args.warmup, args.warmup + args.steps]}
    row["backend"] = args.backend
    rows = [None] * world
    if args.backend == "gloo":
        tdist.all_gather_object(rows, row)
    else:
        rows = [row]  # (world 1)
    if rank == 0:
        for x in rows:
            print(json.dumps(x), flush=True)
    pe.close()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
