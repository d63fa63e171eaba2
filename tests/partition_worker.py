"""One rank of a node-range-partitioned run (tests/test_partition.py). Env: RANK,
WORLD_SIZE, MASTER_ADDR/PORT, GS_PART_OUT (npz path), GS_PART_CASE (small | large),
GS_PART_BACKEND (gloo | nccl), GS_PART_EXCHANGE (prune exchange: auto | records | dense),
GS_PART_BFS (replicated | frontier)."""
import os
import pickle
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import engine_bind as eb  # noqa: E402

from partition_case import CASES, cache_rows, run_case, stakes_of  # noqa: E402

RCCL_REFUSED = 77  # exit code: RCCL would not put two ranks on the one GPU of the box


def main():
    import torch.distributed as tdist
    import gossip_sim_amd.partition as gp
    case = os.environ.get("GS_PART_CASE", "small")
    backend = os.environ.get("GS_PART_BACKEND", "gloo")
    try:
        tdist.init_process_group(backend)
        if backend == "nccl":  # the first collective is where RCCL builds its communicator
            import torch
            torch.cuda.set_device(0)
            t = torch.ones(1, device="cuda")
            tdist.all_reduce(t)
            torch.cuda.synchronize()
    except Exception as ex:  # noqa: BLE001
        if backend == "nccl":
            print(f"RCCL setup failed: {ex}", flush=True)
            sys.exit(RCCL_REFUSED)
        raise
    rank = tdist.get_rank()
    st = stakes_of(case, eb.synth)
    pe = gp.PartitionedEngine(st, len(CASES[case]["mi"]), device=0, seed=CASES[case]["seed"],
                              rotation_probability=CASES[case]["p"],
                              exchange=os.environ.get("GS_PART_EXCHANGE", "auto"),
                              bfs=os.environ.get("GS_PART_BFS", "replicated"))
    modes = []
    out = run_case(pe, case, st, ranges=[(pe.node_lo, pe.node_hi)],
                   on_round=lambda r, e: modes.append((r, e.last_mode or "", e.records)))
    out["lo"], out["hi"] = np.array([pe.node_lo]), np.array([pe.node_hi])
    out["xmodes"] = np.array([m for _, m, _ in modes])
    out["xrecords"] = np.array([n for _, _, n in modes], dtype=np.uint64)
    out["xbytes"] = np.array([pe.bytes_in], dtype=np.uint64)
    out["levels"] = np.array([pe.levels, pe.level_bytes], dtype=np.uint64)
    out["async"] = np.array([pe.async_rounds, pe.async_redo], dtype=np.uint64)
    info = pe.info()
    out["bytes"] = np.array([info["device_bytes"], info["pair_bytes"], info["other_bytes"]], dtype=np.uint64)
    np.savez(os.environ["GS_PART_OUT"], **out)
    rows = {k: cache_rows(pe, case, k, pe.node_lo, pe.node_hi) for k in range(len(CASES[case]["mi"]))}
    with open(os.environ["GS_PART_OUT"] + ".caches", "wb") as f:
        pickle.dump(rows, f)  # (this test's own output, read back by the test)
    tdist.barrier()
    tdist.destroy_process_group()
    print(f"rank {rank}: nodes [{pe.node_lo}, {pe.node_hi}) device bytes {info['device_bytes']} "
          f"(per-pair {info['pair_bytes']}, other {info['other_bytes']}); exchange received {pe.bytes_in} B; "
          f"rounds (mode, records): {[(m, n) for _, m, n in modes if m]} ok", flush=True)


if __name__ == "__main__":
    main()
