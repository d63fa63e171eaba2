"""One rank of a node-range-partitioned run (tests/test_partition.py). Env: RANK,
WORLD_SIZE, MASTER_ADDR/PORT, GS_PART_OUT (npz path), GS_PART_BACKEND (gloo)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import engine_bind as eb  # noqa: E402

from partition_case import CASE, run_case  # noqa: E402


def main():
    import torch.distributed as tdist
    import gossip_sim_amd.partition as gp
    tdist.init_process_group(os.environ.get("GS_PART_BACKEND", "gloo"))
    rank = tdist.get_rank()
    st = eb.synth.network(CASE["n"])[1]
    pe = gp.PartitionedEngine(st, len(CASE["origins"]), device=0, seed=CASE["seed"],
                              rotation_probability=CASE["p"])
    out = run_case(pe)
    out["lo"], out["hi"] = np.array([pe.node_lo]), np.array([pe.node_hi])
    np.savez(os.environ["GS_PART_OUT"], **out)
    tdist.barrier()
    tdist.destroy_process_group()
    print(f"rank {rank}: nodes [{pe.node_lo}, {pe.node_hi}) ok")


if __name__ == "__main__":
    main()
