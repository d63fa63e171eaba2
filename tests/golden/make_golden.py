"""Generate tests/golden/six_node_cluster.json from the oracle (test infrastructure).

The six-node cluster is the one of the reference's test_mst / test_pruning
(gossip.rs:1041-1067, gossip_main.rs:1071-1117): Pubkey::new_unique() counters
1..6, stakes from ChaChaRng::from_seed([189; 32]).gen_range(1, 2^20 SOL), active
sets initialised in Pubkey order from the same stream with sorted candidates
(test = true). The oracle that produced the entries reproduces every assertion
of test_mst and test_pruning (tests/test_oracle_kats.py), so the fixture pins
the GPU path to the reference's own known answers.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_bind as ob  # noqa: E402

LAMPORTS = 1_000_000_000
MAX_STAKE = (1 << 20) * LAMPORTS


def main():
    rng = ob.Rng.chacha(bytes([189] * 32))
    pks = [ob.counter_pubkey(i) for i in range(1, 7)]
    stakes = [rng.gen_range(1, MAX_STAKE) for _ in range(6)]
    sim = ob.Sim(ob.COMPAT, 0, pks, stakes, 2)
    sim.init_compat(rng, 12)
    entries = {str(n): {str(k): sim.entry(n, k) for k in range(25)} for n in range(6)}
    out = {
        "doc": "test_mst/test_pruning six-node cluster; node index = Pubkey order (new_unique counters 1..6)",
        "pubkeys_hex": [p.hex() for p in pks],
        "base58": [ob.base58(p) for p in pks],
        "stakes": stakes,
        "active_set_size": 12,
        "push_fanout": 2,
        "origin_index": 5,
        "entries": entries,
        # reference assertions (gossip.rs:1089-1155, gossip_main.rs:1127-1152)
        "expect_distances": [2, 3, 1, 2, 1, 0],
        "expect_num_inbound": [3, 1, 3, 2, 3],
        "expect_hops": [[0, 1, 4], [0, 4, 2], [1, 0, 3], [2, 0, 3], [2, 3, 3], [2, 5, 1], [4, 2, 2], [4, 3, 3],
                        [4, 5, 1]],
        "expect_prunes_iteration_19": [[2, 0], [0, 1], [4, 3]],
    }
    with open(os.path.join(HERE, "six_node_cluster.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
