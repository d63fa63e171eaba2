"""Debug: level vs binned(all levels) BFS, first differing pair."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import engine_bind as eb
gs = eb.gs
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
st = eb.synth.power_law_stakes(n)
engs = [gs.Engine(st, 3, seed=33, rotation_probability=0.01, bfs_mode=gs.GS_BFS_LEVEL),
        gs.Engine(st, 3, seed=33, rotation_probability=0.01, bfs_mode=gs.GS_BFS_BINNED, binned_all_levels=True)]
for e in engs:
    e.set_slots([0, 17, n - 1], [2, 1, 3], [0.15, 0.3, 0.05])
    e.init_active_sets()
    e.fail_nodes([0.0, 0.2, 0.1])
for r in range(4):
    for e in engs:
        e.run_gossip()
    a, b = engs
    bad = False
    for k in range(3):
        ha, hb = a.hops(k), b.hops(k)
        offa, srca, hopa = a.inbound(k, cap=8 * n)
        offb, srcb, hopb = b.inbound(k, cap=8 * n)
        ca, cb = np.diff(offa.astype(np.int64)), np.diff(offb.astype(np.int64))
        d = np.nonzero(ca != cb)[0]
        print(f"round {r} slot {k}: hops equal {np.array_equal(ha, hb)}, count diffs {len(d)}, E {offa[-1]} vs {offb[-1]}")
        for v in d[:5]:
            print("  node", v, "hop", ha[v], hb[v], "level:", list(zip(srca[offa[v]:offa[v+1]], hopa[offa[v]:offa[v+1]])),
                  "binned:", list(zip(srcb[offb[v]:offb[v+1]], hopb[offb[v]:offb[v+1]])))
            bad = True
    if bad:
        break
    for e in engs:
        e.consume_messages(); e.send_prunes(); e.prune_connections(); e.chance_to_rotate(r)
print("info", engs[1].info())
