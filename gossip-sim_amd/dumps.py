"""The reference's per-round debug dumps (gossip.rs:365-431) for one slot of an Engine:
print_hops, print_node_orders, print_mst, print_prunes, print_pushes, with the same
record texts (env_logger INFO records). The reference iterates HashMaps (arbitrary
order); here entries come in node-id order. Call after gs_run_gossip (and
send_prunes for print_prunes): the step path keeps the inbound records in HBM.
"""
import sys
import time


def _log(out, msg, target="gossip_sim::gossip"):
    t = time.time()
    stamp = time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(t)) + f".{int((t % 1) * 1e9):09d}Z"
    print(f"[{stamp} INFO  {target}] {msg}", file=out)


def print_hops(eng, slot, keys, out=sys.stderr):
    _log(out, "DISTANCES FROM ORIGIN")
    for v, h in enumerate(eng.distances(slot).tolist()):
        _log(out, f"dest node, hops: ({keys[v]}, {h})")


def print_node_orders(eng, slot, keys, out=sys.stderr):
    _log(out, "NODE ORDERS")
    for v, lst in enumerate(eng.inbound_lists(slot)):
        if not lst:
            continue
        _log(out, f"----- dest node, num_inbound: {keys[v]}, {len(lst)} -----")
        for src, hop in lst:
            _log(out, f"neighbor pubkey, order: {keys[src]}, {hop}")


def print_mst(eng, slot, keys, out=sys.stderr):
    _log(out, "MST: ")
    for src, dests in sorted(eng.mst(slot).items()):
        _log(out, f"##### src: {keys[src]} #####")
        for d in dests:
            _log(out, f"dest: {keys[d]}")


def print_prunes(eng, slot, keys, out=sys.stderr):
    _log(out, "PRUNES: ")
    by_pruner = {}
    for pruner, prunee in eng.prunes(slot):
        by_pruner.setdefault(pruner, []).append(prunee)
    for pruner in sorted(by_pruner):
        _log(out, f"--------- Pruner: {keys[pruner]} ---------")
        for prunee in by_pruner[pruner]:
            _log(out, f"Prunee: {keys[prunee]}")


def print_pushes(eng, slot, keys, out=sys.stderr):
    _log(out, "PUSHES: ")
    for src, dests in sorted(eng.pushes(slot).items()):
        _log(out, f"************* SRC: {keys[src]}, # {len(dests)} *************")
        for d in dests:
            _log(out, f"Dest: {keys[d]}")
