#!/usr/bin/env python3
"""bench.py -- push-propagation edges/s on MI355X (BASELINE.json metric).

Headline workload (BASELINE.json configs[1], "C2"): a ~3,000-node synthetic
power-law stake network, ALL 3,000 origins batched as independent sims (slots) of
one engine, rotation probability 0.01, push fanout 6, active-set size 12. A step is
one full gossip iteration for every slot (gossip_main.rs:449-564: run_gossip ->
consume -> send_prunes -> prune_connections -> chance_to_rotate -> the
measured-round statistics), with all inputs resident in HBM. The K timed steps are
rounds [W, W+K) of the simulation (W = --warmup); `config.rounds` says which, and
`steady_state` times rounds [60, 160) of the same engine (past the first prune
waves, where pushes per origin-round settle near 3N).

value = pushes to non-failed peers over all slots and ranks / wall time of the K
timed steps (max over ranks).

Multi-GPU (one process per GPU, no data-path collective). Default --scaling strong: the
ranks split the 3,000 origins of ONE C2 trial (same seed; rank r takes origins
[r*S/K, (r+1)*S/K)) -- the north star's origin-sharded sweep; with --check-shard rank 0
checks the gathered per-round summaries of every origin against all origins run on one
engine. At N > 1 the line also carries `weak_trial`: the ranks then run independent C2
trials (rank r: all 3,000 origins, Philox seed + r), the per-GPU work of one C2 at every N.
--scaling weak makes that the headline instead. --workload c4 / c5 run BASELINE C4's 13
sweep sims (1M nodes) / C5's 16 origins (10M nodes) instead, dealt over the ranks (strong)
or all on every rank as its own trial (weak). torch.distributed carries only the barrier,
the timing max/sum and the summary gather.

roofline: the dominant kernel (k_round_wg) with SURVEY.md 8(d) algorithmic bytes
per launch, divided by that kernel's average duration measured with hipEvents on
the engine stream over the timed steps; `traffic` = HBM bytes per launch from the
committed rocprofv3 --pmc summary of the SAME round window (the newest profiles/r*/ stamped
with the loaded library's kernel hash), or null.
cpu_baseline: the oracle (reference-structure C++ restatement: maps keyed by
32-byte pubkeys, one origin per sim) on all host cores (independent origin-sims
dealt over std::threads) on a bounded sample of the same workload;
cpu_baseline_1core: the same code on one core.
Secondary legs at N = 1 (reported beside `value`, never part of it):
  c4: BASELINE C4 as configured -- 1M-node network, origin rank 1, the fail-nodes
      sweep (0.1..0.5, when-to-fail 0) and the prune-stake-threshold sweep
      (0.05..0.40) as 13 slots of one engine; the propagation path's B_prop
      fraction of HBM peak is the north-star figure.
  c3: BASELINE C3's per-GPU share -- 100k nodes, active-set-size sweep values 12
      and 20 (sims 0 and 8 of 16 dealt over 8 GPUs), one engine per value.
  c5: BASELINE C5's 10M-node graph on one GPU: origin ranks 1..16 (--c5-slots) as the
      slots of one engine (the multi-source BFS), unpartitioned.
"""
import argparse
import glob
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


_KHASH = None


def kernel_hash():
    global _KHASH
    if _KHASH is None:
        _KHASH = sys.modules["gossip_sim_amd"].kernel_hash() if "gossip_sim_amd" in sys.modules \
            else load_pkg().kernel_hash()
    return _KHASH


def pmc_traffic(tag):
    """HBM bytes per launch from the newest committed rocprofv3 --pmc summary named
    profiles/r*/pmc_<tag>.json (scripts/pmc_summary.py, scripts/pmc_round.py), or None.
    A summary counts only if it is stamped with the kernel hash of the sources the library
    is built from (gossip_sim_amd.kernel_hash): a profile of other kernels gives null and
    the reason. Returns (bytes, source, note)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_{tag}.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        src = os.path.relpath(path, ROOT)
        kh = d.get("kernel_hash")
        if kernel_hash() is None:
            return None, src, "no kernel hash: GS_LIB_VARIANT build or libgossip_hip.so older than its sources"
        if kh != kernel_hash():
            return None, src, f"stale: {src} measured kernels {kh}, built kernels are {kernel_hash()}"
        return d["traffic_bytes_per_launch"], src, f"PMC at kernel hash {kh}"
    return None, None, "no PMC summary for this window"


def trace_window(tag):
    """The committed rocprofv3 kernel-trace average of the same window
    (profiles/r*/trace_<tag>.json, scripts/trace_window.py), if stamped with the built
    kernels' hash: (avg_us, source) or (None, reason)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"trace_{tag}.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        src = os.path.relpath(path, ROOT)
        if kernel_hash() is None or d.get("kernel_hash") != kernel_hash():
            return None, f"stale: {src} traced kernels {d.get('kernel_hash')}"
        return round(d["avg_us"], 2), src
    return None, "no kernel trace of this window"


def roofline(bytes_total, ms, launches, kernel, model, traffic_tag=None):
    if ms <= 0:
        return None
    ach = bytes_total / (ms * 1e-3) / 1e9
    traffic, tsrc, tnote = pmc_traffic(traffic_tag) if traffic_tag else (None, None, "not collected")
    tr_us, tr_src = trace_window(traffic_tag) if traffic_tag else (None, "not collected")
    return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
            "traffic_note": tnote, "kernel_hash": kernel_hash(), "kernel": kernel,
            "bytes_model": model, "bytes_per_launch": round(bytes_total / max(launches, 1)),
            "avg_launch_us": round(ms * 1e3 / max(launches, 1), 2), "launches": launches,
            "rocprof_avg_us": tr_us, "rocprof_source": tr_src}


def b_prop(V, E, asz):
    """V*(4*ASZ + 5) + 8*E per origin-round of the propagation kernel."""
    return V * (4 * asz + 5) + 8 * E


# ------------------------------------------------------------------ CPU baseline ----
def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob  # test infrastructure: used only as the baseline/checker here
    return ob


def cpu_baseline_1core(pks, stakes, args, budget_s):
    """Oracle on one core: one origin-sim, rounds until the budget."""
    ob = _oracle()
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
        if (el >= budget_s and rounds >= 3) or rounds >= 60:
            break
    return {"value": edges / el, "unit": "edges/s", "cores": 1, "kind": "port",
            "sample": f"1 origin-sim (origin rank 1) of the same {len(pks)}-node network, rounds 0..{rounds - 1} "
                      f"({edges} pushes in {el:.2f} s; active-set init {t_init:.2f} s untimed); oracle/ "
                      f"reference-structure C++ restatement, single thread",
            "origin_rounds_per_s": rounds / el}


def cpu_baseline_all(pks, stakes, args, rounds=40):
    """Oracle on all the host's cores: independent origin-sims (origins = node ids
    0, 1, ... as in the GPU run) dealt over std::threads, rounds [0, rounds)."""
    import ctypes as C
    import numpy as np
    ob = _oracle()
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    n_sims = threads
    f = ob.lib.or_bench_parallel
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint64, C.c_char_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p, C.c_size_t,
                  C.c_double, C.c_size_t, C.c_double, C.c_uint32, C.c_uint32, C.POINTER(C.c_double),
                  C.POINTER(C.c_double)]
    st = np.ascontiguousarray(stakes, dtype=np.uint64)
    org = np.arange(n_sims, dtype=np.uint32) % len(pks)
    ti, tr = C.c_double(), C.c_double()
    edges = f(args.seed, ob.pk_blob(pks), st.ctypes.data, len(pks), args.fanout, args.active_set_size,
              org.ctypes.data, n_sims, args.threshold, args.min_ingress, args.rotation_probability, rounds, threads,
              C.byref(ti), C.byref(tr))
    return {"value": edges / tr.value, "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"{n_sims} origin-sims (origins = node ids 0..{n_sims - 1}) of the same {len(pks)}-node "
                      f"network, rounds 0..{rounds - 1} each ({edges} pushes in {tr.value:.2f} s wall on {threads} "
                      f"threads; active-set init {ti.value:.2f} s untimed); oracle/ reference-structure C++ "
                      f"restatement, one std::thread per core",
            "origin_rounds_per_s": n_sims * rounds / tr.value}


# ------------------------------------------------------------------ secondary legs ----
def c4_leg(gs, synth, args, nodes=1_000_000, warmup=5, steps=20):
    """BASELINE C4 as configured on one GPU (13 sims as slots of one engine)."""
    import numpy as np
    stakes = synth.power_law_stakes(nodes)
    origin = int(np.argmax(stakes))  # origin rank 1
    fr = [0.1, 0.2, 0.3, 0.4, 0.5] + [0.0] * 8
    thr = [args.threshold] * 5 + [round(0.05 * (j + 1), 2) for j in range(8)]
    if args.c4_sims:  # one rank's share of the sweep (DESIGN 7's multi-GPU predictions)
        pick = [int(x) for x in args.c4_sims.split(",")]
        fr, thr = [fr[i] for i in pick], [thr[i] for i in pick]
    S = len(fr)
    eng = gs.Engine(stakes, S, fanout=args.fanout, active_set_size=args.active_set_size,
                    rotation_probability=0.013333, seed=args.seed, device=0, profile=True, bfs_mode=args.large_mode)
    eng.set_slots([origin] * S, args.min_ingress, thr)
    eng.init_active_sets()
    eng.fail_nodes(fr)  # when-to-fail 0: before the first BFS (gossip_main.rs:449-452)
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
    fam = {k: eng.kernel_time(k)[0] for k in ("bfs", "gather", "gather_consume", "consume", "rotate", "stats")}
    for k in ("gather", "gather_consume"):
        if not fam[k]:
            del fam[k]
    phases = gather_phases(eng)
    info = eng.info()
    eng.close()
    mode = {2: "level", 3: "binned", 4: "multi"}.get(info["bfs_mode"], str(info["bfs_mode"]))
    bp = b_prop(V, E, args.active_set_size)
    # committed PMC / trace summaries are of the 13-slot configuration: a share run
    # (--c4-sims) looks them up under its own slot set, so it never reports another
    # configuration's traffic (null unless a summary of that share exists)
    tag = f"bfs_{mode}_c4" + (f"_s{args.c4_sims.replace(',', '-')}" if args.c4_sims else "")
    pers = info.get("bfs_persistent", False)
    return {"workload": f"C4: {nodes}-node power-law network, origin rank 1, fail-nodes 0.1..0.5 (when-to-fail 0) + "
                        f"prune-stake-threshold 0.05..0.40: {S} sims as slots of one engine",
            "bfs_mode": mode, "rounds": [warmup, warmup + steps], "ms_per_step": dt / steps * 1e3,
            "edges_per_s": E / dt, "origin_rounds_per_s": S * steps / dt,
            "pushes_per_origin_round": E / (S * steps),
            "prunes_per_round_max": int(summ["prunes"].astype("int64").sum(axis=1).max()),
            "us_per_round": {k: round(v * 1e3 / steps, 1) for k, v in fam.items()},
            **({"gather_phases_wg_ms": phases} if phases else {}),
            # multi: the level loop plus the gather that writes hops / in-degrees / inbound rows
            # (with GS_MV_FUSED=1 the gather runs fused with consume, and its whole time is charged)
            "bfs_roofline": roofline(bp, fam["bfs"] + fam.get("gather", 0.0) + fam.get("gather_consume", 0.0), steps,
                                     f"BFS ({mode}: " + (("one persistent launch" if pers else "expand/apply per level")
                                                         + " + " + ("fused gather/consume)" if "gather_consume" in fam
                                                                    else "gather)") if mode == "multi"
                                                         else "per level)"),
                                     "B_prop (SURVEY 8d), summed over slots", tag)}


def gather_phases(eng):
    """GS_PHASE_PROFILE=1 (multi BFS): workgroup-ms per phase (thread 0 of each workgroup),
    and the pool records the gathers read ("pool_records": the count x 1e-5)."""
    if os.environ.get("GS_PHASE_PROFILE") != "1":
        return None
    names = {12: "count_scan", 13: "range_place", 11: "body_all", 14: "body_light", 15: "body_heavy",
             0: "small_setup", 1: "small_expand_loads", 2: "small_atomics_places", 3: "small_lt_barrier",
             4: "small_levels_e-5", 5: "lv_setup", 6: "lv_loads", 7: "lv_atomics_stores", 8: "lv_barrier",
             9: "lv_levels_e-5", 10: "pool_records",
             16: "apply_tcol_scan", 17: "apply_vis_load", 18: "apply_records", 19: "apply_tail"}
    return {nm: round(eng.kernel_time("phase." + chr(65 + i))[0], 2) for i, nm in names.items()}


def c5_leg(gs, synth, args, nodes=10_000_000, slots=None, warmup=3, steps=10):
    """BASELINE C5 as configured, on one GPU: a 10M-node network, origin ranks 1..16 as 16
    slots of ONE engine (the multi-source BFS over one slot group). A node-range partition
    over K ranks divides the per-(slot, node) state; every rank runs this whole BFS
    (DESIGN.md section 7), so the propagation figures are the per-GPU work of C5."""
    import numpy as np
    slots = slots or args.c5_slots
    stakes = synth.power_law_stakes(nodes)
    order = np.lexsort((np.arange(nodes), -stakes.astype(np.float64)))  # rank order, ties by id
    origins = [int(x) for x in order[:slots]]
    eng = gs.Engine(stakes, len(origins), fanout=args.fanout, active_set_size=args.active_set_size,
                    rotation_probability=0.013333, seed=args.seed, device=0, profile=True, bfs_mode=args.large_mode)
    eng.set_slots(origins, args.min_ingress, args.threshold)
    t0 = time.perf_counter()
    eng.init_active_sets()
    eng.sync()
    t_init = time.perf_counter() - t0
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
    fam = {k: eng.kernel_time(k)[0] for k in ("bfs", "gather", "consume", "rotate", "stats")}
    phases = gather_phases(eng)
    info = eng.info()
    eng.close()
    mode = {2: "level", 3: "binned", 4: "multi"}.get(info["bfs_mode"], str(info["bfs_mode"]))
    return {**({"gather_phases_wg_ms": phases} if phases else {}),
            "workload": f"C5 on one GPU: {nodes}-node power-law network, origin ranks 1-{len(origins)} as "
                        f"slots of one engine (unpartitioned; every partition rank runs this BFS)",
            "bfs_mode": mode, "rounds": [warmup, warmup + steps], "ms_per_step": dt / steps * 1e3,
            "edges_per_s": E / dt, "origin_rounds_per_s": len(origins) * steps / dt,
            "pushes_per_origin_round": E / (len(origins) * steps), "init_active_sets_s": t_init,
            "us_per_round": {k: round(v * 1e3 / steps, 1) for k, v in fam.items()},
            "device_bytes": info["device_bytes"], "pair_bytes": info["pair_bytes"],
            "bfs_roofline": roofline(b_prop(V, E, args.active_set_size), fam["bfs"] + fam["gather"], steps,
                                     f"BFS ({mode}" + (": expand/apply per level + gather)" if mode == "multi" else ")"),
                                     "B_prop (SURVEY 8d), summed over slots", f"bfs_{mode}_c5")}


class profile_only:
    """GS_PROFILE_ONLY=<families> around engine creation: the engine records timing events
    only around those families (each recorded family boundary idles the GPU several us;
    the C3 leg's one-slot engines had ~34 us of such gaps per round)."""

    def __init__(self, fams):
        self.fams, self.old = fams, None

    def __enter__(self):
        self.old = os.environ.get("GS_PROFILE_ONLY")
        os.environ["GS_PROFILE_ONLY"] = self.fams
        return self

    def __exit__(self, *exc):
        if self.old is None:
            os.environ.pop("GS_PROFILE_ONLY", None)
        else:
            os.environ["GS_PROFILE_ONLY"] = self.old


BFS_FAMS = "bfs,gather,gather_consume"


def c3_leg(gs, synth, args, nodes=100_000, warmup=5, steps=20):
    """BASELINE C3's share of one GPU: ASZ 12 and 20 (sims 0 and 8 of the 16-sim sweep
    dealt over 8 GPUs), one engine (one slot) per value, origin rank 1."""
    import numpy as np
    stakes = synth.power_law_stakes(nodes)
    origin = int(np.argmax(stakes))
    engs = []
    for asz in (12, 20):
        with profile_only(BFS_FAMS):  # (only the BFS families are reported)
            e = gs.Engine(stakes, 1, fanout=args.fanout, active_set_size=asz, rotation_probability=0.013333,
                          seed=args.seed, device=0, profile=True, bfs_mode=args.large_mode)
        e.set_slots([origin], args.min_ingress, args.threshold)
        e.init_active_sets()
        engs.append((asz, e))
    import threading

    def run(e, r0, r1, rec):  # one host thread per engine: the two sims' BFS level loops overlap
        for r in range(r0, r1):
            e.round(r, record=rec)
        e.sync()

    def both(r0, r1, rec):
        th = [threading.Thread(target=run, args=(e, r0, r1, rec)) for _, e in engs]
        for t in th:
            t.start()
        for t in th:
            t.join()

    both(0, warmup, False)
    for _, e in engs:
        e.kernel_time_reset()
    t0 = time.perf_counter()
    both(warmup, warmup + steps, True)
    dt = time.perf_counter() - t0
    E = bp = b_ms = 0.0
    for asz, e in engs:
        s = e.summaries()
        Ee = float(s["pushes"].astype("float64").sum())
        Ve = float(s["visited"].astype("float64").sum())
        E += Ee
        bp += b_prop(Ve, Ee, asz)
        b_ms += sum(e.kernel_time(k)[0] for k in ("bfs", "gather", "gather_consume"))
        mode = {2: "level", 3: "binned", 4: "multi"}.get(e.info()["bfs_mode"])
        e.close()
    return {"workload": f"C3 per-GPU share: {nodes}-node network, active-set-size sweep values 12 and 20, one "
                        f"engine (stream, host thread) each, run concurrently, origin rank 1", "bfs_mode": mode, "rounds": [warmup, warmup + steps],
            "ms_per_step": dt / steps * 1e3, "edges_per_s": E / dt,
            "bfs_roofline": roofline(bp, b_ms, 2 * steps, f"BFS ({mode})", "B_prop (SURVEY 8d)", f"bfs_{mode}_c3")}


def sweep_workload(gs, synth, args, rank, world, dev, barrier, reduce):
    """--workload c4 | c5 over one process per GPU (independent sims, no
    data-path collective).
    c4: BASELINE C4's 13 sweep sims (fail-nodes 0.1..0.5 at when-to-fail 0, then
        prune-stake-threshold 0.05..0.40) over the 1M-node network;
    c5: BASELINE C5's 16 origins (stake ranks 1..16) over the 10M-node network.
    --scaling strong deals the sims round-robin over the ranks (sweep.shard: the total work
    is fixed); --scaling weak gives every rank all of them as its own trial (Philox seed +
    rank: the per-GPU work is fixed). Each rank runs its sims as slots of one engine;
    value = all ranks' pushes / the slowest rank's time."""
    import numpy as np
    kind = args.workload
    if kind == "c3":
        return c3_sweep_workload(gs, synth, args, rank, world, dev, barrier, reduce)
    if kind == "c4":
        nodes = 1_000_000
        stakes = synth.power_law_stakes(nodes)
        origin = int(np.argmax(stakes))
        n_all = 13
        org_all = [origin] * n_all
        fr_all = [0.1, 0.2, 0.3, 0.4, 0.5] + [0.0] * 8
        thr_all = [args.threshold] * 5 + [round(0.05 * (j + 1), 2) for j in range(8)]
        what = ("C4: 1M-node power-law network, origin rank 1, fail-nodes 0.1..0.5 + prune-stake-threshold "
                "0.05..0.40 (13 sims)")
    else:
        nodes = 10_000_000
        stakes = synth.power_law_stakes(nodes)
        order = np.lexsort((np.arange(nodes), -stakes.astype(np.float64)))
        n_all = 16
        org_all = [int(x) for x in order[:n_all]]
        fr_all = [0.0] * n_all
        thr_all = [args.threshold] * n_all
        what = "C5: 10M-node power-law network, origin ranks 1..16 (16 sims)"
    weak = args.scaling == "weak"
    shard = list(range(n_all)) if weak else list(range(rank, n_all, world))
    seed = args.seed + rank if weak else args.seed
    E = 0.0
    eng = None
    if shard:
        with profile_only(BFS_FAMS):  # (roofline_rank0 reads the BFS families only)
            eng = gs.Engine(stakes, len(shard), fanout=args.fanout, active_set_size=args.active_set_size,
                            rotation_probability=0.013333, seed=seed, device=dev, profile=True,
                            bfs_mode=args.large_mode)
        eng.set_slots([org_all[i] for i in shard], args.min_ingress, [thr_all[i] for i in shard])
        eng.init_active_sets()
        if any(fr_all[i] for i in shard):
            eng.fail_nodes([fr_all[i] for i in shard])  # when-to-fail 0 (gossip_main.rs:449-452)
        for r in range(args.warmup):
            eng.round(r, record=False)
        eng.sync()
        eng.kernel_time_reset()
    barrier()
    t0 = time.perf_counter()
    if eng:
        for r in range(args.warmup, args.warmup + args.steps):
            eng.round(r, record=True)
        eng.sync()
    barrier()
    dt = reduce(time.perf_counter() - t0, lambda d: d.ReduceOp.MAX)
    roof = None
    mode = None
    if eng:
        summ = eng.summaries()
        E = float(summ["pushes"].astype("float64").sum())
        V = float(summ["visited"].astype("float64").sum())
        fam = sum(eng.kernel_time(k)[0] for k in ("bfs", "gather", "gather_consume"))
        roof = roofline(b_prop(V, E, args.active_set_size), fam, args.steps, "BFS (this rank's slot group)",
                        "B_prop (SURVEY 8d), summed over the rank's slots")
        mode = eng.info()["bfs_mode"]
        eng.close()
    E_all = reduce(E, lambda d: d.ReduceOp.SUM)
    sims_total = n_all * (world if weak else 1)
    return {"metric": METRIC, "value": E_all / dt, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (deterministic Philox power-law stakes, SURVEY.md 8(d))",
            "config": {"workload": what + (" per rank, rank r = Philox seed + r" if weak else
                                           " dealt round-robin over the ranks"),
                       "nodes": nodes, "sims_total": sims_total, "sims_rank0": len(shard),
                       "rounds": [args.warmup, args.warmup + args.steps],
                       "parallelism": (f"trial-sharded x{world}" if weak else f"sweep-sharded x{world} (one network)"),
                       "bfs_mode": mode},
            "origin_rounds_per_s": sims_total * args.steps / dt, "roofline_rank0": roof, "cpu_baseline": None}


def c3_sweep_workload(gs, synth, args, rank, world, dev, barrier, reduce):
    """--workload c3: BASELINE C3 -- the 100k-node network's active-set-size sweep
    (num-simulations 16, step 1: active-set sizes 12..27, gossip_main.rs:774-800), sims dealt
    round-robin over the ranks (strong: the total work is fixed) or all 16 on every rank with
    Philox seed + rank (weak). Each sim has its own active sets, so each is one engine of one
    slot; a rank runs its engines concurrently (one host thread and stream each)."""
    import threading
    import numpy as np
    nodes = 100_000
    stakes = synth.power_law_stakes(nodes)
    origin = int(np.argmax(stakes))
    sizes = [12 + i for i in range(16)]
    weak = args.scaling == "weak"
    mine = sizes if weak else sizes[rank::world]
    seed = args.seed + rank if weak else args.seed
    engs = []
    for asz in mine:
        e = gs.Engine(stakes, 1, fanout=args.fanout, active_set_size=asz, rotation_probability=0.013333, seed=seed,
                      device=dev, profile=False, bfs_mode=args.large_mode)  # (no kernel times reported)
        e.set_slots([origin], args.min_ingress, args.threshold)
        e.init_active_sets()
        engs.append((asz, e))

    def run(e, r0, r1, rec):
        for r in range(r0, r1):
            e.round(r, record=rec)
        e.sync()

    def all_engines(r0, r1, rec):
        th = [threading.Thread(target=run, args=(e, r0, r1, rec)) for _, e in engs]
        for t in th:
            t.start()
        for t in th:
            t.join()

    all_engines(0, args.warmup, False)
    for _, e in engs:
        e.kernel_time_reset()
    barrier()
    t0 = time.perf_counter()
    all_engines(args.warmup, args.warmup + args.steps, True)
    barrier()
    dt = reduce(time.perf_counter() - t0, lambda d: d.ReduceOp.MAX)
    E = 0.0
    for _, e in engs:
        E += float(e.summaries()["pushes"].astype("float64").sum())
        e.close()
    E_all = reduce(E, lambda d: d.ReduceOp.SUM)
    sims_total = 16 * (world if weak else 1)
    return {"metric": METRIC, "value": E_all / dt, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": args.scaling, "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (deterministic Philox power-law stakes, SURVEY.md 8(d))",
            "config": {"workload": "C3: 100k-node power-law network, active-set-size sweep 12..27 (16 sims)" +
                                   (" per rank, rank r = Philox seed + r" if weak else " dealt round-robin over the ranks"),
                       "nodes": nodes, "sims_total": sims_total, "sims_rank0": len(mine),
                       "active_set_sizes_rank0": mine, "rounds": [args.warmup, args.warmup + args.steps],
                       "parallelism": (f"trial-sharded x{world}" if weak else f"sweep-sharded x{world} (one network)")},
            "origin_rounds_per_s": sims_total * args.steps / dt, "cpu_baseline": None}


# ------------------------------------------------------------------------ main ----
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--nodes", type=int, default=3000)
    ap.add_argument("--slots", type=int, default=0, help="origin slots (default: all nodes)")
    ap.add_argument("--fanout", type=int, default=6)
    ap.add_argument("--active-set-size", type=int, default=12)
    ap.add_argument("--rotation-probability", type=float, default=0.01)
    ap.add_argument("--threshold", type=float, default=0.15)
    ap.add_argument("--min-ingress", type=int, default=2)
    ap.add_argument("--seed", type=int, default=0x5EED0003)
    ap.add_argument("--bfs-mode", type=int, default=0)
    ap.add_argument("--large-mode", type=int, default=0, help="BFS mode of the c4/c3 legs (0 = AUTO)")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-steady", action="store_true")
    ap.add_argument("--split-round", action="store_true", help="step kernels instead of the one-kernel round")
    ap.add_argument("--no-large", action="store_true", help="skip the c4 / c3 legs")
    ap.add_argument("--only-large", action="store_true", help="run only the c4 / c3 legs (A/B of BFS modes)")
    ap.add_argument("--legs", default="c4,c3", help="with --only-large: which legs (e.g. c4 for a PMC pass)")
    ap.add_argument("--c4-sims", default="", help="c4 leg: only these of the 13 sweep sims (e.g. 0,8: a rank's share)")
    ap.add_argument("--c5-slots", type=int, default=16, help="c5 leg: origin ranks 1..K as slots (16 = C5)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong: the ranks split the origins of one C2 trial (default); weak: rank r runs C2 trial r "
                         "(all origins, Philox seed + r)")
    ap.add_argument("--shard-origins", action="store_true", help="= --scaling strong")
    ap.add_argument("--per-rank-networks", action="store_true", help="= --scaling weak")
    ap.add_argument("--check-shard", action="store_true",
                    help="with origin sharding: rank 0 re-runs all origins on one engine and compares")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="c3: BASELINE C3's 16-sim active-set-size sweep (100k nodes), c4: C4's 13 sims (1M nodes), "
                         "c5: C5's 16 origins (10M nodes) over the ranks (--scaling strong: dealt round-robin; weak: "
                         "every rank all of them, seed + rank)")
    args = ap.parse_args()
    if args.shard_origins:
        args.scaling = "strong"
    elif args.per_rank_networks:
        args.scaling = "weak"
    # strong: one trial's origins split over the ranks; weak: rank r = trial r (all origins,
    # seed + r). At N = 1 both are the same run.
    args.shard_origins = args.scaling == "strong"
    args.per_rank_networks = args.scaling == "weak"

    gs = load_pkg()          # loads libgossip_hip.so (and its HIP runtime) before torch, if torch is used at all
    gs.lib()
    import gossip_sim_amd.synth as synth

    if args.only_large:
        legs = {"c4": c4_leg, "c3": c3_leg, "c5": c5_leg}
        out = {k: legs[k](gs, synth, args) for k in args.legs.split(",")}
        print(json.dumps(out), flush=True)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # GS_BENCH_DEVICE pins every rank to one device (rehearsing the multi-rank path on a one-GPU box)
    dev = int(os.environ.get("GS_BENCH_DEVICE", local_rank))
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

    if args.workload in ("c3", "c4", "c5"):
        out = sweep_workload(gs, synth, args, rank, world, dev, barrier, reduce)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist:
            dist[1].destroy_process_group()
        return

    pks, stakes = synth.network(args.nodes)
    S_all = args.slots or args.nodes
    all_origins = [s % args.nodes for s in range(S_all)]
    if args.shard_origins:
        import gossip_sim_amd.sweep as sweep
        lo, hi = sweep.shard_range(S_all, rank, world)
        origins, seed = all_origins[lo:hi], args.seed
    else:
        origins, seed = all_origins, args.seed + rank
    S = len(origins)
    # (the headline times only the round kernel: an event pair at every family boundary idles
    # the GPU a few us; GS_PROFILE_ONLY is read at engine creation)
    os.environ.setdefault("GS_PROFILE_ONLY", "round,bfs")
    eng = gs.Engine(stakes, S, fanout=args.fanout, active_set_size=args.active_set_size,
                    rotation_probability=args.rotation_probability, seed=seed, device=dev,
                    bfs_mode=args.bfs_mode, profile=not args.no_profile, split_round=args.split_round)
    if os.environ.get("GS_PROFILE_ONLY") == "round,bfs":
        del os.environ["GS_PROFILE_ONLY"]  # (the legs' engines time every family)
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
    einfo = eng.info()
    fused = einfo["fused_round"]
    k_ms, k_n = eng.kernel_time("round" if fused else "bfs")
    dt = reduce(dt_local, lambda d: d.ReduceOp.MAX)
    E_all = reduce(E, lambda d: d.ReduceOp.SUM)
    asz = args.active_set_size
    # SURVEY.md 8(d) algorithmic bytes of this rank's timed steps:
    #   propagation  B_prop    = V*(4*ASZ + 5) + 8*E
    #   consume      B_consume = 5*E + 16*R        (R = receiving pairs = V - origins)
    #   statistics   B_stats   = 8 per (origin, node)
    bp = b_prop(V, E, asz)
    R = V - S * args.steps
    b_round = bp + 5 * E + 16 * R + 8.0 * args.nodes * S * args.steps
    win = f"c2_r{args.warmup}-{args.warmup + args.steps - 1}"
    if fused:
        roof = roofline(b_round, k_ms, k_n, "k_round_wg", "B_prop+B_consume+B_stats (SURVEY 8d)",
                        f"k_round_wg_{win}" if S == 3000 and world == 1 else None)
    else:
        roof = roofline(bp, k_ms, k_n, "BFS", "B_prop (SURVEY 8d)")
    phases = None
    if os.environ.get("GS_PHASE_PROFILE") == "1" and fused:  # workgroup-ms per k_round_wg phase
        names = ["init", "bfs", "csr_stats", "consume_prune", "heavy", "outputs_stats", "summary"]
        phases = {nm: round(eng.kernel_time("phase." + chr(65 + i))[0], 2) for i, nm in enumerate(names)}
    shard_check = None
    if args.shard_origins and world > 1:
        # every origin's per-round summaries, gathered rank-major, against one engine running all origins
        import numpy as np
        import gossip_sim_amd.sweep as sweep
        full = sweep.gather_rows(dist, summ.view(np.uint8).reshape(args.steps, -1), S_all, world,
                                 row_bytes=summ.dtype.itemsize)
        if rank == 0 and args.check_shard:
            ref = gs.Engine(stakes, S_all, fanout=args.fanout, active_set_size=asz,
                            rotation_probability=args.rotation_probability, seed=args.seed, device=dev,
                            bfs_mode=args.bfs_mode)
            ref.set_slots(all_origins, args.min_ingress, args.threshold)
            ref.init_active_sets()
            for r in range(args.warmup + args.steps):
                ref.round(r, record=r >= args.warmup)
            want = ref.summaries().view(np.uint8).reshape(args.steps, -1)
            ref.close()
            shard_check = bool(np.array_equal(full, want))
            if not shard_check:
                raise SystemExit("origin-sharded summaries differ from the one-engine run")
    weak_trial = None
    if world > 1 and args.shard_origins:  # the same ranks as independent trials: rank r = all origins, seed + r
        eng.close()
        wt = gs.Engine(stakes, S_all, fanout=args.fanout, active_set_size=args.active_set_size,
                       rotation_probability=args.rotation_probability, seed=args.seed + rank, device=dev,
                       bfs_mode=args.bfs_mode, profile=False, split_round=args.split_round)
        wt.set_slots(all_origins, args.min_ingress, args.threshold)
        wt.init_active_sets()
        for r in range(args.warmup):
            wt.round(r, record=False)
        wt.sync()
        barrier()
        t1 = time.perf_counter()
        for r in range(args.warmup, args.warmup + args.steps):
            wt.round(r, record=True)
        wt.sync()
        barrier()
        dtw = reduce(time.perf_counter() - t1, lambda d: d.ReduceOp.MAX)
        Ew = reduce(float(wt.summaries()["pushes"].astype("float64").sum()), lambda d: d.ReduceOp.SUM)
        wt.close()
        eng = None
        weak_trial = {"value": Ew / dtw, "unit": "edges/s", "ms_per_step": dtw / args.steps * 1e3,
                      "scaling": "weak", "parallelism": f"trial-sharded x{world} (rank r: all {S_all} origins, "
                                                        f"Philox seed + r)"}
    steady = None
    if not args.no_steady and world == 1 and args.warmup + args.steps <= 60:
        for r in range(args.warmup + args.steps, 60):
            eng.round(r, record=False)
        eng.sync()
        eng.kernel_time_reset()
        n_before = eng.summaries().shape[0]
        t1 = time.perf_counter()
        for r in range(60, 160):
            eng.round(r, record=True)
        eng.sync()
        dts = time.perf_counter() - t1
        ss = eng.summaries()[n_before:]
        Es = float(ss["pushes"].astype("float64").sum())
        Vs = float(ss["visited"].astype("float64").sum())
        ks_ms, ks_n = eng.kernel_time("round" if fused else "bfs")
        bs = b_prop(Vs, Es, asz) + 5 * Es + 16 * (Vs - S * 100) + 8.0 * args.nodes * S * 100
        steady = {"rounds": [60, 160], "value": Es / dts, "ms_per_step": dts / 100 * 1e3,
                  "pushes_per_origin_round": Es / (S * 100),
                  "roofline": roofline(bs if fused else b_prop(Vs, Es, asz), ks_ms, ks_n,
                                       "k_round_wg" if fused else "BFS",
                                       "B_prop+B_consume+B_stats (SURVEY 8d)" if fused else "B_prop (SURVEY 8d)",
                                       "k_round_wg_c2_r60-159" if fused and S == 3000 else None)}
    out = {
        "metric": METRIC,
        "value": E_all / dt,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if args.per_rank_networks else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (deterministic Philox power-law stakes, SURVEY.md 8(d))",
        "config": {"workload": "C2: ~3,000-node power-law network, all origins batched, rotation-probability 0.01",
                   "nodes": args.nodes, "origin_slots_per_gpu": S, "origins_total": S_all if args.shard_origins
                   else S * world, "push_fanout": args.fanout, "active_set_size": asz,
                   "rotation_probability": args.rotation_probability, "prune_stake_threshold": args.threshold,
                   "min_ingress_nodes": args.min_ingress, "bfs_mode": einfo["bfs_mode"], "fused_round": fused,
                   "rounds": [args.warmup, args.warmup + args.steps],
                   "pushes_per_origin_round": E_all / (S * world * args.steps) if not args.shard_origins
                   else E_all / (S_all * args.steps),
                   # which part of the simulation the window times: before the first prune wave
                   # (round ~19) every node pushes to its whole fanout (~6N pushes per
                   # origin-round); after the waves settle (rounds >= 60, `steady_state`) ~3N
                   "regime": ("pre-prune, through the first prune wave (~6N pushes per origin-round)"
                              if args.warmup + args.steps <= 40 else
                              "steady state after the prune waves (~3N pushes per origin-round)"
                              if args.warmup >= 60 else "mixed: the first prune waves and after"),
                   "parallelism": (f"origin-sharded x{world} (one trial)" if args.shard_origins else
                                   f"trial-sharded x{world} (rank r: all origins, Philox seed + r)")},
        "origin_rounds_per_s": (S_all if args.shard_origins else S * world) * args.steps / dt,
        "roofline": roof,
        **({"steady_state": steady} if steady else {}),
        **({"shard_check": shard_check} if shard_check is not None else {}),
        **({"weak_trial": weak_trial} if weak_trial else {}),
        **({"phases_wg_ms": phases} if phases else {}),
        "cpu_baseline": None,
    }
    if eng is not None:
        eng.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_all(pks, stakes, args)
        out["cpu_baseline_1core"] = cpu_baseline_1core(pks, stakes, args, args.cpu_budget)
    if rank == 0 and world == 1 and not args.no_large:
        out["c4"] = c4_leg(gs, synth, args)
        out["c3"] = c3_leg(gs, synth, args)
        out["c5"] = c5_leg(gs, synth, args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist[1].destroy_process_group()


if __name__ == "__main__":
    main()
