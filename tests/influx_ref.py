"""Checker for gossip-sim --influx-file: the data points influx_db.rs:253-602 builds, in
the order gossip_main.rs:372-645 enqueues them, restated in Python over the named
result arrays (test infrastructure only; the product writer is
gossip-sim_amd/cli/gs_influx.cpp). Timestamps follow the writer's reproducible clock:
reading k of the clock is base + 1000 k; a data point reads it once when created
(InfluxDataPoint::new), each histogram line once more (set_and_append_timestamp).
"""
import report_ref as rr


def render(n_nodes, sims, params, *, iterations, warm_up, num_sims, test_type, step, api, base,
           nb_stranded=10, nb_hops=15):
    clock = [0]

    def now():
        t = base + 1000 * clock[0]
        clock[0] += 1
        return t

    start = str(base)
    out = []
    measured = max(iterations - warm_up, 0)
    step_s = str(step) if isinstance(step, int) else rr.display(step)
    for k, ((f, u), p) in enumerate(zip(sims, params)):
        tags = f",simulation_iter={k},start_time={start}"
        if k == 0:
            ts = now()
            sv = {1: p["asz"], 2: p["min_ingress"], 3: p["fanout"], 4: p["thr"], 5: p["fraction"],
                  6: p["origin_rank"], 7: p["p"]}.get(test_type)
            start_value = "N/A" if test_type == 0 else rr.display(float(sv))
            out.append(f"simulation_config,start_time={start} num_simulations={num_sims},"
                       f"gossip_iterations_per_simulation={iterations},warm_up_rounds={warm_up},step_size={step_s},"
                       f"node_count={n_nodes},probability_of_rotation={rr.display(p['p'])},api=\"{api}\","
                       f"start_value=\"{start_value}\",test_type=\"{rr.TEST_TYPE_NAMES[test_type]}\" {ts}")
            vh = u["validator_hist"]
            for i in range(0, len(vh) - 1, 2):
                out.append(f"validator_stake_distribution,start_time={start} bucket={vh[i]},count={vh[i + 1]} {now()}")
        now()  # the "start" marker point
        for it in range(iterations):
            if it % 10 == 0:
                ts = now()
                out.append(f"config{tags} push_fanout={p['fanout']},active_set_size={p['asz']},"
                           f"origin_rank={p['origin_rank']},prune_stake_threshold={rr.display(p['thr'])},"
                           f"min_ingress_nodes={p['min_ingress']},fraction_to_fail={rr.display(p['fraction'])},"
                           f"rotation_probability={rr.display(p['p'])} {ts}")
            if it < warm_up:
                continue
            r = it - warm_up
            ts = now()
            out.append(f"rmr{tags} rmr={rr.display(f['rmr'][r])},m={u['rmr_m'][r]},n={u['rmr_n'][r]} {ts}")
            out.append(f"coverage{tags} data={rr.display(f['coverage'][r])} {ts}")
            out.append(f"hops_stat{tags} mean={rr.display(f['hop_mean'][r])},median={rr.display(f['hop_median'][r])},"
                       f"max={u['hop_max'][r]} {ts}")
            out.append(f"stranded_node_stats{tags} count={u['stranded_round_count'][r]},"
                       f"mean={rr.display(f['stranded_round_mean'][r])},"
                       f"median={rr.display(f['stranded_round_median'][r])},max={u['stranded_round_max'][r]},"
                       f"min={u['stranded_round_min'][r]} {ts}")
            out.append(f"branching_factor{tags} data={rr.display(f['branching'][r])} {ts}")
            out.append(f"iteration{tags} gossip_iter={r},simulation_iter_val={k} {ts}")
        if len(f["coverage"]) == 0:
            continue
        ts = now()
        sf, su = f["stranded"], u["stranded"]
        out.append(f"stranded_node_iterations{tags} total_stranded={su[0]},mean_iter_stranded_per_node={rr.display(sf[0])},"
                   f"mean_stranded_per_iter={rr.display(sf[1])},mean_iter_stranded={rr.display(sf[2])},"
                   f"median_iter_stranded={rr.display(sf[3])},mean_weighted_stake={rr.display(sf[6])},"
                   f"median_weighted_stake={rr.display(sf[7])} {ts}")

        def hist(name, kv, upper, nb):  # Histogram::build geometry (gossip_stats.rs:575-593)
            rng = 1 if (upper == 0 or upper == 1) else upper // nb
            for i in range(0, len(kv) - 1, 2):
                bmax = (kv[i] + 1) * rng - 1
                out.append(f"{name} bucket={bmax},count={kv[i + 1]} {now()}")

        hist("stranded_node_histogram", u["stranded_hist"], measured, nb_stranded)
        hb = int(40.0 * (1.0 + p["fraction"])) if test_type == 5 else (50 if test_type == 2 else 30)
        hist("aggregate_hops_histogram", u["hops_hist"], hb, nb_hops)
        for d, name in (("egress_message_count", "egress_hist"), ("ingress_message_count", "ingress_hist"),
                        ("prune_message_count", "prune_hist")):
            kv = u[name]
            for i in range(0, len(kv) - 1, 2):
                out.append(f"{d},simulation_iter={k},start_time={start} bucket={kv[i]},count={kv[i + 1]} {now()}")
        out.append(f"iteration{tags} gossip_iter=0,simulation_iter_val={k} {ts}")
    return out
