"""The gossip-sim driver (gossip-sim_amd/cli): flags and validation of gossip_main.rs,
stake YAML I/O (gossip_main.rs:304-318, write_accounts_main.rs), and the end-of-run
report (GossipStatsCollection::print_all) printed from result arrays.

CPU tests replay result arrays produced by the oracle (test infrastructure) through
the CLI's report printer and compare with report_ref.render, a line-by-line
restatement of the reference's print functions. The GPU test runs the CLI for real
and compares its saved arrays with the oracle's, bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

import engine_bind as eb
import oracle_bind as ob
import influx_ref as ir
import report_ref as rr

HERE = os.path.dirname(os.path.abspath(__file__))
CLI = os.path.join(HERE, "..", "gossip-sim_amd", "gossip-sim")
F64_NAMES = ["coverage", "rmr", "branching", "hop_mean", "hop_median", "coverage_stats", "rmr_stats",
             "branching_stats", "aggregate_hops", "ldh", "stranded", "stranded_round_mean", "stranded_round_median"]
U64_NAMES = ["origin", "hop_max", "hop_min", "aggregate_hops", "ldh", "stranded", "stranded_times",
             "stranded_round_count", "stranded_round_max", "stranded_round_min", "hops_hist", "stranded_hist",
             "egress_hist", "ingress_hist", "prune_hist", "egress_cpb", "validator_hist", "hist_errors",
             "failed_count", "rmr_m", "rmr_n"]


def cli(*args, check=True):
    r = subprocess.run([CLI, *map(str, args)], capture_output=True, text=True, timeout=600)
    if check and r.returncode != 0:
        raise AssertionError(f"gossip-sim {' '.join(map(str, args))} -> {r.returncode}\n{r.stderr[-3000:]}")
    return r


@pytest.fixture(scope="module")
def yaml_net(tmp_path_factory):
    """write-accounts of a 60-node synthetic network; (path, keys by id, stakes by id, pubkeys)."""
    d = tmp_path_factory.mktemp("acct")
    path = str(d / "accounts.yaml")
    cli("write-accounts", "--synthetic", 60, "--account-file", path)
    pks, st = eb.synth.network(60)
    keys = [eb.gs.b58encode(p) for p in pks]
    return path, keys, st, pks


def test_write_accounts_yaml_matches_synthetic_network(yaml_net):
    path, keys, st, _ = yaml_net
    text = open(path).read()
    assert text.startswith("---\n")
    rows = [ln.split(": ") for ln in text.strip().split("\n")[1:]]
    assert [k for k, _ in rows] == keys  # written sorted by base58 key = node id order
    np.testing.assert_array_equal(np.array([int(v) for _, v in rows], dtype=np.uint64), st)


def test_write_accounts_num_nodes_and_zero_stakes(tmp_path):
    p = str(tmp_path / "a.yaml")
    cli("write-accounts", "--synthetic", 40, "--num-nodes", 7, "--account-file", p)
    assert len(open(p).read().strip().split("\n")) == 1 + 7
    cli("write-accounts", "--synthetic", 40, "--zero-stakes", "--account-file", p)  # no zero stakes: empty map
    assert open(p).read().strip() == "---"


def test_flag_validation():
    r = cli("--synthetic", 20, "-p", "1.5", check=False)
    assert r.returncode == 2 and "active_set_rotation_probability must be between 0 and 1" in r.stderr
    r = cli("--synthetic", 20, "--prune-stake-threshold", "-0.1", check=False)
    assert r.returncode != 0
    r = cli("--synthetic", 20, "--test-type", "nope", check=False)
    assert r.returncode == 2 and "Invalid test type" in r.stderr
    r = cli("--synthetic", 20, "--step-size", "x", check=False)
    assert r.returncode == 1 and "Invalid step_size value" in r.stderr
    r = cli("--synthetic", 20, "--influx", "l", check=False)
    assert r.returncode == 1 and "not available offline" in r.stderr
    r = cli("--iterations", 5, check=False)  # no accounts source: the reference would pull from RPC
    assert r.returncode == 1 and "not available offline" in r.stderr
    r = cli("--accounts-from-yaml", check=False)
    assert "need --acount-file" in r.stderr


def test_yaml_errors(tmp_path):
    p = tmp_path / "bad.yaml"
    p.write_text("---\nnot-base58-0OIl: 5\n")
    r = cli("--accounts-from-yaml", "--account-file", str(p), "--replay-results", "/dev/null", check=False)
    assert r.returncode == 1 and "invalid pubkey" in r.stderr
    p.write_text("---\n11111111111111111111111111111111: 5\n11111111111111111111111111111111: 6\n")
    r = cli("--accounts-from-yaml", "--account-file", str(p), check=False)
    assert r.returncode == 1 and "duplicate key" in r.stderr
    p.write_text("---\n11111111111111111111111111111111: -5\n")
    r = cli("--accounts-from-yaml", "--account-file", str(p), check=False)
    assert r.returncode == 1 and "not a u64" in r.stderr


def test_origin_rank_checks(yaml_net):
    path = yaml_net[0]
    r = cli("--accounts-from-yaml", "--account-file", path, "--origin-rank", 1, 2, "--num-simulations", 3,
            check=False)
    assert r.returncode == 0 and "not enough origin ranks" in r.stderr
    r = cli("--accounts-from-yaml", "--account-file", path, "--origin-rank", 1, 2, "--num-simulations", 2,
            check=False)
    assert r.returncode == 0 and "test type is not OriginRank" in r.stderr


def oracle_sims(pks, st, params, *, seed):
    out = []
    for p in params:
        o = ob.run_simulation(pks, st, fanout=p["fanout"], asz=p["asz"], iterations=p["iterations"],
                              origin_rank=p["origin_rank"], p=p["p"], thr=p["thr"], min_ingress=p["min_ingress"],
                              fraction_to_fail=p["fraction"], when_to_fail=p["when_to_fail"],
                              test_type=p["test_type"], warm_up=p["warm_up"], seed=seed)
        out.append(({n: o.f64(n) for n in F64_NAMES}, {n: o.u64(n) for n in U64_NAMES}))
    return out


def sweep_params(test_type, n_sims, *, iterations, warm_up, step, ranks=(1,), fanout=6, asz=12, p=0.013333,
                 thr=0.15, mi=2, fraction=0.1, when=0):
    """Per-simulation parameters of the test-type loops (gossip_main.rs:774-951)."""
    out = []
    for i in range(n_sims):
        q = dict(fanout=fanout, asz=asz, iterations=iterations, origin_rank=ranks[0], p=p, thr=thr, min_ingress=mi,
                 fraction=fraction, when_to_fail=when, test_type=test_type, num_sims=n_sims, step_size=step,
                 warm_up=warm_up)
        if test_type == 1:  # gossip_main.rs:775-797
            q["asz"] = asz + i * int(step)
        elif test_type == 3:  # gossip_main.rs:798-825: the active set grows to the fanout
            q["fanout"] = fanout + i * int(step)
            if q["fanout"] > q["asz"]:
                q["asz"] = q["fanout"]
        elif test_type == 7:  # gossip_main.rs:915-937
            q["p"] = p + i * float(step)
        elif test_type == 6:
            q["origin_rank"] = ranks[i]
        elif test_type == 5:
            q["fraction"] = fraction + i * float(step)
        elif test_type == 4:
            q["thr"] = thr + i * float(step)
        elif test_type == 2:
            q["min_ingress"] = mi + i * int(step)
        out.append(q)
    return out


# gossip_main.rs:706-716 lets num_simulations > 1 through for a non-origin-rank test type
# only when MORE origin ranks than simulations are given (it warns and uses the first)
REPLAY_CASES = [
    ("no-test", 0, 1, 1, (1,), []),
    ("origin-rank", 6, 3, 1, (1, 5, 30), ["--origin-rank", 1, 5, 30]),
    ("fail-nodes", 5, 2, 0.2, (1,), ["--fraction-to-fail", 0.1, "--when-to-fail", 3, "--origin-rank", 1, 1, 1]),
    ("min-ingress-nodes", 2, 2, 1, (1,), ["--origin-rank", 1, 9, 9]),
    ("prune-stake-threshold", 4, 2, 0.25, (1,), ["--origin-rank", 1, 1, 1]),
    # the engine-changing sweeps: one engine (active-set trajectory) per value
    ("active-set-size", 1, 3, 2, (1,), ["--origin-rank", 1, 1, 1, 1]),
    ("push-fanout", 3, 3, 4, (1,), ["--origin-rank", 1, 1, 1, 1]),  # fanout 14 > 12 raises the set to 14
    ("rotate-probability", 7, 3, 0.25, (1,), ["--origin-rank", 1, 1, 1, 1]),
]
ENGINE_SWEEPS = REPLAY_CASES[5:]


@pytest.mark.parametrize("name,tt,n_sims,step,ranks,extra", REPLAY_CASES, ids=[c[0] for c in REPLAY_CASES])
def test_report_replay_matches_reference_format(yaml_net, tmp_path, name, tt, n_sims, step, ranks, extra):
    path, keys, st, pks = yaml_net
    iters, warm, seed = 36, 6, 77
    params = sweep_params(tt, n_sims, iterations=iters, warm_up=warm, step=step, ranks=ranks,
                          fraction=0.1, when=3 if tt == 5 else 0)
    sims = oracle_sims(pks, st, params, seed=seed)
    res = str(tmp_path / "r.txt")
    rr.write_results(res, sims)
    args = ["--accounts-from-yaml", "--account-file", path, "--iterations", iters, "--warm-up-rounds", warm,
            "--print-stats", "--replay-results", res, "--seed", seed]
    if tt:
        args += ["--test-type", name, "--num-simulations", n_sims, "--step-size", step]
    r = cli(*args, *extra)
    got = rr.report_lines(r.stderr)
    want = rr.render(keys, st, sims, params, iterations=iters, warm_up=warm, num_sims=n_sims, test_type=tt)
    assert got == want


@pytest.mark.parametrize("name,tt,n_sims,step,ranks,extra", REPLAY_CASES[:3], ids=[c[0] for c in REPLAY_CASES[:3]])
def test_influx_file_matches_reference_series(yaml_net, tmp_path, name, tt, n_sims, step, ranks, extra):
    """--influx-file writes influx_db.rs's data points (series, tags, fields, Rust float
    formatting, enqueue order of gossip_main.rs:372-645) as line protocol; with a time
    base the timestamps are reproducible and checked too."""
    path, keys, st, pks = yaml_net
    iters, warm, seed, base = 24, 4, 77, 1_700_000_000_000_000_000
    params = sweep_params(tt, n_sims, iterations=iters, warm_up=warm, step=step, ranks=ranks,
                          fraction=0.1, when=3 if tt == 5 else 0)
    sims = oracle_sims(pks, st, params, seed=seed)
    res, lp = str(tmp_path / "r.txt"), str(tmp_path / "influx.lp")
    rr.write_results(res, sims)
    args = ["--accounts-from-yaml", "--account-file", path, "--iterations", iters, "--warm-up-rounds", warm,
            "--replay-results", res, "--seed", seed, "--influx-file", lp, "--influx-time-base", base]
    if tt:
        args += ["--test-type", name, "--num-simulations", n_sims, "--step-size", step]
    cli(*args, *extra)
    got = open(lp).read().splitlines()
    want = ir.render(len(st), sims, params, iterations=iters, warm_up=warm, num_sims=n_sims, test_type=tt,
                     step=step, api=path, base=base)
    assert got == want
    assert got[0].startswith("simulation_config,") and got[-1].startswith("iteration,")


def test_influx_http_refused(yaml_net):
    r = cli("--accounts-from-yaml", "--account-file", yaml_net[0], "--influx", "l", check=False)
    assert r.returncode == 1 and "not available offline" in r.stderr


def test_report_empty_collection_warns(yaml_net, tmp_path):
    res = str(tmp_path / "r.txt")
    rr.write_results(res, [({}, {})])
    r = cli("--accounts-from-yaml", "--account-file", yaml_net[0], "--iterations", 5, "--warm-up-rounds", 5,
            "--print-stats", "--replay-results", res)
    assert "Gossip Stats Collection is empty" in r.stderr


def test_rust_float_formatting():
    assert rr.display(1.0) == "1" and rr.display(0.1 + 0.2) == "0.30000000000000004"
    assert rr.debug(1.0) == "1.0" and rr.debug(0.15) == "0.15" and rr.debug(1e-7) == "1e-7"
    assert rr.debug(1e16) == "1e16" and rr.debug(0.013333) == "0.013333"
    assert rr.display(724161057685112.0) == "724161057685112"


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [1, 2])
def test_cli_run_matches_oracle(yaml_net, tmp_path, gpus):
    """gossip-sim on the GPU: an origin-rank sweep's result arrays equal the oracle's bit
    for bit, and its report equals the reference-format rendering of the oracle arrays.
    --gpus 2 deals the sims to two workers (two engines; on a one-GPU box both on it)."""
    path, keys, st, pks = yaml_net
    iters, warm, seed = 40, 8, 5
    params = sweep_params(6, 3, iterations=iters, warm_up=warm, step=1, ranks=(1, 4, 22), p=0.05)
    res = str(tmp_path / "g.txt")
    r = cli("--accounts-from-yaml", "--account-file", path, "--iterations", iters, "--warm-up-rounds", warm,
            "-p", 0.05, "--test-type", "origin-rank", "--num-simulations", 3, "--origin-rank", 1, 4, 22,
            "--print-stats", "--save-results", res, "--seed", seed, "--gpus", gpus)
    got = rr.read_results(res)
    want = oracle_sims(pks, st, params, seed=seed)
    for k, ((gf, gu), (wf, wu)) in enumerate(zip(got, want)):
        for n in F64_NAMES:
            np.testing.assert_array_equal(gf[n], wf[n], err_msg=f"sim {k} {n}")
        for n in U64_NAMES:
            np.testing.assert_array_equal(gu[n], wu[n], err_msg=f"sim {k} {n}")
    assert rr.report_lines(r.stderr) == rr.render(keys, st, want, params, iterations=iters, warm_up=warm,
                                                  num_sims=3, test_type=6)


@pytest.mark.gpu
@pytest.mark.parametrize("name,tt,n_sims,step,ranks,extra", ENGINE_SWEEPS, ids=[c[0] for c in ENGINE_SWEEPS])
def test_cli_engine_sweeps_match_oracle(yaml_net, tmp_path, name, tt, n_sims, step, ranks, extra):
    """The sweeps that change the engine itself (gossip_main.rs:775-825,915-937): the
    active-set size, the push fanout (with its raise of the active-set size to the fanout,
    :809-811) and the rotation probability. The CLI runs one engine per value on the GPU;
    every sim's result arrays equal the oracle's run_simulation with that value, and the
    report equals the reference-format rendering."""
    path, keys, st, pks = yaml_net
    iters, warm, seed = 34, 6, 13
    params = sweep_params(tt, n_sims, iterations=iters, warm_up=warm, step=step, ranks=ranks)
    res = str(tmp_path / "g.txt")
    r = cli("--accounts-from-yaml", "--account-file", path, "--iterations", iters, "--warm-up-rounds", warm,
            "--test-type", name, "--num-simulations", n_sims, "--step-size", step, *extra,
            "--print-stats", "--save-results", res, "--seed", seed, "--gpus", 2)
    got = rr.read_results(res)
    want = oracle_sims(pks, st, params, seed=seed)
    for k, ((gf, gu), (wf, wu)) in enumerate(zip(got, want)):
        for n in F64_NAMES:
            np.testing.assert_array_equal(gf[n], wf[n], err_msg=f"{name} sim {k} {n}")
        for n in U64_NAMES:
            np.testing.assert_array_equal(gu[n], wu[n], err_msg=f"{name} sim {k} {n}")
    assert rr.report_lines(r.stderr) == rr.render(keys, st, want, params, iterations=iters, warm_up=warm,
                                                  num_sims=n_sims, test_type=tt)
