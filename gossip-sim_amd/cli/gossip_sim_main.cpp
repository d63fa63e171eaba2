// gossip_sim_main.cpp -- the `gossip-sim` driver (gossip_main.rs:53-981) on the HIP
// engine, plus `gossip-sim write-accounts` (write_accounts_main.rs:18-128).
//
// Same flags, defaults, validation and test-type sweeps as the reference. A sweep's
// simulations that share one active-set trajectory (no-test, origin-rank,
// min-ingress-nodes, prune-stake-threshold, fail-nodes) run as slots of ONE engine;
// engine-changing test types (active-set-size, push-fanout, rotate-probability) give
// each value its own engine. With --gpus K the simulations are dealt over K devices,
// one host thread and engine per device (results do not depend on the split: the
// Philox contract makes every slot a pure function of its own parameters).
//
// Offline stand-ins for the reference's network services: accounts come from the
// stake YAML (--accounts-from-yaml --account-file) or the deterministic synthetic
// network (--synthetic N) instead of an RPC pull; --influx other than `n` is refused.
// --save-results / --replay-results keep the named result arrays of a run in a text
// file and print the report from it again without a GPU.
#include <algorithm>
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/gossip_hip.h"
#include "gs_io.h"
#include "gs_report.h"

namespace {

const char* TMAIN = "gossip_sim";

const char* F64_NAMES[] = {"coverage", "rmr", "branching", "hop_mean", "hop_median", "coverage_stats", "rmr_stats",
                           "branching_stats", "aggregate_hops", "ldh", "stranded", "stranded_round_mean",
                           "stranded_round_median"};
const char* U64_NAMES[] = {"origin", "hop_max", "hop_min", "aggregate_hops", "ldh", "stranded", "stranded_times",
                           "stranded_round_count", "stranded_round_max", "stranded_round_min", "hops_hist",
                           "stranded_hist", "egress_hist", "ingress_hist", "prune_hist", "egress_cpb",
                           "validator_hist", "hist_errors", "failed_count", "rmr_m", "rmr_n"};

[[noreturn]] void die(int code, const std::string& msg) {
  std::fprintf(stderr, "error: %s\n", msg.c_str());
  std::exit(code);
}

bool parse_u64(const std::string& s, uint64_t& out) {
  if (s.empty() || s.find_first_not_of("0123456789") != std::string::npos) return false;
  errno = 0;
  char* end = nullptr;
  out = std::strtoull(s.c_str(), &end, 10);
  return errno == 0 && end && *end == 0;
}
bool parse_f64(const std::string& s, double& out) {
  if (s.empty()) return false;
  char* end = nullptr;
  out = std::strtod(s.c_str(), &end);
  return end && *end == 0;
}

struct Cli {
  std::string account_file, url = "https://api.mainnet-beta.solana.com", influx = "n", test_type_s;
  bool accounts_from_yaml = false, filter_zero = false, print_stats = false;
  uint64_t fanout = 6, asz = 12, iterations = 1, min_ingress = 2, nb_stranded = 10, nb_message = 5, nb_hops = 15;
  std::vector<uint64_t> origin_ranks = {1};
  std::string p_s = ".013333", thr_s = ".15", num_sims_s = "1", step_s = "1", frac_s = "0.1";
  uint64_t when_to_fail = 0, warm_up = 200;
  // engine / offline extensions
  uint64_t synthetic = 0, seed = 0x5EED0003ull, gpus = 1, bfs_mode = GS_BFS_AUTO;
  std::string save_results, replay_results;
  std::string influx_file;  // offline Influx line protocol (gs_influx.cpp)
  uint64_t influx_time_base = 0;
};

void usage() {
  std::puts(
      "gossip-sim: push-propagation gossip simulator (MI355X HIP engine)\n"
      "  --account-file PATH            yaml of accounts to read (with --accounts-from-yaml)\n"
      "  --accounts-from-yaml           read pubkey: stake pairs from --account-file\n"
      "  -f, --filter-zero-staked-nodes drop zero-staked nodes\n"
      "  --push-fanout N [6]  --active-set-size N [12]  --iterations N [1]\n"
      "  --origin-rank N... [1]  -p, --rotation-probability P [.013333]\n"
      "  --min-ingress-nodes N [2]  --prune-stake-threshold T [.15]\n"
      "  --num-buckets-stranded N [10]  --num-buckets-message N [5]  --num-buckets-hops N [15]\n"
      "  --test-type active-set-size|push-fanout|min-ingress-nodes|prune-stake-threshold|origin-rank|\n"
      "              rotate-probability|fail-nodes\n"
      "  --num-simulations N [1]  --step-size X [1]  --fraction-to-fail F [0.1]  --when-to-fail N [0]\n"
      "  --warm-up-rounds N [200]  --influx n  --print-stats  --url URL (no RPC offline)\n"
      "engine / offline options:\n"
      "  --synthetic N        the deterministic synthetic power-law network of N nodes instead of RPC\n"
      "  --seed S [0x5EED0003] --gpus K [1] --bfs-mode 0..5 [0 = auto; 1 workgroup, 2 level, 3 binned, 4 multi, 5 hybrid]\n"
      "  --save-results PATH  --replay-results PATH (print the report of a saved run, no GPU)\n"
      "  --influx-file PATH   write the Influx series (influx_db.rs) as line protocol to PATH\n"
      "  --influx-time-base NS  reproducible Influx timestamps NS + 1000 k (default: wall clock)\n"
      "gossip-sim write-accounts --account-file PATH --synthetic N [--num-nodes K] [--zero-stakes] [-f]");
}

Cli parse(int argc, char** argv) {
  Cli c;
  std::vector<std::string> args;  // "--flag=value" split into two tokens
  for (int i = 1; i < argc; ++i) {
    const std::string x = argv[i];
    const size_t eq = x.find('=');
    if (x.rfind("--", 0) == 0 && eq != std::string::npos) {
      args.push_back(x.substr(0, eq));
      args.push_back(x.substr(eq + 1));
    } else {
      args.push_back(x);
    }
  }
  const int n = (int)args.size();
  auto need = [&](int& i) -> std::string {
    if (i + 1 >= n) die(2, "missing value for " + args[i]);
    return args[++i];
  };
  auto u64 = [&](int& i, uint64_t& dst) {
    const std::string flag = args[i], v = need(i);
    if (!parse_u64(v, dst)) die(2, "invalid value '" + v + "' for " + flag);
  };
  for (int i = 0; i < n; ++i) {
    const std::string a = args[i];
    if (a == "-h" || a == "--help") { usage(); std::exit(0); }
    else if (a == "--url") c.url = need(i);
    else if (a == "--account-file") c.account_file = need(i);
    else if (a == "--accounts-from-yaml") c.accounts_from_yaml = true;
    else if (a == "-f" || a == "--filter-zero-staked-nodes") c.filter_zero = true;
    else if (a == "--push-fanout") u64(i, c.fanout);
    else if (a == "--active-set-size") u64(i, c.asz);
    else if (a == "--iterations") u64(i, c.iterations);
    else if (a == "--origin-rank") {
      c.origin_ranks.clear();
      while (i + 1 < n && args[i + 1][0] != '-') {
        uint64_t r = 0;
        if (!parse_u64(args[i + 1], r)) die(2, "invalid value '" + args[i + 1] + "' for --origin-rank");
        c.origin_ranks.push_back(r);
        ++i;
      }
      if (c.origin_ranks.empty()) die(2, "missing value for --origin-rank");
    } else if (a == "-p" || a == "--rotation-probability") c.p_s = need(i);
    else if (a == "--min-ingress-nodes") u64(i, c.min_ingress);
    else if (a == "--prune-stake-threshold") c.thr_s = need(i);
    else if (a == "--num-buckets-stranded") u64(i, c.nb_stranded);
    else if (a == "--num-buckets-message") u64(i, c.nb_message);
    else if (a == "--num-buckets-hops") u64(i, c.nb_hops);
    else if (a == "--test-type") c.test_type_s = need(i);
    else if (a == "--num-simulations") c.num_sims_s = need(i);
    else if (a == "--step-size") c.step_s = need(i);
    else if (a == "--fraction-to-fail") c.frac_s = need(i);
    else if (a == "--when-to-fail") u64(i, c.when_to_fail);
    else if (a == "--warm-up-rounds") u64(i, c.warm_up);
    else if (a == "--influx") c.influx = need(i);
    else if (a == "--print-stats") c.print_stats = true;
    else if (a == "--synthetic") u64(i, c.synthetic);
    else if (a == "--seed") {
      const std::string v = need(i);
      char* end = nullptr;
      c.seed = std::strtoull(v.c_str(), &end, 0);
      if (!end || *end) die(2, "invalid value '" + v + "' for --seed");
    } else if (a == "--gpus") u64(i, c.gpus);
    else if (a == "--bfs-mode") u64(i, c.bfs_mode);
    else if (a == "--save-results") c.save_results = need(i);
    else if (a == "--replay-results") c.replay_results = need(i);
    else if (a == "--influx-file") c.influx_file = need(i);
    else if (a == "--influx-time-base") u64(i, c.influx_time_base);
    else die(2, "unexpected argument '" + a + "' (see --help)");
  }
  return c;
}

// Accounts -> (keys, stakes) in id order (make_gossip_cluster gossip.rs:883-925).
void load_nodes(const Cli& c, std::vector<std::string>& keys, std::vector<uint64_t>& stakes) {
  std::vector<gsio::Account> acc;
  std::string err;
  if (c.accounts_from_yaml) {
    if (c.account_file.empty()) {
      gsrep::log_warn(stderr, TMAIN,
                      "Failed to pass in account file to read from with --accounts-from-yaml flag. need --acount-file <path>");
      std::exit(255);
    }
    gsrep::log_info(stderr, TMAIN, "Reading " + c.account_file);
    if (!gsio::read_stake_yaml(c.account_file, acc, err)) die(1, err);
    gsrep::log_info(stderr, TMAIN, std::to_string(acc.size()) + " accounts read in");
  } else if (c.synthetic) {
    acc = gsio::synthetic_network((uint32_t)c.synthetic);
  } else {
    die(1, "the RPC account pull (" + c.url + ") is not available offline: use --accounts-from-yaml "
           "--account-file PATH or --synthetic N");
  }
  std::vector<gsio::Account> kept;
  for (auto& a : acc) {
    if (c.filter_zero && a.stake == 0) continue;
    uint8_t pk[32];
    std::string why;
    if (!gsio::b58decode_pubkey(a.key, pk, &why)) die(1, "invalid pubkey '" + a.key + "': " + why);
    kept.push_back(a);
  }
  stakes = gsio::to_id_order(kept);
  keys.clear();
  for (auto& a : kept) keys.push_back(a.key);
}

struct Job {
  gs_sim_config cfg;
  int device = 0;
  std::vector<size_t> sims;  // global simulation indices
  std::vector<uint32_t> ranks, mi;
  std::vector<double> thr, frac;
};

void run_job(const Job& j, const std::vector<uint64_t>& stakes, std::vector<gsrep::SimArrays>& out,
             std::string& err) {
  gs_sim_config cfg = j.cfg;
  cfg.device = j.device;
  gs_sim_result* r = nullptr;
  const int rc = gs_run_simulations(&cfg, stakes.data(), (uint32_t)stakes.size(), (uint32_t)j.sims.size(),
                                    j.ranks.data(), j.mi.data(), j.thr.data(), j.frac.data(), &r);
  if (rc) {
    err = std::string("gs_run_simulations: ") + gs_last_error();
    return;
  }
  for (size_t k = 0; k < j.sims.size(); ++k) {
    gsrep::SimArrays& a = out[j.sims[k]];
    for (const char* nm : F64_NAMES) {
      const size_t n = gs_result_f64(r, (uint32_t)k, nm, nullptr, 0);
      if (n == SIZE_MAX) continue;
      a.f[nm].resize(n);
      gs_result_f64(r, (uint32_t)k, nm, a.f[nm].data(), n);
    }
    for (const char* nm : U64_NAMES) {
      const size_t n = gs_result_u64(r, (uint32_t)k, nm, nullptr, 0);
      if (n == SIZE_MAX) continue;
      a.u[nm].resize(n);
      gs_result_u64(r, (uint32_t)k, nm, a.u[nm].data(), n);
    }
  }
  gs_result_free(r);
}

int write_accounts_main(int argc, char** argv) {
  // write_accounts_main.rs:62-127 over the synthetic network (no RPC offline)
  std::string file;
  uint64_t num_nodes = UINT64_MAX, synthetic = 0;
  bool zero_only = false, filter_zero = false;
  for (int i = 2; i < argc; ++i) {
    const std::string a = argv[i];
    auto need = [&]() -> std::string {
      if (i + 1 >= argc) die(2, "missing value for " + a);
      return argv[++i];
    };
    if (a == "--account-file") file = need();
    else if (a == "--num-nodes") { if (!parse_u64(need(), num_nodes)) die(2, "invalid --num-nodes"); }
    else if (a == "--synthetic") { if (!parse_u64(need(), synthetic)) die(2, "invalid --synthetic"); }
    else if (a == "--zero-stakes") zero_only = true;
    else if (a == "-f" || a == "--filter-zero-staked-nodes") filter_zero = true;
    else if (a == "--url") need();
    else die(2, "unexpected argument '" + a + "'");
  }
  if (file.empty()) die(2, "--account-file PATH is required");
  if (!synthetic) die(1, "the RPC account pull is not available offline: pass --synthetic N");
  std::vector<gsio::Account> nodes = gsio::synthetic_network((uint32_t)synthetic), out;
  for (auto& n : nodes) {
    if (filter_zero && n.stake == 0) continue;
    if (zero_only && n.stake != 0) continue;
    out.push_back(n);
    if (out.size() > num_nodes - 1) break;
  }
  gsrep::log_info(stderr, "write_accounts", "Writing " + file);
  std::string err;
  if (!gsio::write_stake_yaml(file, out, err)) die(1, err);
  gsrep::log_info(stderr, "write_accounts", "Wrote " + std::to_string(out.size()) + " keys to file: " + file);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 1 && std::strcmp(argv[1], "write-accounts") == 0) return write_accounts_main(argc, argv);
  const Cli c = parse(argc, argv);
  const uint64_t start_ns = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(  // gossip_main.rs:724
                                std::chrono::system_clock::now().time_since_epoch()).count();

  // validators and value parsing of gossip_main.rs:120-148,248-252,655-704
  double p0 = 0, thr0 = 0, frac0 = 0;
  if (!parse_f64(c.p_s, p0) || !(p0 >= 0.0 && p0 <= 1.0))
    die(2, "active_set_rotation_probability must be between 0 and 1");
  if (!parse_f64(c.thr_s, thr0) || !(thr0 >= 0.0 && thr0 <= 1.0))
    die(2, "prune_stake_threshold must be between 0 and 1");
  if (!parse_f64(c.frac_s, frac0)) die(2, "invalid value '" + c.frac_s + "' for --fraction-to-fail");
  int test_type = gsrep::NO_TEST;
  if (!c.test_type_s.empty()) {
    test_type = gsrep::parse_test_type(c.test_type_s);
    if (test_type < 0) die(2, "Invalid test type");
  }
  uint64_t num_sims = 0;
  if (!parse_u64(c.num_sims_s, num_sims)) die(1, "Invalid num_simulations value");
  gsrep::StepSize step;
  if (!parse_u64(c.step_s, step.i)) {
    step.is_int = false;
    if (!parse_f64(c.step_s, step.f)) die(1, "Invalid step_size value");
  }
  if (c.influx != "n") die(1, "influx reporting over HTTP is not available offline (--influx n)");
  if (c.gpus < 1) die(2, "--gpus must be >= 1");

  if (c.origin_ranks.size() < num_sims) {
    gsrep::log_warn(stderr, TMAIN, "ERROR: not enough origin ranks provided for num_simulations! origin_ranks.len(): " +
                                       std::to_string(c.origin_ranks.size()) + ", num_simulations: " +
                                       std::to_string(num_sims));
    return 0;
  } else if (c.origin_ranks.size() > num_sims) {
    gsrep::log_warn(stderr, TMAIN, "WARNING: more origin ranks than number of simulations. Not going to hit all origin ranks");
  } else if (c.origin_ranks.size() > 1 && test_type != gsrep::ORIGIN_RANK) {
    gsrep::log_warn(stderr, TMAIN, "ERROR: multiple origin_ranks passed in but test type is not OriginRank. "
                                   "This would end up running all simulations with origin_rank[0]: " +
                                       std::to_string(c.origin_ranks[0]));
    return 0;
  }
  if (c.iterations <= c.warm_up)
    gsrep::log_warn(stderr, TMAIN, "WARNING: Gossip Iterations (" + std::to_string(c.iterations) + ") <= Warm Up Rounds (" +
                                       std::to_string(c.warm_up) + "). No stats will be recorded....");

  std::vector<std::string> keys;
  std::vector<uint64_t> stakes;
  load_nodes(c, keys, stakes);
  gsrep::log_info(stderr, "gossip_sim::gossip", "num of cluster nodes: " + std::to_string(stakes.size()));

  // per-simulation parameters (the test-type loops of gossip_main.rs:774-951)
  std::vector<gsrep::SimParams> params(num_sims);
  for (uint64_t i = 0; i < num_sims; ++i) {
    gsrep::SimParams& q = params[i];
    q.gossip_push_fanout = c.fanout;
    q.gossip_active_set_size = c.asz;
    q.gossip_iterations = c.iterations;
    q.origin_rank = c.origin_ranks[0];
    q.probability_of_rotation = p0;
    q.prune_stake_threshold = thr0;
    q.min_ingress_nodes = c.min_ingress;
    q.fraction_to_fail = frac0;
    q.when_to_fail = c.when_to_fail;
    q.test_type = test_type;
    q.num_simulations = num_sims;
    q.step_size = step;
    switch (test_type) {
      case gsrep::ACTIVE_SET_SIZE: q.gossip_active_set_size = c.asz + i * step.as_usize(); break;
      case gsrep::PUSH_FANOUT:
        q.gossip_push_fanout = c.fanout + i * step.as_usize();
        if (q.gossip_push_fanout > q.gossip_active_set_size) q.gossip_active_set_size = q.gossip_push_fanout;
        break;
      case gsrep::MIN_INGRESS_NODES: q.min_ingress_nodes = c.min_ingress + i * step.as_usize(); break;
      case gsrep::PRUNE_STAKE_THRESHOLD: q.prune_stake_threshold = thr0 + (double)i * step.as_f64(); break;
      case gsrep::ORIGIN_RANK: q.origin_rank = c.origin_ranks[i]; break;
      case gsrep::FAIL_NODES: q.fraction_to_fail = frac0 + (double)i * step.as_f64(); break;
      case gsrep::ROTATE_PROBABILITY: q.probability_of_rotation = p0 + (double)i * step.as_f64(); break;
      default: break;
    }
    if (stakes.size() < q.origin_rank)
      die(101, "ERROR: origin_rank larger than number of simulation nodes. nodes.len(): " + std::to_string(stakes.size()) +
                   ", origin_rank: " + std::to_string(q.origin_rank));
  }

  std::vector<gsrep::SimArrays> sims(num_sims);
  if (!c.replay_results.empty()) {
    std::string err;
    if (!gsrep::load_results(c.replay_results, sims, err)) die(1, err);
    if (sims.size() != num_sims) die(1, "results file holds " + std::to_string(sims.size()) + " simulations, not " +
                                            std::to_string(num_sims));
  } else if (num_sims) {
    // engines: sims sharing (fanout, active-set size, rotation probability) batch into one
    auto base_cfg = [&](const gsrep::SimParams& q) {
      gs_sim_config cfg{};
      cfg.push_fanout = (uint32_t)q.gossip_push_fanout;
      cfg.active_set_size = (uint32_t)q.gossip_active_set_size;
      cfg.iterations = (uint32_t)c.iterations;
      cfg.warm_up_rounds = (uint32_t)c.warm_up;
      cfg.min_ingress_nodes = (uint32_t)q.min_ingress_nodes;
      cfg.when_to_fail = (uint32_t)c.when_to_fail;
      cfg.rotation_probability = std::min(q.probability_of_rotation, 1.0);  // gen::<f64>() < p: p > 1 acts as 1
      cfg.prune_stake_threshold = q.prune_stake_threshold;
      cfg.fraction_to_fail = q.fraction_to_fail;
      cfg.num_buckets_stranded = c.nb_stranded;
      cfg.num_buckets_message = c.nb_message;
      cfg.num_buckets_hops = c.nb_hops;
      cfg.test_type = test_type;
      cfg.seed = c.seed;
      cfg.bfs_mode = (uint32_t)c.bfs_mode;
      return cfg;
    };
    const bool per_value_engine = test_type == gsrep::ACTIVE_SET_SIZE || test_type == gsrep::PUSH_FANOUT ||
                                  test_type == gsrep::ROTATE_PROBABILITY;
    std::vector<std::vector<size_t>> groups;
    if (per_value_engine) {
      for (size_t i = 0; i < num_sims; ++i) groups.push_back({i});
    } else {  // one batch, split into contiguous chunks over the devices
      const size_t K = std::min<size_t>(c.gpus, num_sims);
      for (size_t d = 0; d < K; ++d) {
        std::vector<size_t> g;
        for (size_t i = num_sims * d / K; i < num_sims * (d + 1) / K; ++i) g.push_back(i);
        groups.push_back(g);
      }
    }
    std::vector<Job> jobs;
    for (size_t gi = 0; gi < groups.size(); ++gi) {
      Job j;
      j.cfg = base_cfg(params[groups[gi][0]]);
      j.device = (int)(gi % c.gpus);
      j.sims = groups[gi];
      for (size_t i : groups[gi]) {
        j.ranks.push_back((uint32_t)params[i].origin_rank);
        j.mi.push_back((uint32_t)params[i].min_ingress_nodes);
        j.thr.push_back(params[i].prune_stake_threshold);
        j.frac.push_back(params[i].fraction_to_fail);
      }
      jobs.push_back(std::move(j));
    }
    for (size_t i = 0; i < num_sims; ++i)
      gsrep::log_info(stderr, TMAIN, "##### SIMULATION ITERATION: " + std::to_string(i) + " #####");
    // one worker thread per requested device; workers beyond the visible devices share
    // them (engines are independent), so the split itself runs on any box
    int ndev = 0;
    gs_device_count(&ndev);
    std::vector<std::string> errs(c.gpus);
    std::vector<std::thread> th;
    for (uint64_t d = 0; d < c.gpus; ++d)
      th.emplace_back([&, d]() {
        for (auto& j : jobs) {
          if ((uint64_t)j.device != d || !errs[d].empty()) continue;
          Job jj = j;
          jj.device = ndev > 0 ? (int)(d % (uint64_t)ndev) : 0;
          run_job(jj, stakes, sims, errs[d]);
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (!e.empty()) die(1, e);
    for (size_t i = 0; i < num_sims; ++i) {
      const auto& o = sims[i].u["origin"];
      if (!o.empty()) gsrep::log_info(stderr, TMAIN, "ORIGIN: " + keys[o[0]]);
    }
  }
  if (!c.save_results.empty()) {
    std::string err;
    if (!gsrep::save_results(c.save_results, sims, err)) die(1, err);
  }
  if (!c.influx_file.empty()) {  // the datapoint queue's text, in enqueue order (gossip_main.rs:372-645)
    gsrep::ReportInput in;
    in.keys = keys;
    in.stakes = stakes;
    in.iterations = c.iterations;
    in.warm_up_rounds = c.warm_up;
    in.num_simulations = num_sims;
    in.test_type = test_type;
    in.nb_stranded = c.nb_stranded;
    in.nb_message = c.nb_message;
    in.nb_hops = c.nb_hops;
    in.params = params;
    in.sims = sims;
    gsrep::InfluxOptions io;
    io.time_base = c.influx_time_base;
    io.start_time = std::to_string(c.influx_time_base ? c.influx_time_base : start_ns);
    io.api = c.accounts_from_yaml ? c.account_file : "synthetic:" + std::to_string(c.synthetic);
    if (num_sims) {
      const gsrep::SimParams& q = params[0];
      switch (test_type) {
        case gsrep::ACTIVE_SET_SIZE: io.start_value = (double)q.gossip_active_set_size; break;
        case gsrep::PUSH_FANOUT: io.start_value = (double)c.fanout; break;
        case gsrep::MIN_INGRESS_NODES: io.start_value = (double)q.min_ingress_nodes; break;
        case gsrep::PRUNE_STAKE_THRESHOLD: io.start_value = q.prune_stake_threshold; break;
        case gsrep::ORIGIN_RANK: io.start_value = (double)q.origin_rank; break;
        case gsrep::FAIL_NODES: io.start_value = q.fraction_to_fail; break;
        case gsrep::ROTATE_PROBABILITY: io.start_value = q.probability_of_rotation; break;
        default: break;
      }
    }
    FILE* f = std::fopen(c.influx_file.c_str(), "w");
    if (!f) die(1, "cannot write " + c.influx_file);
    gsrep::write_influx(f, in, io);
    std::fclose(f);
  }
  if (c.print_stats) {
    // GossipStatsCollection holds only simulations that recorded rounds (gossip_main.rs:567-593)
    gsrep::ReportInput in;
    in.keys = keys;
    in.stakes = stakes;
    in.iterations = c.iterations;
    in.warm_up_rounds = c.warm_up;
    in.num_simulations = num_sims;
    in.test_type = test_type;
    in.nb_stranded = c.nb_stranded;
    in.nb_message = c.nb_message;
    in.nb_hops = c.nb_hops;
    if (c.iterations > c.warm_up) {
      in.params = params;
      in.sims = sims;
    }
    if (!in.sims.empty()) gsrep::print_all(stderr, in);
    else gsrep::log_warn(stderr, TMAIN, "WARNING: Gossip Stats Collection is empty. Is `Iterations` <= `warm-up-rounds`?");
  }
  return 0;
}
