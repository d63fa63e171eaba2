// gs_report.cpp -- the reference's end-of-run report (gossip_stats.rs print_* at
// 1315-1965, Display impls lib.rs:66-86 / gossip.rs:45-109) over the named result
// arrays of the engine, and the save / replay file of those arrays.
#include "gs_report.h"

#include <algorithm>
#include <charconv>
#include <cinttypes>
#include <cmath>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>

namespace gsrep {

const char* test_type_name(int t) {
  switch (t) {
    case ACTIVE_SET_SIZE: return "ActiveSetSize";
    case PUSH_FANOUT: return "PushFanout";
    case MIN_INGRESS_NODES: return "MinIngressNodes";
    case PRUNE_STAKE_THRESHOLD: return "PruneStakeThreshold";
    case ORIGIN_RANK: return "OriginRank";
    case FAIL_NODES: return "FailNodes";
    case ROTATE_PROBABILITY: return "RotateProbability";
    default: return "NoTest";
  }
}

int parse_test_type(const std::string& s) {
  if (s == "active-set-size") return ACTIVE_SET_SIZE;
  if (s == "push-fanout") return PUSH_FANOUT;
  if (s == "min-ingress-nodes") return MIN_INGRESS_NODES;
  if (s == "prune-stake-threshold") return PRUNE_STAKE_THRESHOLD;
  if (s == "origin-rank") return ORIGIN_RANK;
  if (s == "fail-nodes") return FAIL_NODES;
  if (s == "rotate-probability") return ROTATE_PROBABILITY;
  if (s == "no-test") return NO_TEST;
  return -1;
}

static std::string nonfinite(double x) {
  if (std::isnan(x)) return "NaN";
  return x < 0 ? "-inf" : "inf";
}

std::string rust_display(double x) {
  if (!std::isfinite(x)) return nonfinite(x);
  char b[400];
  auto r = std::to_chars(b, b + sizeof(b), x, std::chars_format::fixed);
  return std::string(b, r.ptr);
}

std::string rust_debug(double x) {
  if (!std::isfinite(x)) return nonfinite(x);
  const double a = std::fabs(x);
  char b[400];
  if ((a != 0.0 && a < 1e-4) || a >= 1e16) {  // float_to_exponential_common_shortest: "1e-5", "1.5e16"
    auto r = std::to_chars(b, b + sizeof(b), x, std::chars_format::scientific);
    std::string s(b, r.ptr);
    const size_t e = s.find('e');
    std::string mant = s.substr(0, e), ex = s.substr(e + 1);
    if (!ex.empty() && ex[0] == '+') ex = ex.substr(1);
    bool neg = !ex.empty() && ex[0] == '-';
    if (neg) ex = ex.substr(1);
    while (ex.size() > 1 && ex[0] == '0') ex = ex.substr(1);
    return mant + "e" + (neg ? "-" : "") + ex;
  }
  auto r = std::to_chars(b, b + sizeof(b), x, std::chars_format::fixed);
  std::string s(b, r.ptr);
  if (s.find('.') == std::string::npos) s += ".0";
  return s;
}

std::string rust_prec(double x, int prec) {
  if (!std::isfinite(x)) return nonfinite(x);
  char b[400];
  std::snprintf(b, sizeof(b), "%.*f", prec, x);
  return b;
}

static void log_rec(FILE* out, const char* level, const char* target, const std::string& msg) {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  tm t;
  gmtime_r(&ts.tv_sec, &t);
  char when[64];
  std::strftime(when, sizeof(when), "%Y-%m-%dT%H:%M:%S", &t);
  std::fprintf(out, "[%s.%09ldZ %-5s %s] %s\n", when, (long)ts.tv_nsec, level, target, msg.c_str());
}
void log_info(FILE* out, const char* target, const std::string& msg) { log_rec(out, "INFO", target, msg); }
void log_warn(FILE* out, const char* target, const std::string& msg) { log_rec(out, "WARN", target, msg); }

namespace {

const char* T = "gossip_sim::gossip_stats";

struct Printer {
  FILE* out;
  void operator()(const std::string& m) const { log_info(out, T, m); }
};

std::string u(uint64_t x) { return std::to_string(x); }

const std::vector<double>& F(const SimArrays& s, const char* n) {
  static const std::vector<double> none;
  auto it = s.f.find(n);
  return it == s.f.end() ? none : it->second;
}
const std::vector<uint64_t>& U(const SimArrays& s, const char* n) {
  static const std::vector<uint64_t> none;
  auto it = s.u.find(n);
  return it == s.u.end() ? none : it->second;
}
double f_at(const SimArrays& s, const char* n, size_t i) {
  const auto& v = F(s, n);
  return i < v.size() ? v[i] : 0.0;
}
uint64_t u_at(const SimArrays& s, const char* n, size_t i) {
  const auto& v = U(s, n);
  return i < v.size() ? v[i] : 0;
}

// StatCollection::print_stats (gossip_stats.rs:338-346) with Stats' Display (lib.rs:77-86)
void stat_collection(const Printer& P, const char* type, const std::vector<double>& v4) {
  const char* lab[4] = {"Mean", "Median", "Max", "Min"};
  for (int i = 0; i < 4; ++i)
    P(std::string(type) + " " + lab[i] + ": " + rust_prec(i < (int)v4.size() ? v4[i] : 0.0, 6));
}

// Histogram geometry of Histogram::build / build_from_map (gossip_stats.rs:575-666)
struct Geo {
  uint64_t min_entry, range, nb;
};
Geo build_geo(uint64_t upper, uint64_t lower, uint64_t nb) {
  const uint64_t range = (upper == lower || lower + 1 == upper) ? 1 : (nb ? (upper - lower) / nb : 0);
  return {lower, range, nb};
}
Geo map_geo(uint64_t max_entry, uint64_t nb) {
  const uint64_t range = (max_entry == 0 || max_entry + 1 == max_entry) ? 1 : (nb ? max_entry / nb : 0);
  return {0, range, nb};
}

// GossipStats::print_histogram (gossip_stats.rs:1351-1370): entries as (bucket, count) pairs
void histogram(const Printer& P, const std::string& type, const Geo& g, const std::vector<uint64_t>& kv) {
  P("|------------------------------------------------|");
  P("|---- " + type + " HISTOGRAM W/ " + u(g.nb) + " BUCKETS ----|");
  P("|------------------------------------------------|");
  for (size_t i = 0; i + 1 < kv.size(); i += 2) {
    const uint64_t b = kv[i], c = kv[i + 1];
    const uint64_t lo = g.min_entry + b * g.range;
    const uint64_t hi = g.min_entry + (b + 1) * g.range - 1;  // u64 wrapping, as in a release build
    if (lo == hi) P("Bucket: " + u(hi) + ": Count: " + u(c));
    else P("Bucket: " + u(lo) + "-" + u(hi) + ": Count: " + u(c));
  }
}

std::string params_debug(const SimParams& p) {
  std::string s = "SimulationParamaters {\n";
  s += "    gossip_push_fanout: " + u(p.gossip_push_fanout) + ",\n";
  s += "    gossip_active_set_size: " + u(p.gossip_active_set_size) + ",\n";
  s += "    gossip_iterations: " + u(p.gossip_iterations) + ",\n";
  s += "    origin_rank: " + u(p.origin_rank) + ",\n";
  s += "    probability_of_rotation: " + rust_debug(p.probability_of_rotation) + ",\n";
  s += "    prune_stake_threshold: " + rust_debug(p.prune_stake_threshold) + ",\n";
  s += "    min_ingress_nodes: " + u(p.min_ingress_nodes) + ",\n";
  s += "    fraction_to_fail: " + rust_debug(p.fraction_to_fail) + ",\n";
  s += "    when_to_fail: " + u(p.when_to_fail) + ",\n";
  s += std::string("    test_type: ") + test_type_name(p.test_type) + ",\n";
  s += "    num_simulations: " + u(p.num_simulations) + ",\n";
  if (p.step_size.is_int) s += "    step_size: Integer(\n        " + u(p.step_size.i) + ",\n    ),\n";
  else s += "    step_size: Float(\n        " + rust_debug(p.step_size.f) + ",\n    ),\n";
  s += "}";
  return s;
}

// GossipStats::print_all (gossip_stats.rs:1869-1883) of one simulation
void print_sim(const Printer& P, const ReportInput& in, size_t k) {
  const SimArrays& s = in.sims[k];
  const SimParams& prm = in.params[k];
  // print_coverage_stats
  P("|------------------------|");
  P("|---- COVERAGE STATS ----|");
  P("|------------------------|");
  stat_collection(P, "Coverage", F(s, "coverage_stats"));
  // print_rmr_stats
  P("|-------------------------------------------------|");
  P("|---- RELATIVE MESSAGE REDUNDANCY (RMR) STATS ----|");
  P("|-------------------------------------------------|");
  stat_collection(P, "RMR", F(s, "rmr_stats"));
  // print_aggregate_hop_stats (HopsStats' Display, lib.rs:66-75)
  P("|---------------------------------|");
  P("|------ AGGREGATE HOP STATS ------|");
  P("|---------------------------------|");
  P("Aggregate Hops Mean: " + rust_prec(f_at(s, "aggregate_hops", 0), 6));
  P("Aggregate Hops Median: " + rust_prec(f_at(s, "aggregate_hops", 1), 2));
  P("Aggregate Hops Max: " + u(u_at(s, "aggregate_hops", 0)));
  // print_aggregate_hops_stats_histogram: bounds of gossip_main.rs:573-587
  uint64_t hb = 30;  // STANDARD_HISTOGRAM_UPPER_BOUND
  if (in.test_type == FAIL_NODES) hb = (uint64_t)(40.0 * (1.0 + prm.fraction_to_fail));
  else if (in.test_type == MIN_INGRESS_NODES) hb = 50;
  histogram(P, "HOPS STATS", build_geo(hb, 0, in.nb_hops), U(s, "hops_hist"));
  // print_last_delivery_hop_stats
  P("|-------------------------------------|");
  P("|------ LAST DELIVERY HOP STATS ------|");
  P("|-------------------------------------|");
  P("LDH Mean: " + rust_prec(f_at(s, "ldh", 0), 6));
  P("LDH Median: " + rust_prec(f_at(s, "ldh", 1), 2));
  P("LDH Max: " + u(u_at(s, "ldh", 0)));
  P("LDH Min: " + u(u_at(s, "ldh", 1)));
  // print_stranded_stats (gossip_stats.rs:1625-1655)
  P("|-----------------------------|");
  P("|---- STRANDED NODE STATS ----|");
  P("|-----------------------------|");
  P("Total stranded node iterations -> SUM(stranded_node_iterations): " + u(u_at(s, "stranded", 0)));
  P("Mean number of iterations a gossip node was stranded for: " + rust_prec(f_at(s, "stranded", 0), 6));
  P("Mean number of nodes stranded during each gossip iteration: " + rust_prec(f_at(s, "stranded", 1), 6));
  P("Mean number of iterations a stranded node was stranded for: " + rust_prec(f_at(s, "stranded", 2), 6));
  P("Median number of iterations a stranded node was stranded for: " + rust_display(f_at(s, "stranded", 3)));
  P("Mean stake: " + rust_prec(f_at(s, "stranded", 4), 2));
  P("Median stake: " + rust_display(f_at(s, "stranded", 5)));
  P("Max stake: " + u(u_at(s, "stranded", 2)));
  P("Min stake: " + u(u_at(s, "stranded", 3)));
  P("Mean Weighted stake: " + rust_prec(f_at(s, "stranded", 6), 2));
  P("Median Weighted stake: " + rust_display(f_at(s, "stranded", 7)));
  // print_stranded_node_histogram: build(measured rounds, 0, num_buckets) (gossip_main.rs:568-572)
  const uint64_t measured = in.iterations > in.warm_up_rounds ? in.iterations - in.warm_up_rounds : 0;
  histogram(P, "STRANDED NODES", build_geo(measured, 0, in.nb_stranded), U(s, "stranded_hist"));
  // print_stranded (gossip_stats.rs:1555-1569): sorted by (times desc, stake desc); equal
  // (times, stake) pairs, in HashMap order in the reference, by ascending node id here
  const auto& st = U(s, "stranded_times");  // (node, times) pairs
  std::vector<std::pair<uint64_t, uint64_t>> nodes;
  for (size_t i = 0; i + 1 < st.size(); i += 2) nodes.push_back({st[i], st[i + 1]});
  std::stable_sort(nodes.begin(), nodes.end(), [&](const auto& a, const auto& b) {
    if (a.second != b.second) return a.second > b.second;
    const uint64_t sa = in.stakes[a.first], sb = in.stakes[b.first];
    if (sa != sb) return sa > sb;
    return a.first < b.first;
  });
  P("|----------------------------------------------------------|");
  P("|---- STRANDED NODES (Pubkey, stake, # times stranded) ----|");
  P("|----------------------------------------------------------|");
  P("Total stranded nodes: " + u(nodes.size()));
  for (auto& nd : nodes) {
    const uint64_t stake = in.stakes[nd.first];
    P(in.keys[nd.first] + ",\t" + u(stake) + (stake == 0 ? ",\t\t" : ",\t") + u(nd.second));
  }
  // print_failed_nodes (the node list itself is debug! output)
  P("|----------------------|");
  P("|---- FAILED NODES ----|");
  P("|----------------------|");
  P("Total Failed: " + u(u_at(s, "failed_count", 0)));
  // print_branching_factor_stats
  P("|-----------------------------------|");
  P("|---- OUTBOUND BRANCHING FACTOR ----|");
  P("|-----------------------------------|");
  stat_collection(P, "Outbound Branching Factor", F(s, "branching_stats"));
  // print_egress_message_histogram (gossip_stats.rs:1804-1816): build_from_map over stakes
  uint64_t max_stake = 0;
  for (uint64_t x : in.stakes) max_stake = std::max(max_stake, x);
  histogram(P, "EGRESS MESSAGES", map_geo(max_stake, in.nb_message), U(s, "egress_hist"));
  P("Bucket counts for Egress Messages");
  const auto& cpb = U(s, "egress_cpb");
  for (size_t i = 0; i < cpb.size(); ++i) P("bucket index, count: " + u(i) + ", " + u(cpb[i]));
}

}  // namespace

void print_all(FILE* out, const ReportInput& in) {
  const Printer P{out};
  const uint64_t measured = in.iterations - in.warm_up_rounds;  // usize subtraction of gossip_stats.rs:1948
  P("|----------------------------------------------------------|");
  P("|--- GOSSIP STATS COLLECTION ACROSS ALL " + u(in.num_simulations) + " SIMULATION(S) ---|");
  P("|--- Gossip Iterations: " + u(in.iterations) + " ");
  P("|--- Warm Up Rounds: " + u(in.warm_up_rounds));
  P("|--- Total Measured Rounds For Gossip Stats: " + u(measured));
  P(std::string("|--- Test Type: ") + test_type_name(in.test_type) + " ");
  P("|----------------------------------------------------------|");
  uint64_t total = 0;
  for (size_t k = 0; k < in.sims.size(); ++k) {
    P("|#######################################################################################|");
    P("Simulation Iteration: " + u(k) + ", Origin: " + in.keys[u_at(in.sims[k], "origin", 0)]);
    P(params_debug(in.params[k]));
    print_sim(P, in, k);
    total += u_at(in.sims[k], "stranded", 0);
  }
  P("Total stranded node iterations across all simulations " + u(total));
}

bool save_results(const std::string& path, const std::vector<SimArrays>& sims, std::string& err) {
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) {
    err = "cannot create " + path + ": " + std::strerror(errno);
    return false;
  }
  std::fprintf(f, "gossip-sim-results 1\nsims %zu\n", sims.size());
  for (size_t k = 0; k < sims.size(); ++k) {
    std::fprintf(f, "sim %zu\n", k);
    for (auto& kv : sims[k].f) {
      std::fprintf(f, "f %s %zu", kv.first.c_str(), kv.second.size());
      for (double x : kv.second) std::fprintf(f, " %a", x);
      std::fprintf(f, "\n");
    }
    for (auto& kv : sims[k].u) {
      std::fprintf(f, "u %s %zu", kv.first.c_str(), kv.second.size());
      for (uint64_t x : kv.second) std::fprintf(f, " %" PRIu64, x);
      std::fprintf(f, "\n");
    }
  }
  const bool ok = std::fclose(f) == 0;
  if (!ok) err = "write failed: " + path;
  return ok;
}

bool load_results(const std::string& path, std::vector<SimArrays>& sims, std::string& err) {
  std::ifstream f(path);
  if (!f) {
    err = "cannot open " + path;
    return false;
  }
  std::string tag;
  int ver = 0;
  size_t n = 0;
  if (!(f >> tag >> ver) || tag != "gossip-sim-results" || ver != 1) {
    err = path + ": not a gossip-sim results file";
    return false;
  }
  if (!(f >> tag >> n) || tag != "sims") {
    err = path + ": missing sims count";
    return false;
  }
  sims.assign(n, SimArrays());
  long cur = -1;
  while (f >> tag) {
    if (tag == "sim") {
      f >> cur;
      if (cur < 0 || (size_t)cur >= n) {
        err = path + ": sim index out of range";
        return false;
      }
      continue;
    }
    std::string name;
    size_t cnt = 0;
    if (cur < 0 || !(f >> name >> cnt) || (tag != "f" && tag != "u")) {
      err = path + ": malformed record";
      return false;
    }
    if (tag == "f") {
      auto& v = sims[cur].f[name];
      v.resize(cnt);
      for (size_t i = 0; i < cnt; ++i) {
        std::string x;
        f >> x;
        v[i] = std::strtod(x.c_str(), nullptr);
      }
    } else {
      auto& v = sims[cur].u[name];
      v.resize(cnt);
      for (size_t i = 0; i < cnt; ++i) f >> v[i];
    }
    if (!f) {
      err = path + ": truncated record " + name;
      return false;
    }
  }
  return true;
}

}  // namespace gsrep
