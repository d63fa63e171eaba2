// gs_influx.cpp -- the gossip-sim InfluxDB series (influx_db.rs:253-602) as an offline
// line-protocol file. The reference pushes each InfluxDataPoint's text to an HTTP
// /write endpoint from a queue thread (influx_db.rs:36-98,146-250); here the same text
// goes to a file, in the order gossip_main.rs:372-645 enqueues it:
//   simulation 0:  simulation_config + validator_stake_distribution        (:372-404)
//   each iteration: config every 10 iterations, before the round           (:425-447)
//   measured rounds: rmr, coverage, hops_stat, stranded_node_stats,
//                    branching_factor, iteration                           (:516-553)
//   after the rounds: stranded_node_iterations, stranded_node_histogram,
//                    aggregate_hops_histogram, egress/ingress/prune
//                    message counts, iteration(0, sim)                     (:595-642)
// Field values use Rust's Display for f64 (`{}`) and integers as the reference does.
// Timestamps: a data point's own timestamp is taken when it is created
// (InfluxDataPoint::new), histogram lines take a fresh one each
// (set_and_append_timestamp, which sleeps 1 us so that no two are equal). The clock
// is the wall clock in ns made strictly increasing by >= 1000 per reading, or, with a
// time base, base + 1000 * reading index (reproducible files for tests).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <string>

#include "gs_report.h"

namespace gsrep {

namespace {

struct Clock {
  uint64_t base = 0, last = 0, n = 0;
  uint64_t now() {
    uint64_t t;
    if (base) {
      t = base + 1000 * n;
    } else {
      t = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
              std::chrono::system_clock::now().time_since_epoch()).count();
      if (n && t < last + 1000) t = last + 1000;
    }
    ++n;
    last = t;
    return t;
  }
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
template <class T>
T at(const std::vector<T>& v, size_t i) { return i < v.size() ? v[i] : T(0); }

// InfluxDataPoint (influx_db.rs:253-345): text accumulated by the create_* calls
struct Point {
  Clock& clk;
  std::string data, start;
  size_t sim;
  uint64_t ts;
  Point(Clock& c, const std::string& start_ts, size_t sim_iter) : clk(c), start(start_ts), sim(sim_iter), ts(c.now()) {}
  void stamp() { data += u(ts) + "\n"; }                // append_timestamp
  void fresh_stamp() { data += u(clk.now()) + "\n"; }  // set_and_append_timestamp
  std::string tags() const { return ",simulation_iter=" + u(sim) + ",start_time=" + start; }
};

std::string step_display(const StepSize& s) { return s.is_int ? u(s.i) : rust_display(s.f); }

// Histogram geometry of Histogram::build (gossip_stats.rs:575-619): the bucket's upper bound
uint64_t bucket_max(uint64_t upper, uint64_t lower, uint64_t nb, uint64_t bucket) {
  const uint64_t range = (upper == lower || lower + 1 == upper) ? 1 : (nb ? (upper - lower) / nb : 0);
  return lower + (bucket + 1) * range - 1;  // u64 wrapping, as in a release build
}

}  // namespace

void write_influx(FILE* out, const ReportInput& in, const InfluxOptions& opt) {
  Clock clk;
  clk.base = opt.time_base;
  const std::string start = opt.start_time;
  auto emit = [&](const Point& p) { std::fwrite(p.data.data(), 1, p.data.size(), out); };
  const uint64_t measured = in.iterations > in.warm_up_rounds ? in.iterations - in.warm_up_rounds : 0;
  for (size_t k = 0; k < in.sims.size(); ++k) {
    const SimArrays& s = in.sims[k];
    const SimParams& prm = in.params[k];
    if (k == 0) {  // gossip_main.rs:372-404
      Point p(clk, start, k);
      p.data += "simulation_config,start_time=" + start + " num_simulations=" + u(in.num_simulations) +
                ",gossip_iterations_per_simulation=" + u(in.iterations) + ",warm_up_rounds=" + u(in.warm_up_rounds) +
                ",step_size=" + step_display(prm.step_size) + ",node_count=" + u(in.stakes.size()) +
                ",probability_of_rotation=" + rust_display(prm.probability_of_rotation) + ",api=\"" + opt.api +
                "\",start_value=\"" + (in.test_type == NO_TEST ? std::string("N/A") : rust_display(opt.start_value)) +
                "\",test_type=\"" + test_type_name(in.test_type) + "\" ";
      p.stamp();
      const auto& vh = U(s, "validator_hist");
      for (size_t i = 0; i + 1 < vh.size(); i += 2) {
        p.data += "validator_stake_distribution,start_time=" + start + " bucket=" + u(vh[i]) + ",count=" + u(vh[i + 1]) + " ";
        p.fresh_stamp();
      }
      emit(p);
    }
    { Point marker(clk, start, k); }  // the "start" marker point (influx_db.rs:290-303): not written
    const auto& cov = F(s, "coverage");
    const auto& rmr = F(s, "rmr");
    const auto& rm = U(s, "rmr_m");
    const auto& rn = U(s, "rmr_n");
    const auto& br = F(s, "branching");
    const auto& hmean = F(s, "hop_mean");
    const auto& hmed = F(s, "hop_median");
    const auto& hmax = U(s, "hop_max");
    const auto& scnt = U(s, "stranded_round_count");
    const auto& smean = F(s, "stranded_round_mean");
    const auto& smed = F(s, "stranded_round_median");
    const auto& smax = U(s, "stranded_round_max");
    const auto& smin = U(s, "stranded_round_min");
    for (uint64_t it = 0; it < in.iterations; ++it) {
      if (it % 10 == 0) {  // gossip_main.rs:426-447
        Point p(clk, start, k);
        p.data += "config" + p.tags() + " push_fanout=" + u(prm.gossip_push_fanout) + ",active_set_size=" +
                  u(prm.gossip_active_set_size) + ",origin_rank=" + u(prm.origin_rank) +
                  ",prune_stake_threshold=" + rust_display(prm.prune_stake_threshold) +
                  ",min_ingress_nodes=" + u(prm.min_ingress_nodes) + ",fraction_to_fail=" +
                  rust_display(prm.fraction_to_fail) + ",rotation_probability=" +
                  rust_display(prm.probability_of_rotation) + " ";
        p.stamp();
        emit(p);
      }
      if (it < in.warm_up_rounds) continue;
      const size_t r = it - in.warm_up_rounds;  // steady_state_iteration
      Point p(clk, start, k);
      if (r < rmr.size())  // Ok(..) of relative_message_redundancy
        p.data += "rmr" + p.tags() + " rmr=" + rust_display(rmr[r]) + ",m=" + u(at(rm, r)) + ",n=" + u(at(rn, r)) + " ";
      if (r < rmr.size()) p.stamp();
      p.data += "coverage" + p.tags() + " data=" + rust_display(at(cov, r)) + " ";
      p.stamp();
      p.data += "hops_stat" + p.tags() + " mean=" + rust_display(at(hmean, r)) + ",median=" + rust_display(at(hmed, r)) +
                ",max=" + u(at(hmax, r)) + " ";
      p.stamp();
      p.data += "stranded_node_stats" + p.tags() + " count=" + u(at(scnt, r)) + ",mean=" + rust_display(at(smean, r)) +
                ",median=" + rust_display(at(smed, r)) + ",max=" + u(at(smax, r)) + ",min=" + u(at(smin, r)) + " ";
      p.stamp();
      p.data += "branching_factor" + p.tags() + " data=" + rust_display(at(br, r)) + " ";
      p.stamp();
      p.data += "iteration" + p.tags() + " gossip_iter=" + u(r) + ",simulation_iter_val=" + u(k) + " ";
      p.stamp();
      emit(p);
    }
    if (cov.empty()) continue;  // stats.is_empty(): no measured rounds
    Point p(clk, start, k);
    p.data += "stranded_node_iterations" + p.tags() + " total_stranded=" + u(at(U(s, "stranded"), 0)) +
              ",mean_iter_stranded_per_node=" + rust_display(at(F(s, "stranded"), 0)) +
              ",mean_stranded_per_iter=" + rust_display(at(F(s, "stranded"), 1)) +
              ",mean_iter_stranded=" + rust_display(at(F(s, "stranded"), 2)) +
              ",median_iter_stranded=" + rust_display(at(F(s, "stranded"), 3)) +
              ",mean_weighted_stake=" + rust_display(at(F(s, "stranded"), 6)) +
              ",median_weighted_stake=" + rust_display(at(F(s, "stranded"), 7)) + " ";
    p.stamp();
    // create_histogram_point: "{type} bucket={bucket upper bound},count={count}" (no tags)
    auto hist = [&](const char* type, const std::vector<uint64_t>& kv, uint64_t upper, uint64_t nb) {
      for (size_t i = 0; i + 1 < kv.size(); i += 2) {
        p.data += std::string(type) + " bucket=" + u(bucket_max(upper, 0, nb, kv[i])) + ",count=" + u(kv[i + 1]) + " ";
        p.fresh_stamp();
      }
    };
    hist("stranded_node_histogram", U(s, "stranded_hist"), measured, in.nb_stranded);
    uint64_t hb = 30;  // aggregate hops histogram bounds (gossip_main.rs:573-587)
    if (in.test_type == FAIL_NODES) hb = (uint64_t)(40.0 * (1.0 + prm.fraction_to_fail));
    else if (in.test_type == MIN_INGRESS_NODES) hb = 50;
    hist("aggregate_hops_histogram", U(s, "hops_hist"), hb, in.nb_hops);
    // create_messages_point: raw bucket index, tags with the simulation index
    auto msgs = [&](const char* dir, const std::vector<uint64_t>& kv) {
      for (size_t i = 0; i + 1 < kv.size(); i += 2) {
        p.data += std::string(dir) + ",simulation_iter=" + u(k) + ",start_time=" + start + " bucket=" + u(kv[i]) +
                  ",count=" + u(kv[i + 1]) + " ";
        p.fresh_stamp();
      }
    };
    msgs("egress_message_count", U(s, "egress_hist"));
    msgs("ingress_message_count", U(s, "ingress_hist"));
    msgs("prune_message_count", U(s, "prune_hist"));
    p.data += "iteration" + p.tags() + " gossip_iter=0,simulation_iter_val=" + u(k) + " ";
    p.stamp();
    emit(p);
  }
}

}  // namespace gsrep
