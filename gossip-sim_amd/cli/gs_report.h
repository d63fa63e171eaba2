// gs_report.h -- GossipStatsCollection::print_all (gossip_stats.rs:1869-1965) for the
// gossip-sim driver, and a text file of a run's named result arrays (save / replay).
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <vector>

namespace gsrep {

// Named arrays of one finished simulation: the names of gs_result_f64/u64.
struct SimArrays {
  std::map<std::string, std::vector<double>> f;
  std::map<std::string, std::vector<uint64_t>> u;
};

// Testing (gossip.rs:33-76), in gs_sim_config.test_type numbering.
enum TestType { NO_TEST = 0, ACTIVE_SET_SIZE = 1, MIN_INGRESS_NODES = 2, PUSH_FANOUT = 3, PRUNE_STAKE_THRESHOLD = 4,
                FAIL_NODES = 5, ORIGIN_RANK = 6, ROTATE_PROBABILITY = 7 };
const char* test_type_name(int t);          // Display: "ActiveSetSize", ...
int parse_test_type(const std::string& s);  // FromStr: "active-set-size", ...; -1 when invalid

// StepSize (gossip.rs:78-109): an integer when the flag parses as usize, else f64.
struct StepSize {
  bool is_int = true;
  uint64_t i = 1;
  double f = 1.0;
  uint64_t as_usize() const { return is_int ? i : (uint64_t)f; }
  double as_f64() const { return is_int ? (double)i : f; }
};

// SimulationParamaters (gossip_stats.rs:1193-1226) of one simulation.
struct SimParams {
  uint64_t gossip_push_fanout = 0, gossip_active_set_size = 0, gossip_iterations = 0, origin_rank = 0;
  double probability_of_rotation = 0, prune_stake_threshold = 0;
  uint64_t min_ingress_nodes = 0;
  double fraction_to_fail = 0;
  uint64_t when_to_fail = 0;
  int test_type = NO_TEST;
  uint64_t num_simulations = 0;
  StepSize step_size;
};

struct ReportInput {
  std::vector<std::string> keys;  // base58 pubkey by node id
  std::vector<uint64_t> stakes;   // stake by node id
  uint64_t iterations = 0, warm_up_rounds = 0, num_simulations = 0;
  int test_type = NO_TEST;
  uint64_t nb_stranded = 10, nb_message = 5, nb_hops = 15;
  std::vector<SimParams> params;  // per simulation
  std::vector<SimArrays> sims;    // per simulation
};

// Rust formatting of f64: Display `{}` (shortest round trip, no exponent),
// Debug `{:?}` (shortest, ".0" on integers, exponent below 1e-4 / from 1e16), `{:.N}`.
std::string rust_display(double x);
std::string rust_debug(double x);
std::string rust_prec(double x, int prec);

// One log record the way solana_logger / env_logger prints it: "[<UTC time> INFO  <target>] <msg>".
void log_info(FILE* out, const char* target, const std::string& msg);
void log_warn(FILE* out, const char* target, const std::string& msg);

// GossipStatsCollection::print_all(gossip_iterations, warm_up_rounds, test_type).
void print_all(FILE* out, const ReportInput& in);

// The InfluxDB series of influx_db.rs as an offline line-protocol file (gs_influx.cpp).
struct InfluxOptions {
  std::string start_time;   // start_time tag: the run's start in ns (gossip_main.rs:724)
  std::string api;          // simulation_config.api: where the accounts came from
  double start_value = 0;   // simulation_config.start_value: the swept parameter of simulation 0
  uint64_t time_base = 0;   // 0: wall clock; else timestamps base + 1000 * k (reproducible)
};
void write_influx(FILE* out, const ReportInput& in, const InfluxOptions& opt);

// Result arrays as text: hex-float f64 (exact), decimal u64.
bool save_results(const std::string& path, const std::vector<SimArrays>& sims, std::string& err);
bool load_results(const std::string& path, std::vector<SimArrays>& sims, std::string& err);

}  // namespace gsrep
