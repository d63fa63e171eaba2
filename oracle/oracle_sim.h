// oracle/oracle_sim.h -- TEST INFRASTRUCTURE ONLY (see oracle_core.h).
// Restatement of gossip.rs Cluster/Node, gossip_stats.rs and the driver loop of
// gossip_main.rs. Keys are 32-byte pubkeys throughout, as in the reference.
#pragma once
#include "oracle_core.h"
#include <cmath>

namespace orc {

enum Mode { COMPAT = 0, PHILOX = 1 };

struct Node {  // gossip.rs:774-786 (table/receiver/clock carry no behaviour)
  Pubkey pk;
  uint64_t stake = 0;
  PushActiveSet active_set;
  ReceivedCache received_cache;
  bool failed = false;
};

struct Cluster {  // gossip.rs:135-190
  size_t gossip_push_fanout;
  PkSet visited;
  std::deque<Pubkey> queue;
  PkMap<uint64_t> distances;
  PkMap<PkMap<uint64_t>> orders;  // dest -> src -> hops
  PkMap<PkSet> mst;
  PkMap<PkSet> pushes;
  uint64_t rmr_m = 0, rmr_n = 0;
  double rmr = 0.0;
  PkMap<PkMap<std::vector<Pubkey>>> prunes;  // pruner -> prunee -> origins
  PkSet failed_nodes;
  size_t total_prunes = 0;
  PkMap<uint64_t> egress_message_count, ingress_message_count, prune_messages_sent;

  explicit Cluster(size_t fanout) : gossip_push_fanout(fanout) {}
  void clear_maps();
  void run_gossip(const Pubkey& origin, const Stakes& stakes, const PkMap<Node*>& node_map);
  void consume_messages(const Pubkey& origin, std::vector<Node>& nodes,
                        const std::function<const std::string&(const Pubkey&)>& to_string);
  void send_prunes(const Pubkey& origin, std::vector<Node>& nodes, double thr, size_t min_ingress,
                   const Stakes& stakes, const std::function<uint64_t(const Pubkey&)>& tie_rank);
  void prune_connections(const PkMap<Node*>& node_map, const Stakes& stakes);
  std::pair<double, size_t> coverage(const Stakes& stakes) const;
  std::vector<Pubkey> stranded_nodes() const;
  // relative_message_redundancy (gossip.rs:435-443 + gossip_stats.rs:511-521)
  bool relative_message_redundancy(double* rmr_out, uint64_t* m, uint64_t* n);
};

// ------------------------------------------------------------ stats ----
struct HopsStat {  // gossip_stats.rs:28-98
  double mean = 0.0, median = 0.0;
  uint64_t max = 0, min = 0;
  static HopsStat make(std::vector<uint64_t> hops);
};

struct Histogram {  // gossip_stats.rs:549-743
  std::map<uint64_t, uint64_t> entries;
  uint64_t min_entry = 0, max_entry = 0, bucket_range = 0, num_buckets = 0;
  int errors = 0;  // out-of-range entries the reference logs and drops
  void build(uint64_t upper, uint64_t lower, uint64_t nb, const std::vector<uint64_t>& input);
  // build_from_map with the stakes sorted largest first; returns false where the
  // reference would panic (count_per_bucket index out of range).
  bool build_from_map(uint64_t nb, const PkMap<uint64_t>& input,
                      const std::vector<std::pair<Pubkey, uint64_t>>& sorted_stakes,
                      std::vector<uint64_t>& count_per_bucket);
  void normalize(const std::vector<uint64_t>& v);
};

struct StatCollection {  // gossip_stats.rs:229-347
  std::vector<double> collection;
  double mean = 0.0, median = 0.0, max = 0.0, min = 0.0;
  void calculate_stats();
};

struct StrandedNodeStats {  // gossip_stats.rs:745-843
  size_t count = 0;
  double mean = 0.0, median = 0.0;
  uint64_t max = 0, min = 0;
  static StrandedNodeStats make(const std::vector<Pubkey>& stranded, const Stakes& stakes);
};

struct StrandedNodeCollection {  // gossip_stats.rs:846-1166
  std::vector<StrandedNodeStats> per_iter;
  PkMap<std::pair<uint64_t, uint64_t>> stranded_nodes;  // stake, times
  uint64_t total_gossip_iterations = 0, total_stranded_iterations = 0;
  double mean_stranded_per_iteration = 0, mean_iters_per_stranded_node = 0, median_iters_per_stranded_node = 0;
  double stranded_iterations_per_node = 0;
  size_t total_nodes = 0;
  uint64_t total_stranded_stake = 0;
  double mean_stake = 0, median_stake = 0;
  uint64_t max_stake = 0, min_stake = 0;
  uint64_t weighted_total_stranded_stake = 0;
  double weighted_mean_stake = 0, weighted_median_stake = 0;
  Histogram histogram;
  void insert_nodes(const std::vector<Pubkey>& stranded, const Stakes& stakes);
  void calculate_stats();
};

struct Tracker {  // EgressIngressMessageTracker gossip_stats.rs:359-461
  PkMap<uint64_t> counts;
  std::vector<uint64_t> count_per_bucket;
  Histogram histogram;
  bool ok = true;
  void init(const Stakes& stakes);
  void update(const PkMap<uint64_t>& m);
  void build(uint64_t nb, const Stakes& stakes, bool normalize);
};

struct GossipStats {  // gossip_stats.rs:1228-1884
  std::vector<HopsStat> per_round_hops;
  std::vector<uint64_t> raw_hops;
  HopsStat aggregate_hops, ldh;
  Histogram hops_histogram;
  StatCollection coverage, rmr, branching;
  std::vector<uint64_t> rmr_m, rmr_n;  // per measured round: the (m, n) of the rmr datapoint (influx_db.rs:346-360)
  StrandedNodeCollection stranded;
  Tracker egress, ingress, prune;
  Histogram validator_stake_distribution;
  size_t failed_count = 0;
  void insert_hops_stat(const PkMap<uint64_t>& distances);
  void calculate_branching(const PkMap<PkSet>& pushes);
  void run_all_calculations();
};

// ------------------------------------------------------------ sim ----
struct Sim {
  Mode mode;
  uint64_t seed;
  std::vector<Node> nodes;           // reference `nodes` Vec, in the caller's order
  Stakes stakes;
  PkMap<size_t> index;               // pubkey -> position in the caller's order
  PkMap<std::string> b58;            // cached Display strings (same result as to_string())
  PkMap<uint64_t> rank;              // base58-string rank: the node id of the build
  std::vector<Pubkey> by_rank;       // id -> pubkey
  Cluster cluster;
  Sim(Mode m, uint64_t seed, const std::vector<Pubkey>& pks, const std::vector<uint64_t>& stakes, size_t fanout);
  PkMap<Node*> node_map();
  // gossip_main.rs:263-277 / tests' run_gossip(test=true): COMPAT = shared rng, nodes
  // in Pubkey order, candidates sorted by Pubkey; PHILOX = INIT substream per (node, k),
  // candidates in id order.
  void init_compat(Rng& rng, size_t active_set_size);
  void init_philox(size_t active_set_size);
  void rotate_node(Node& n, const std::function<Rng&(int)>& rng_for_k, size_t size, bool sort_by_pubkey);
  void chance_to_rotate(size_t active_set_size, double p, uint32_t round, Rng* compat_rng);
  size_t fail_nodes(double fraction);  // PHILOX: smallest (FAIL key, id) first
  const Node* find_nth_largest(size_t n) const;  // gossip_main.rs:279-290 (ties: first in Vec order)
  void round_steps(const Pubkey& origin, double thr, size_t min_ingress, size_t asz, double p, uint32_t round,
                   Rng* compat_rng);
};

struct SimConfig {
  size_t push_fanout = 6, active_set_size = 12, iterations = 1, origin_rank = 1;
  double rotation_probability = 0.013333, prune_stake_threshold = 0.15;
  size_t min_ingress_nodes = 2;
  uint64_t num_buckets_stranded = 10, num_buckets_message = 5, num_buckets_hops = 15;
  double fraction_to_fail = 0.1;
  size_t when_to_fail = 0;
  int test_type = 0;  // 0 none, 5 fail-nodes, 2 min-ingress (affects hop histogram bound)
  size_t warm_up_rounds = 200;
  uint64_t seed = 0;
};

// run_simulation (gossip_main.rs:292-647) in PHILOX mode; fills stats.
void run_simulation(const SimConfig& cfg, const std::vector<Pubkey>& pks, const std::vector<uint64_t>& stakes,
                    GossipStats& stats, Pubkey* origin_out);

}  // namespace orc
