// oracle/oracle_sim.cpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.h).
#include "oracle_sim.h"
#include <algorithm>
#include <queue>
#include <stdexcept>

namespace orc {

// ----------------------------------------------------------- Cluster ----
void Cluster::clear_maps() {  // gossip.rs:214-229
  visited.clear(); queue.clear(); distances.clear(); orders.clear(); mst.clear(); prunes.clear();
  pushes.clear(); rmr_m = 0; rmr_n = 0; rmr = 0.0; total_prunes = 0;
  egress_message_count.clear(); ingress_message_count.clear(); prune_messages_sent.clear();
}

void Cluster::run_gossip(const Pubkey& origin, const Stakes& stakes, const PkMap<Node*>& node_map) {
  // gossip.rs:483-615
  clear_maps();
  for (auto& kv : stakes) distances[kv.first] = UINT64_MAX;
  distances[origin] = 0;
  queue.push_back(origin);
  visited.insert(origin);
  rmr_n += 1;
  while (!queue.empty()) {
    Pubkey cur = queue.front();
    queue.pop_front();
    uint64_t cur_d = distances.at(cur);
    const Node* node = node_map.at(cur);
    pushes[cur] = PkSet{};
    egress_message_count[cur] = 0;
    std::vector<Pubkey> peers = node->active_set.get_nodes(cur, origin, stakes);
    size_t take = std::min(peers.size(), gossip_push_fanout);  // .take(fanout) before the failed check
    for (size_t i = 0; i < take; ++i) {
      const Pubkey& nb = peers[i];
      if (node_map.at(nb)->failed) continue;
      pushes[cur].insert(nb);
      egress_message_count[cur] += 1;
      ingress_message_count[nb] += 1;
      rmr_m += 1;
      if (!visited.count(nb)) {
        visited.insert(nb);
        distances[nb] = cur_d + 1;
        queue.push_back(nb);
        mst[cur].insert(nb);
        rmr_n += 1;
      }
      orders[nb][cur] = cur_d + 1;
    }
  }
}

void Cluster::consume_messages(const Pubkey& origin, std::vector<Node>& nodes,
                               const std::function<const std::string&(const Pubkey&)>& to_string) {
  // gossip.rs:618-653
  for (auto& node : nodes) {
    if (node.pk == origin) continue;
    auto it = orders.find(node.pk);
    if (it == orders.end()) continue;
    std::vector<std::pair<Pubkey, uint64_t>> sorted(it->second.begin(), it->second.end());
    std::sort(sorted.begin(), sorted.end(), [&](const auto& a, const auto& b) {
      if (a.second == b.second) return to_string(a.first) < to_string(b.first);
      return a.second < b.second;
    });
    for (size_t count = 0; count < sorted.size(); ++count)
      node.received_cache.record(origin, sorted[count].first, count);
  }
}

void Cluster::send_prunes(const Pubkey& origin, std::vector<Node>& nodes, double thr, size_t min_ingress,
                          const Stakes& stakes, const std::function<uint64_t(const Pubkey&)>& tie_rank) {
  // gossip.rs:657-697
  for (auto& node : nodes) {
    auto prunees = node.received_cache.prune(node.pk, origin, thr, min_ingress, stakes, tie_rank);
    PkMap<std::vector<Pubkey>> grouped;  // .zip(repeat(origin)).into_group_map()
    for (auto& p : prunees) grouped[p].push_back(origin);
    for (auto& kv : grouped) rmr_m += kv.second.size();
    prunes[node.pk] = std::move(grouped);
  }
}

void Cluster::prune_connections(const PkMap<Node*>& node_map, const Stakes& stakes) {
  // gossip.rs:701-737
  for (auto& kv : prunes) {
    const Pubkey& pruner = kv.first;
    if (!kv.second.empty()) total_prunes += kv.second.size();
    uint64_t& count = prune_messages_sent[pruner];
    for (auto& pe : kv.second) {
      auto it = node_map.find(pe.first);
      if (it == node_map.end()) throw std::runtime_error("prunee not in node_map");
      it->second->active_set.prune(pe.first, pruner, pe.second, stakes);
      count += pe.second.size();
    }
  }
}

std::pair<double, size_t> Cluster::coverage(const Stakes& stakes) const {  // gossip.rs:321-327
  return {(double)visited.size() / (double)stakes.size(), stakes.size() - visited.size()};
}

std::vector<Pubkey> Cluster::stranded_nodes() const {  // gossip.rs:329-345
  std::vector<Pubkey> out;
  for (auto& kv : distances)
    if (kv.second == UINT64_MAX && !failed_nodes.count(kv.first)) out.push_back(kv.first);
  return out;
}

bool Cluster::relative_message_redundancy(double* r, uint64_t* m, uint64_t* n) {
  if (rmr == 0.0) {
    if (rmr_n == 0) return false;
    rmr = (double)rmr_m / (double)(rmr_n - 1) - 1.0;
  }
  *r = rmr; *m = rmr_m; *n = rmr_n;
  return true;
}

// ------------------------------------------------------------- stats ----
HopsStat HopsStat::make(std::vector<uint64_t> hops) {  // gossip_stats.rs:47-98
  std::sort(hops.begin(), hops.end());
  std::vector<uint64_t> h;
  for (auto v : hops) if (v != UINT64_MAX && v != 0) h.push_back(v);
  HopsStat s;
  size_t count = h.size();
  uint64_t sum = 0;
  for (auto v : h) sum += v;
  s.mean = (double)sum / (double)count;
  if (count == 0) s.median = 0.0;
  else if (count == 1) s.median = (double)h[0];
  else if (count % 2 == 0) s.median = (double)(h[count / 2 - 1] + h[count / 2]) / 2.0;
  else s.median = (double)h[count / 2];
  s.max = count ? h.back() : 0;
  s.min = count ? h.front() : 0;
  return s;
}

void Histogram::build(uint64_t upper, uint64_t lower, uint64_t nb, const std::vector<uint64_t>& input) {
  min_entry = lower; max_entry = upper; num_buckets = nb;
  if (upper == lower || lower + 1 == upper) bucket_range = 1;
  else bucket_range = (upper - lower) / nb;
  entries.clear();
  for (uint64_t b = 0; b < nb; ++b) entries[b] = 0;
  for (auto e : input) {
    if (e >= min_entry && e <= max_entry) {
      if (bucket_range == 0) throw std::runtime_error("Histogram::build: bucket_range 0 (reference panics)");
      uint64_t b = (e - min_entry) / bucket_range;
      if (b == num_buckets) b -= 1;
      entries[b] += 1;
    } else {
      errors += 1;
    }
  }
}

bool Histogram::build_from_map(uint64_t nb, const PkMap<uint64_t>& input,
                               const std::vector<std::pair<Pubkey, uint64_t>>& sorted,
                               std::vector<uint64_t>& cpb) {
  min_entry = 0; max_entry = sorted[0].second; num_buckets = nb;
  if (max_entry == min_entry) bucket_range = 1;
  else bucket_range = (max_entry - min_entry) / nb;
  entries.clear();
  for (uint64_t b = 0; b < nb; ++b) entries[b] = 0;
  for (auto& kv : sorted) {
    uint64_t msgs = input.at(kv.first);
    if (kv.second >= min_entry && kv.second <= max_entry) {
      if (bucket_range == 0) return false;
      uint64_t b = (kv.second - min_entry) / bucket_range;
      if (b == num_buckets) b -= 1;
      entries[b] += msgs;
      if (b >= cpb.size()) return false;
      cpb[b] += 1;
    } else {
      errors += 1;
    }
  }
  return true;
}

void Histogram::normalize(const std::vector<uint64_t>& v) {
  for (auto& kv : entries) {
    uint64_t n = v.at(kv.first);
    if (n != 0) kv.second /= n;
  }
}

void StatCollection::calculate_stats() {  // gossip_stats.rs:266-295
  std::vector<double> s = collection;
  std::sort(s.begin(), s.end());
  size_t len = s.size();
  double sum = 0.0;
  for (double v : s) sum += v;
  mean = sum / (double)len;
  if (len == 0) median = std::nan("");
  else if (len % 2 == 0) median = (s[len / 2 - 1] + s[len / 2]) / 2.0;
  else median = s[len / 2];
  max = len ? s.back() : 0.0;
  min = len ? s.front() : 0.0;
}

StrandedNodeStats StrandedNodeStats::make(const std::vector<Pubkey>& stranded, const Stakes& stakes) {
  StrandedNodeStats r;
  if (stranded.empty()) return r;
  std::vector<uint64_t> st;
  for (auto& p : stranded) st.push_back(stakes.at(p));
  if (st.size() == 1) {
    r.count = 1; r.mean = (double)st[0]; r.median = (double)st[0]; r.max = st[0]; r.min = st[0];
    return r;
  }
  std::sort(st.begin(), st.end());
  size_t len = st.size();
  uint64_t sum = 0;
  for (auto v : st) sum += v;
  r.count = len;
  r.mean = (double)sum / (double)len;
  r.median = len % 2 == 0 ? (double)(st[len / 2 - 1] + st[len / 2]) / 2.0 : (double)st[len / 2];
  r.max = st.back();
  r.min = st.front();
  return r;
}

void StrandedNodeCollection::insert_nodes(const std::vector<Pubkey>& stranded, const Stakes& stakes) {
  per_iter.push_back(StrandedNodeStats::make(stranded, stakes));
  for (auto& p : stranded) {
    auto it = stranded_nodes.find(p);
    if (it != stranded_nodes.end()) it->second.second += 1;
    else {
      auto s = stakes.find(p);
      if (s != stakes.end()) stranded_nodes[p] = {s->second, 1};
    }
  }
  total_gossip_iterations += 1;
  if (total_nodes == 0) total_nodes = stakes.size();
}

static double median_u64(std::vector<uint64_t>& v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  size_t n = v.size();
  if (n % 2 == 0) return (double)(v[n / 2 - 1] + v[n / 2]) / 2.0;
  return (double)v[n / 2];
}

void StrandedNodeCollection::calculate_stats() {  // gossip_stats.rs:964-1038
  total_stranded_iterations = 0; total_stranded_stake = 0; weighted_total_stranded_stake = 0;
  std::vector<uint64_t> iters, stakes_v, weighted;
  for (auto& kv : stranded_nodes) {
    uint64_t stake = kv.second.first, times = kv.second.second;
    total_stranded_iterations += times;
    iters.push_back(times);
    total_stranded_stake += stake;
    weighted_total_stranded_stake += stake * times;
    stakes_v.push_back(stake);
    for (uint64_t t = 0; t < times; ++t) weighted.push_back(stake);
  }
  double count = (double)stranded_nodes.size();
  mean_stranded_per_iteration = (double)total_stranded_iterations / (double)total_gossip_iterations;
  mean_stake = (double)total_stranded_stake / count;
  mean_iters_per_stranded_node = (double)total_stranded_iterations / count;
  weighted_mean_stake = (double)weighted_total_stranded_stake / (double)total_stranded_iterations;
  median_iters_per_stranded_node = median_u64(iters);
  stranded_iterations_per_node = (double)total_stranded_iterations / (double)total_nodes;
  median_stake = median_u64(stakes_v);
  weighted_median_stake = median_u64(weighted);
  max_stake = stakes_v.empty() ? 0 : stakes_v.back();
  min_stake = stakes_v.empty() ? 0 : stakes_v.front();
}

void Tracker::init(const Stakes& stakes) {
  for (auto& kv : stakes) counts[kv.first] = 0;
}
void Tracker::update(const PkMap<uint64_t>& m) {
  for (auto& kv : m) counts.at(kv.first) += kv.second;
}
void Tracker::build(uint64_t nb, const Stakes& stakes, bool normalize) {
  std::vector<std::pair<Pubkey, uint64_t>> sv(stakes.begin(), stakes.end());
  std::stable_sort(sv.begin(), sv.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
  count_per_bucket.assign(nb, 0);
  ok = histogram.build_from_map(nb, counts, sv, count_per_bucket);
  if (ok && normalize) histogram.normalize(count_per_bucket);
}

void GossipStats::insert_hops_stat(const PkMap<uint64_t>& distances) {
  std::vector<uint64_t> v;
  for (auto& kv : distances) v.push_back(kv.second);
  per_round_hops.push_back(HopsStat::make(v));
  for (auto h : v) if (h != UINT64_MAX) raw_hops.push_back(h);
}

void GossipStats::calculate_branching(const PkMap<PkSet>& pushes) {  // gossip_stats.rs:1173-1191
  size_t total = pushes.size(), out = 0;
  for (auto& kv : pushes) out += kv.second.size();
  branching.collection.push_back(total ? (double)out / (double)total : 0.0);
}

void GossipStats::run_all_calculations() {  // gossip_stats.rs:1858-1867
  coverage.calculate_stats();
  rmr.calculate_stats();
  aggregate_hops = HopsStat::make(raw_hops);
  std::vector<uint64_t> maxes;
  for (auto& h : per_round_hops) maxes.push_back(h.max);
  ldh = HopsStat::make(maxes);
  stranded.calculate_stats();
  branching.calculate_stats();
}

// --------------------------------------------------------------- Sim ----
Sim::Sim(Mode m, uint64_t seed_, const std::vector<Pubkey>& pks, const std::vector<uint64_t>& st, size_t fanout)
    : mode(m), seed(seed_), cluster(fanout) {
  nodes.resize(pks.size());
  for (size_t i = 0; i < pks.size(); ++i) {
    nodes[i].pk = pks[i];
    nodes[i].stake = st[i];
    stakes[pks[i]] = st[i];
    index[pks[i]] = i;
    b58[pks[i]] = base58(pks[i]);
  }
  by_rank = pks;
  std::sort(by_rank.begin(), by_rank.end(), [&](const Pubkey& a, const Pubkey& b) { return b58[a] < b58[b]; });
  for (size_t r = 0; r < by_rank.size(); ++r) rank[by_rank[r]] = r;
}

PkMap<Node*> Sim::node_map() {
  PkMap<Node*> m;
  for (auto& n : nodes) m[n.pk] = &n;
  return m;
}

void Sim::rotate_node(Node& n, const std::function<Rng&(int)>& rng_for_k, size_t size, bool sort_by_pubkey) {
  // Node::rotate_active_set gossip.rs:815-842: candidates = stake keys minus self.
  std::vector<Pubkey> cand;
  cand.reserve(nodes.size());
  if (sort_by_pubkey) {
    for (auto& kv : stakes) if (kv.first != n.pk) cand.push_back(kv.first);
    std::sort(cand.begin(), cand.end());
  } else {
    for (auto& p : by_rank) if (p != n.pk) cand.push_back(p);
  }
  n.active_set.rotate(rng_for_k, size, cand, stakes);
}

void Sim::init_compat(Rng& rng, size_t asz) {
  std::vector<size_t> order(nodes.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return nodes[a].pk < nodes[b].pk; });
  for (size_t i : order) rotate_node(nodes[i], [&](int) -> Rng& { return rng; }, asz, true);
}

void Sim::init_philox(size_t asz) {
  for (auto& n : nodes) {
    uint32_t id = (uint32_t)rank.at(n.pk);
    std::vector<PhiloxStream> streams;
    for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k) streams.emplace_back(seed, P_INIT, id, (uint32_t)k);
    rotate_node(n, [&](int k) -> Rng& { return streams[k]; }, asz, false);
  }
}

void Sim::chance_to_rotate(size_t asz, double p, uint32_t round, Rng* compat_rng) {
  // gossip.rs:739-754 (the reference draws from StdRng::from_entropy per node).
  for (auto& n : nodes) {
    if (mode == COMPAT) {
      if (gen_f64(*compat_rng) < p) rotate_node(n, [&](int) -> Rng& { return *compat_rng; }, asz, true);
      continue;
    }
    uint32_t id = (uint32_t)rank.at(n.pk);
    PhiloxStream dec(seed, P_DECIDE, id, round);
    if (gen_f64(dec) < p) {
      std::vector<PhiloxStream> streams;
      for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k)
        streams.emplace_back(seed, P_ROTATE, id, (round << 5) | (uint32_t)k);
      rotate_node(n, [&](int k) -> Rng& { return streams[k]; }, asz, false);
    }
  }
}

size_t Sim::fail_nodes(double fraction) {  // gossip.rs:756-771
  size_t total = (size_t)(fraction * (double)nodes.size());
  if (fraction < 0 || std::isnan(fraction)) total = 0;
  if (total > nodes.size()) throw std::runtime_error("fail_nodes: more nodes than the cluster (reference panics)");
  std::vector<std::pair<uint64_t, uint64_t>> keys;  // (FAIL key, id)
  for (auto& n : nodes) {
    uint32_t id = (uint32_t)rank.at(n.pk);
    PhiloxStream s(seed, P_FAIL, id, 0);
    keys.push_back({s.next_u64(), id});
  }
  std::sort(keys.begin(), keys.end());
  for (size_t i = 0; i < total; ++i) {
    const Pubkey& pk = by_rank[keys[i].second];
    nodes[index.at(pk)].failed = true;
    cluster.failed_nodes.insert(pk);
  }
  return total;
}

const Node* Sim::find_nth_largest(size_t n) const {
  std::priority_queue<uint64_t, std::vector<uint64_t>, std::greater<uint64_t>> heap;  // min-heap
  for (auto& nd : nodes) {
    if (heap.size() < n) heap.push(nd.stake);
    else if (nd.stake >= heap.top()) { heap.pop(); heap.push(nd.stake); }
  }
  if (heap.empty()) return nullptr;
  uint64_t s = heap.top();
  for (auto& nd : nodes) if (nd.stake == s) return &nd;
  return nullptr;
}

void Sim::round_steps(const Pubkey& origin, double thr, size_t min_ingress, size_t asz, double p, uint32_t round,
                      Rng* compat_rng) {
  auto nm = node_map();
  cluster.run_gossip(origin, stakes, nm);
  cluster.consume_messages(origin, nodes, [&](const Pubkey& k) -> const std::string& { return b58.at(k); });
  cluster.send_prunes(origin, nodes, thr, min_ingress, stakes, [&](const Pubkey& k) { return rank.at(k); });
  cluster.prune_connections(nm, stakes);
  chance_to_rotate(asz, p, round, compat_rng);
}

void run_simulation(const SimConfig& cfg, const std::vector<Pubkey>& pks, const std::vector<uint64_t>& st,
                    GossipStats& stats, Pubkey* origin_out) {
  // gossip_main.rs:292-647 (PHILOX mode; influx and logging omitted)
  Sim sim(PHILOX, cfg.seed, pks, st, cfg.push_fanout);
  if (sim.nodes.size() < cfg.origin_rank) throw std::runtime_error("origin_rank larger than number of nodes");
  sim.init_philox(cfg.active_set_size);
  const Node* on = sim.find_nth_largest(cfg.origin_rank);
  Pubkey origin = on->pk;
  if (origin_out) *origin_out = origin;
  stats.egress.init(sim.stakes); stats.ingress.init(sim.stakes); stats.prune.init(sim.stakes);
  {
    std::vector<uint64_t> sv;
    for (auto& kv : sim.stakes) sv.push_back(kv.second);
    std::sort(sv.begin(), sv.end(), std::greater<uint64_t>());
    stats.validator_stake_distribution.build(sv[0], 0, 50, sv);
  }
  for (size_t it = 0; it < cfg.iterations; ++it) {
    if (cfg.test_type == 5 && it == cfg.when_to_fail) stats.failed_count = sim.fail_nodes(cfg.fraction_to_fail);
    sim.round_steps(origin, cfg.prune_stake_threshold, cfg.min_ingress_nodes, cfg.active_set_size,
                    cfg.rotation_probability, (uint32_t)it, nullptr);
    if (it >= cfg.warm_up_rounds) {
      auto cov = sim.cluster.coverage(sim.stakes);
      stats.coverage.collection.push_back(cov.first);
      stats.insert_hops_stat(sim.cluster.distances);
      stats.stranded.insert_nodes(sim.cluster.stranded_nodes(), sim.stakes);
      stats.calculate_branching(sim.cluster.pushes);
      stats.egress.update(sim.cluster.egress_message_count);
      stats.ingress.update(sim.cluster.ingress_message_count);
      stats.prune.update(sim.cluster.prune_messages_sent);
      double r; uint64_t m, n;
      if (sim.cluster.relative_message_redundancy(&r, &m, &n)) {
        stats.rmr.collection.push_back(r);
        stats.rmr_m.push_back(m);
        stats.rmr_n.push_back(n);
      }
    }
  }
  if (!stats.coverage.collection.empty()) {
    uint64_t measured = (uint64_t)(cfg.iterations - cfg.warm_up_rounds);
    std::vector<uint64_t> times;
    for (auto& kv : stats.stranded.stranded_nodes) times.push_back(kv.second.second);
    stats.stranded.histogram.build(measured, 0, cfg.num_buckets_stranded, times);
    uint64_t hb = 30;
    if (cfg.test_type == 5) hb = (uint64_t)(40.0 * (1.0 + cfg.fraction_to_fail));
    else if (cfg.test_type == 2) hb = 50;
    stats.hops_histogram.build(hb, 0, cfg.num_buckets_hops, stats.raw_hops);
    stats.egress.build(cfg.num_buckets_message, sim.stakes, true);
    stats.ingress.build(cfg.num_buckets_message, sim.stakes, true);
    stats.prune.build(cfg.num_buckets_message, sim.stakes, true);
    stats.run_all_calculations();
  }
}

}  // namespace orc
