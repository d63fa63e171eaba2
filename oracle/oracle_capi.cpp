// oracle/oracle_capi.cpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.h).
// Flat C entry points so pytest (ctypes) can drive the CPU restatement. Nodes
// are addressed by their index in the pubkey array the caller passed in.
#include "oracle_sim.h"
#include <algorithm>
#include <chrono>
#include <stdexcept>
#include <thread>
#include <string>

using namespace orc;

namespace {
Pubkey pk_at(const uint8_t* p, size_t i = 0) {
  Pubkey k;
  std::memcpy(k.b, p + 32 * i, 32);
  return k;
}
std::vector<Pubkey> pk_vec(const uint8_t* p, size_t n) {
  std::vector<Pubkey> v(n);
  for (size_t i = 0; i < n; ++i) v[i] = pk_at(p, i);
  return v;
}
size_t put_pks(const std::vector<Pubkey>& v, uint8_t* out, size_t cap) {
  for (size_t i = 0; i < v.size() && i < cap; ++i) std::memcpy(out + 32 * i, v[i].b, 32);
  return v.size();
}
thread_local std::string g_err;

struct StatsHandle {
  GossipStats st;
  size_t origin_index = 0;
  PkMap<size_t> index;  // for per-node outputs
};

size_t put_f(const std::vector<double>& v, double* out, size_t cap) {
  for (size_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
  return v.size();
}
size_t put_u(const std::vector<uint64_t>& v, uint64_t* out, size_t cap) {
  for (size_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
  return v.size();
}
std::vector<uint64_t> hist_kv(const Histogram& h) {
  std::vector<uint64_t> v;
  for (auto& kv : h.entries) { v.push_back(kv.first); v.push_back(kv.second); }
  return v;
}
}  // namespace

extern "C" {

const char* or_last_error() { return g_err.c_str(); }

// ------------------------------------------------------------- RNG ----
void* or_chacha_new(const uint8_t* seed) { return new ChaCha20Rng(seed); }
void* or_philox_stream_new(uint64_t seed, uint32_t purpose, uint32_t a, uint32_t b) {
  return new PhiloxStream(seed, purpose, a, b);
}
void or_rng_free(void* r) { delete (Rng*)r; }
uint64_t or_rng_next_u64(void* r) { return ((Rng*)r)->next_u64(); }
uint64_t or_gen_range(void* r, uint64_t lo, uint64_t hi) { return sample_single_u64(lo, hi, *(Rng*)r); }
double or_gen_f64(void* r) { return gen_f64(*(Rng*)r); }
void or_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) { philox4x32_10(ctr, key, out); }
int or_base58(const uint8_t* pk, char* out) {
  std::string s = base58(pk_at(pk));
  std::memcpy(out, s.c_str(), s.size() + 1);
  return (int)s.size();
}
void or_pubkey_from_counter(uint64_t i, uint8_t* out) { std::memcpy(out, pubkey_from_counter(i).b, 32); }
int or_stake_bucket(uint64_t stake, int has) { return get_stake_bucket(has ? &stake : nullptr); }

void* or_stakes_new(const uint8_t* pks, const uint64_t* vals, size_t n) {
  auto* s = new Stakes();
  for (size_t i = 0; i < n; ++i) (*s)[pk_at(pks, i)] = vals[i];
  return s;
}
void or_stakes_free(void* s) { delete (Stakes*)s; }

// ------------------------------------------------ PushActiveSetEntry ----
void* or_entry_new() { return new PushActiveSetEntry(); }
void or_entry_free(void* e) { delete (PushActiveSetEntry*)e; }
void or_entry_rotate(void* e, void* rng, size_t size, const uint8_t* nodes, const uint64_t* weights, size_t n) {
  std::vector<uint64_t> w(weights, weights + n);
  ((PushActiveSetEntry*)e)->rotate(*(Rng*)rng, size, pk_vec(nodes, n), w);
}
size_t or_entry_keys(void* e, uint8_t* out, size_t cap) { return put_pks(((PushActiveSetEntry*)e)->keys, out, cap); }
size_t or_entry_get_nodes(void* e, const uint8_t* origin, int force, uint8_t* out, size_t cap) {
  auto v = ((PushActiveSetEntry*)e)->get_nodes(pk_at(origin), [&](const Pubkey&) { return force != 0; });
  return put_pks(v, out, cap);
}
void or_entry_prune(void* e, const uint8_t* node, const uint8_t* origin) {
  ((PushActiveSetEntry*)e)->prune(pk_at(node), pk_at(origin));
}
int or_entry_filter_contains(void* e, const uint8_t* node, const uint8_t* key) {
  auto* en = (PushActiveSetEntry*)e;
  const long i = en->index_of(pk_at(node));
  if (i < 0) return -1;
  return en->filter_contains((size_t)i, pk_at(key)) ? 1 : 0;
}

// ------------------------------------------------------ PushActiveSet ----
void* or_pas_new() { return new PushActiveSet(); }
void or_pas_free(void* p) { delete (PushActiveSet*)p; }
void or_pas_rotate(void* p, void* rng, size_t size, const uint8_t* nodes, size_t n, void* stakes) {
  ((PushActiveSet*)p)->rotate([&](int) -> Rng& { return *(Rng*)rng; }, size, pk_vec(nodes, n), *(Stakes*)stakes);
}
size_t or_pas_get_nodes(void* p, const uint8_t* self, const uint8_t* origin, void* stakes, uint8_t* out, size_t cap) {
  return put_pks(((PushActiveSet*)p)->get_nodes(pk_at(self), pk_at(origin), *(Stakes*)stakes), out, cap);
}
void or_pas_prune(void* p, const uint8_t* self, const uint8_t* node, const uint8_t* origins, size_t no, void* stakes) {
  ((PushActiveSet*)p)->prune(pk_at(self), pk_at(node), pk_vec(origins, no), *(Stakes*)stakes);
}
size_t or_pas_entry_keys(void* p, int k, uint8_t* out, size_t cap) {
  return put_pks(((PushActiveSet*)p)->e[k].keys, out, cap);
}
int or_pas_filter_contains(void* p, int k, const uint8_t* node, const uint8_t* key) {
  return or_entry_filter_contains(&((PushActiveSet*)p)->e[k], node, key);
}

// ------------------------------------------------------ ReceivedCache ----
void* or_rc_new() { return new ReceivedCache(); }
void or_rc_free(void* r) { delete (ReceivedCache*)r; }
void* or_rc_clone(void* r) { return new ReceivedCache(*(ReceivedCache*)r); }
void or_rc_record(void* r, const uint8_t* origin, const uint8_t* node, size_t dups) {
  ((ReceivedCache*)r)->record(pk_at(origin), pk_at(node), dups);
}
long or_rc_entry(void* r, const uint8_t* origin, uint64_t* upserts, uint8_t* nodes, uint64_t* scores, size_t cap) {
  auto* rc = (ReceivedCache*)r;
  auto it = rc->m.find(pk_at(origin));
  if (it == rc->m.end()) return -1;
  *upserts = it->second.num_upserts;
  std::vector<std::pair<Pubkey, uint64_t>> v(it->second.nodes.begin(), it->second.nodes.end());
  std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first < b.first; });
  for (size_t i = 0; i < v.size() && i < cap; ++i) {
    std::memcpy(nodes + 32 * i, v[i].first.b, 32);
    scores[i] = v[i].second;
  }
  return (long)v.size();
}
size_t or_rc_prune(void* r, const uint8_t* self, const uint8_t* origin, double thr, size_t min_ingress, void* stakes,
                   uint8_t* out, size_t cap) {
  auto v = ((ReceivedCache*)r)->prune(pk_at(self), pk_at(origin), thr, min_ingress, *(Stakes*)stakes,
                                      [](const Pubkey& k) { return (uint64_t)0 * k.b[0]; });
  return put_pks(v, out, cap);
}

// ---------------------------------------------------------------- Sim ----
void* or_sim_new(int mode, uint64_t seed, const uint8_t* pks, const uint64_t* stakes, size_t n, size_t fanout) {
  return new Sim((Mode)mode, seed, pk_vec(pks, n), std::vector<uint64_t>(stakes, stakes + n), fanout);
}
void or_sim_free(void* s) { delete (Sim*)s; }
void or_sim_init_compat(void* s, void* rng, size_t asz) { ((Sim*)s)->init_compat(*(Rng*)rng, asz); }
void or_sim_init_philox(void* s, size_t asz) { ((Sim*)s)->init_philox(asz); }
void or_sim_run_gossip(void* sp, size_t origin) {
  Sim* s = (Sim*)sp;
  auto nm = s->node_map();
  s->cluster.run_gossip(s->nodes[origin].pk, s->stakes, nm);
}
void or_sim_consume(void* sp, size_t origin) {
  Sim* s = (Sim*)sp;
  s->cluster.consume_messages(s->nodes[origin].pk, s->nodes,
                              [&](const Pubkey& k) -> const std::string& { return s->b58.at(k); });
}
void or_sim_send_prunes(void* sp, size_t origin, double thr, size_t min_ingress) {
  Sim* s = (Sim*)sp;
  s->cluster.send_prunes(s->nodes[origin].pk, s->nodes, thr, min_ingress, s->stakes,
                         [&](const Pubkey& k) { return s->rank.at(k); });
}
void or_sim_prune_connections(void* sp) {
  Sim* s = (Sim*)sp;
  auto nm = s->node_map();
  s->cluster.prune_connections(nm, s->stakes);
}
void or_sim_chance_to_rotate(void* s, size_t asz, double p, uint32_t round, void* compat_rng) {
  ((Sim*)s)->chance_to_rotate(asz, p, round, (Rng*)compat_rng);
}
long or_sim_fail_nodes(void* s, double f) {
  try { return (long)((Sim*)s)->fail_nodes(f); } catch (std::exception& e) { g_err = e.what(); return -1; }
}
size_t or_sim_find_nth_largest(void* sp, size_t n) {
  Sim* s = (Sim*)sp;
  const Node* nd = s->find_nth_largest(n);
  return nd ? s->index.at(nd->pk) : (size_t)-1;
}
// One full reference iteration (gossip_main.rs:449-473) for the CPU baseline;
// returns the pushes to non-failed peers of this round.
uint64_t or_sim_round(void* sp, size_t origin, double thr, size_t min_ingress, size_t asz, double p, uint32_t round) {
  Sim* s = (Sim*)sp;
  s->round_steps(s->nodes[origin].pk, thr, min_ingress, asz, p, round, nullptr);
  uint64_t e = 0;
  for (auto& kv : s->cluster.ingress_message_count) e += kv.second;
  return e;
}
size_t or_sim_rank(void* sp, size_t idx) { Sim* s = (Sim*)sp; return s->rank.at(s->nodes[idx].pk); }
size_t or_sim_visited_len(void* s) { return ((Sim*)s)->cluster.visited.size(); }
void or_sim_distances(void* sp, uint64_t* out) {
  Sim* s = (Sim*)sp;
  for (size_t i = 0; i < s->nodes.size(); ++i) {
    auto it = s->cluster.distances.find(s->nodes[i].pk);
    out[i] = it == s->cluster.distances.end() ? UINT64_MAX : it->second;
  }
}
long or_sim_orders(void* sp, size_t dest, uint32_t* src, uint64_t* hops, size_t cap) {
  Sim* s = (Sim*)sp;
  auto it = s->cluster.orders.find(s->nodes[dest].pk);
  if (it == s->cluster.orders.end()) return -1;
  std::vector<std::pair<uint64_t, uint64_t>> v;  // (hop, rank) -- the consume order
  for (auto& kv : it->second) v.push_back({kv.second, s->rank.at(kv.first)});
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size() && i < cap; ++i) {
    src[i] = (uint32_t)s->index.at(s->by_rank[v[i].second]);
    hops[i] = v[i].first;
  }
  return (long)v.size();
}
static long set_out(Sim* s, const PkMap<PkSet>& m, size_t key, uint32_t* out, size_t cap) {
  auto it = m.find(s->nodes[key].pk);
  if (it == m.end()) return -1;
  std::vector<uint32_t> v;
  for (auto& p : it->second) v.push_back((uint32_t)s->index.at(p));
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
  return (long)v.size();
}
long or_sim_pushes(void* s, size_t src, uint32_t* out, size_t cap) {
  return set_out((Sim*)s, ((Sim*)s)->cluster.pushes, src, out, cap);
}
long or_sim_mst(void* s, size_t src, uint32_t* out, size_t cap) {
  return set_out((Sim*)s, ((Sim*)s)->cluster.mst, src, out, cap);
}
size_t or_sim_prunes_len(void* s) { return ((Sim*)s)->cluster.prunes.size(); }
size_t or_sim_prunes(void* sp, uint32_t* pruner, uint32_t* prunee, size_t cap) {
  Sim* s = (Sim*)sp;
  std::vector<std::pair<uint32_t, uint32_t>> v;
  for (auto& kv : s->cluster.prunes)
    for (auto& pe : kv.second) v.push_back({(uint32_t)s->index.at(kv.first), (uint32_t)s->index.at(pe.first)});
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size() && i < cap; ++i) { pruner[i] = v[i].first; prunee[i] = v[i].second; }
  return v.size();
}
void or_sim_counters(void* sp, uint64_t* egress, uint64_t* ingress, uint64_t* prune_sent) {
  Sim* s = (Sim*)sp;
  auto fill = [&](const PkMap<uint64_t>& m, uint64_t* out) {
    for (size_t i = 0; i < s->nodes.size(); ++i) {
      auto it = m.find(s->nodes[i].pk);
      out[i] = it == m.end() ? UINT64_MAX : it->second;
    }
  };
  fill(s->cluster.egress_message_count, egress);
  fill(s->cluster.ingress_message_count, ingress);
  fill(s->cluster.prune_messages_sent, prune_sent);
}
int or_sim_rmr(void* s, double* r, uint64_t* m, uint64_t* n) {
  return ((Sim*)s)->cluster.relative_message_redundancy(r, m, n) ? 0 : -1;
}
uint64_t or_sim_rmr_m(void* s) { return ((Sim*)s)->cluster.rmr_m; }
uint64_t or_sim_rmr_n(void* s) { return ((Sim*)s)->cluster.rmr_n; }
double or_sim_coverage(void* sp, size_t* left_out) {
  Sim* s = (Sim*)sp;
  auto c = s->cluster.coverage(s->stakes);
  *left_out = c.second;
  return c.first;
}
size_t or_sim_stranded(void* sp, uint32_t* out, size_t cap) {
  Sim* s = (Sim*)sp;
  std::vector<uint32_t> v;
  for (auto& p : s->cluster.stranded_nodes()) v.push_back((uint32_t)s->index.at(p));
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size() && i < cap; ++i) out[i] = v[i];
  return v.size();
}
long or_sim_entry(void* sp, size_t node, int k, uint32_t* peers, size_t cap) {
  Sim* s = (Sim*)sp;
  auto& keys = s->nodes[node].active_set.e[k].keys;
  for (size_t i = 0; i < keys.size() && i < cap; ++i) peers[i] = (uint32_t)s->index.at(keys[i]);
  return (long)keys.size();
}
// Bulk: every entry in FIFO order, peers[(node*25+k)*cap + i] (index space), len[node*25+k].
void or_sim_entries(void* sp, uint32_t* peers, uint8_t* len, size_t cap) {
  Sim* s = (Sim*)sp;
  for (size_t n = 0; n < s->nodes.size(); ++n)
    for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k) {
      auto& keys = s->nodes[n].active_set.e[k].keys;
      len[n * 25 + k] = (uint8_t)keys.size();
      for (size_t i = 0; i < cap; ++i)
        peers[(n * 25 + k) * cap + i] = i < keys.size() ? (uint32_t)s->index.at(keys[i]) : 0xFFFFFFFFu;
    }
}
// Bulk: FIFO prune mask of every node's entry for `origin` (bit i = i-th peer's filter holds origin).
void or_sim_pruned_all(void* sp, size_t origin, uint32_t* out) {
  Sim* s = (Sim*)sp;
  const Pubkey& o = s->nodes[origin].pk;
  for (size_t n = 0; n < s->nodes.size(); ++n) {
    const uint64_t* m = opt_min(stake_of(s->stakes, s->nodes[n].pk), stake_of(s->stakes, o));
    auto& e = s->nodes[n].active_set.e[get_stake_bucket(m)];
    uint32_t bits = 0;
    for (size_t i = 0; i < e.keys.size(); ++i)
      if (e.keys[i] != o && e.filter_contains(i, o)) bits |= 1u << i;
    out[n] = bits;
  }
}
// Bulk: every node's cache entry for `origin`: upserts (UINT32_MAX when absent), len, keys sorted (cap each).
void or_sim_caches(void* sp, size_t origin, uint32_t* up, uint32_t* len, uint32_t* keys, uint32_t* scores,
                   size_t cap) {
  Sim* s = (Sim*)sp;
  const Pubkey& o = s->nodes[origin].pk;
  for (size_t n = 0; n < s->nodes.size(); ++n) {
    auto& rc = s->nodes[n].received_cache;
    auto it = rc.m.find(o);
    std::vector<std::pair<uint32_t, uint64_t>> v;
    if (it != rc.m.end())
      for (auto& kv : it->second.nodes) v.push_back({(uint32_t)s->index.at(kv.first), kv.second});
    std::sort(v.begin(), v.end());
    up[n] = it == rc.m.end() ? 0xFFFFFFFFu : (uint32_t)it->second.num_upserts;
    len[n] = (uint32_t)v.size();
    for (size_t i = 0; i < cap; ++i) {
      keys[n * cap + i] = i < v.size() ? v[i].first : 0xFFFFFFFFu;
      scores[n * cap + i] = i < v.size() ? (uint32_t)v[i].second : 0;
    }
  }
}
// 1 if `origin` is in the filter of `peer` inside entry k of `node` (prune state).
int or_sim_entry_pruned(void* sp, size_t node, int k, size_t peer, size_t origin) {
  Sim* s = (Sim*)sp;
  auto& en = s->nodes[node].active_set.e[k];
  const long i = en.index_of(s->nodes[peer].pk);
  if (i < 0) return -1;
  return en.filter_contains((size_t)i, s->nodes[origin].pk) ? 1 : 0;
}
long or_sim_cache(void* sp, size_t node, size_t origin, uint64_t* upserts, uint32_t* keys, uint64_t* scores,
                  size_t cap) {
  Sim* s = (Sim*)sp;
  auto& rc = s->nodes[node].received_cache;
  auto it = rc.m.find(s->nodes[origin].pk);
  if (it == rc.m.end()) return -1;
  *upserts = it->second.num_upserts;
  std::vector<std::pair<uint32_t, uint64_t>> v;
  for (auto& kv : it->second.nodes) v.push_back({(uint32_t)s->index.at(kv.first), kv.second});
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size() && i < cap; ++i) { keys[i] = v[i].first; scores[i] = v[i].second; }
  return (long)v.size();
}
void or_sim_failed(void* sp, uint8_t* out) {
  Sim* s = (Sim*)sp;
  for (size_t i = 0; i < s->nodes.size(); ++i) out[i] = s->nodes[i].failed;
}
size_t or_sim_total_prunes(void* s) { return ((Sim*)s)->cluster.total_prunes; }

// Bulk upload of every node's active set (the engine's, for checks at sizes where the
// reference's O(25 N^2) initialize_gossip cannot run): entry k of node n gets the peers
// peers[(n*25+k)*cap + i], i < len[n*25+k], in FIFO order, each with a fresh filter
// (only the key itself), as PushActiveSetEntry::rotate leaves a newly inserted key
// (push_active_set.rs:171-180). Indices are the caller's node indices.
int or_sim_set_entries(void* sp, const uint32_t* peers, const uint8_t* len, size_t cap) {
  Sim* s = (Sim*)sp;
  const size_t n = s->nodes.size();
  for (size_t v = 0; v < n; ++v)
    for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k) {
      auto& e = s->nodes[v].active_set.e[k];
      const size_t L = len[v * 25 + k];
      if (L > cap) { g_err = "entry longer than cap"; return -1; }
      e.keys.clear();
      e.keys.shrink_to_fit();
      e.keys.reserve(L);
      e.pruned.clear();
      for (size_t i = 0; i < L; ++i) {
        const uint32_t p = peers[(v * 25 + k) * cap + i];
        if (p >= n || p == v) { g_err = "bad peer index"; return -1; }
        e.keys.push_back(s->nodes[p].pk);
      }
    }
  return 0;
}

// Bulk orders (gossip.rs:601-607) of every destination as CSR in caller-index order:
// off[n + 1]; each list in consume order (hop, then base58 rank) as or_sim_orders.
// Returns the record count, or -1 when it exceeds cap (nothing written past cap).
long or_sim_orders_all(void* sp, uint32_t* off, uint32_t* src, uint8_t* hop, size_t cap) {
  Sim* s = (Sim*)sp;
  size_t w = 0;
  off[0] = 0;
  std::vector<std::pair<uint64_t, uint64_t>> v;
  for (size_t d = 0; d < s->nodes.size(); ++d) {
    auto it = s->cluster.orders.find(s->nodes[d].pk);
    if (it != s->cluster.orders.end()) {
      v.clear();
      for (auto& kv : it->second) v.push_back({kv.second, s->rank.at(kv.first)});
      std::sort(v.begin(), v.end());
      if (w + v.size() > cap) return -1;
      for (auto& pr : v) {
        src[w] = (uint32_t)s->index.at(s->by_rank[pr.second]);
        hop[w] = (uint8_t)std::min<uint64_t>(pr.first, 255);
        ++w;
      }
    }
    off[d + 1] = (uint32_t)w;
  }
  return (long)w;
}

// One node's active set after initialize_gossip and `rounds` chance_to_rotate calls in
// PHILOX mode, replayed for that node alone: the determinism contract makes a node's
// entries a function of (seed, its id, the rounds) only. Nodes are ids 0..n-1 (the id
// order is the candidate order); their pubkeys are stand-ins (only equality matters).
// Follows Sim::init_philox / Sim::chance_to_rotate (gossip.rs:739-754, 805-842,
// push_active_set.rs:153-187). Writes peers[k*cap + i] (ids, FIFO order) and len[k];
// returns the number of rotations the node made, -1 on a bad argument.
long or_replay_node_entries(uint64_t seed, const uint64_t* stakes_by_id, size_t n, size_t node, size_t asz,
                            double p, uint32_t rounds, uint32_t* peers, uint8_t* len, size_t cap) {
  if (node >= n || asz > cap) { g_err = "bad argument"; return -1; }
  auto pk = [](size_t i) {
    Pubkey k{};
    for (int b = 0; b < 8; ++b) k.b[31 - b] = (uint8_t)(i >> (8 * b));
    k.b[0] = 0xA5;  // never all-zero
    return k;
  };
  Stakes st;
  st.reserve(n);
  std::vector<Pubkey> cand;
  cand.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    st[pk(i)] = stakes_by_id[i];
    if (i != node) cand.push_back(pk(i));
  }
  PushActiveSet as;
  const uint32_t id = (uint32_t)node;
  {
    std::vector<PhiloxStream> streams;
    for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k) streams.emplace_back(seed, P_INIT, id, (uint32_t)k);
    as.rotate([&](int k) -> Rng& { return streams[k]; }, asz, cand, st);
  }
  long rot = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    PhiloxStream dec(seed, P_DECIDE, id, r);
    if (gen_f64(dec) < p) {
      std::vector<PhiloxStream> streams;
      for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k)
        streams.emplace_back(seed, P_ROTATE, id, (r << 5) | (uint32_t)k);
      as.rotate([&](int k) -> Rng& { return streams[k]; }, asz, cand, st);
      ++rot;
    }
  }
  for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k) {
    const auto& keys = as.e[k].keys;
    len[k] = (uint8_t)keys.size();
    for (size_t i = 0; i < cap; ++i) {
      uint32_t v = 0xFFFFFFFFu;
      if (i < keys.size()) {
        v = 0;
        for (int b = 0; b < 8; ++b) v |= (uint32_t)keys[i].b[31 - b] << (8 * b);  // ids < 2^32
      }
      peers[(size_t)k * cap + i] = v;
    }
  }
  return rot;
}

// --------------------------------------------------------------- stats ----
void* or_stats_new() { return new StatsHandle(); }
void or_stats_free(void* h) { delete (StatsHandle*)h; }
void or_stats_insert_hops(void* h, const uint64_t* d, size_t n) {
  PkMap<uint64_t> m;
  for (size_t i = 0; i < n; ++i) m[pubkey_from_counter(i + 1)] = d[i];
  ((StatsHandle*)h)->st.insert_hops_stat(m);
}
void or_stats_insert_coverage(void* h, double v) { ((StatsHandle*)h)->st.coverage.collection.push_back(v); }
void or_stats_insert_rmr(void* h, double v) { ((StatsHandle*)h)->st.rmr.collection.push_back(v); }
void or_stats_insert_stranded(void* h, const uint8_t* pks, size_t n, void* stakes) {
  ((StatsHandle*)h)->st.stranded.insert_nodes(pk_vec(pks, n), *(Stakes*)stakes);
}
void or_stats_branching(void* h, const uint64_t* set_sizes, size_t n_srcs) {
  PkMap<PkSet> pushes;
  for (size_t i = 0; i < n_srcs; ++i) {
    PkSet s;
    for (uint64_t j = 0; j < set_sizes[i]; ++j) s.insert(pubkey_from_counter(j + 1));
    pushes[pubkey_from_counter(1000000 + i)] = s;
  }
  ((StatsHandle*)h)->st.calculate_branching(pushes);
}
void or_stats_calculate(void* h) { ((StatsHandle*)h)->st.run_all_calculations(); }

void* or_run_simulation(const uint8_t* pks, const uint64_t* stakes, size_t n, size_t fanout, size_t asz,
                        size_t iterations, size_t origin_rank, double p, double thr, size_t min_ingress,
                        uint64_t nb_stranded, uint64_t nb_message, uint64_t nb_hops, double fraction_to_fail,
                        size_t when_to_fail, int test_type, size_t warm_up, uint64_t seed) {
  SimConfig c;
  c.push_fanout = fanout; c.active_set_size = asz; c.iterations = iterations; c.origin_rank = origin_rank;
  c.rotation_probability = p; c.prune_stake_threshold = thr; c.min_ingress_nodes = min_ingress;
  c.num_buckets_stranded = nb_stranded; c.num_buckets_message = nb_message; c.num_buckets_hops = nb_hops;
  c.fraction_to_fail = fraction_to_fail; c.when_to_fail = when_to_fail; c.test_type = test_type;
  c.warm_up_rounds = warm_up; c.seed = seed;
  auto* h = new StatsHandle();
  auto v = pk_vec(pks, n);
  for (size_t i = 0; i < n; ++i) h->index[v[i]] = i;
  try {
    Pubkey origin;
    run_simulation(c, v, std::vector<uint64_t>(stakes, stakes + n), h->st, &origin);
    h->origin_index = h->index.at(origin);
  } catch (std::exception& e) {
    g_err = e.what();
    delete h;
    return nullptr;
  }
  return h;
}

size_t or_res_f64(void* hp, const char* name, double* out, size_t cap) {
  auto* h = (StatsHandle*)hp;
  auto& st = h->st;
  std::string n(name);
  auto s4 = [](const StatCollection& c) { return std::vector<double>{c.mean, c.median, c.max, c.min}; };
  if (n == "coverage") return put_f(st.coverage.collection, out, cap);
  if (n == "rmr") return put_f(st.rmr.collection, out, cap);
  if (n == "branching") return put_f(st.branching.collection, out, cap);
  if (n == "coverage_stats") return put_f(s4(st.coverage), out, cap);
  if (n == "rmr_stats") return put_f(s4(st.rmr), out, cap);
  if (n == "branching_stats") return put_f(s4(st.branching), out, cap);
  if (n == "hop_mean" || n == "hop_median") {
    std::vector<double> v;
    for (auto& x : st.per_round_hops) v.push_back(n == "hop_mean" ? x.mean : x.median);
    return put_f(v, out, cap);
  }
  if (n == "aggregate_hops") return put_f({st.aggregate_hops.mean, st.aggregate_hops.median}, out, cap);
  if (n == "ldh") return put_f({st.ldh.mean, st.ldh.median}, out, cap);
  if (n == "stranded_round_mean" || n == "stranded_round_median") {
    std::vector<double> v;
    for (auto& x : st.stranded.per_iter) v.push_back(n == "stranded_round_mean" ? x.mean : x.median);
    return put_f(v, out, cap);
  }
  if (n == "stranded") {
    auto& s = st.stranded;
    // get_stranded_stats order (gossip_stats.rs:1572-1602), f64 members only
    return put_f({s.stranded_iterations_per_node, s.mean_stranded_per_iteration, s.mean_iters_per_stranded_node,
                  s.median_iters_per_stranded_node, s.mean_stake, s.median_stake, s.weighted_mean_stake,
                  s.weighted_median_stake},
                 out, cap);
  }
  return (size_t)-1;
}

size_t or_res_u64(void* hp, const char* name, uint64_t* out, size_t cap) {
  auto* h = (StatsHandle*)hp;
  auto& st = h->st;
  std::string n(name);
  if (n == "origin") return put_u({h->origin_index}, out, cap);
  if (n == "hop_max" || n == "hop_min") {
    std::vector<uint64_t> v;
    for (auto& x : st.per_round_hops) v.push_back(n == "hop_max" ? x.max : x.min);
    return put_u(v, out, cap);
  }
  if (n == "aggregate_hops") return put_u({st.aggregate_hops.max, st.aggregate_hops.min}, out, cap);
  if (n == "rmr_m") return put_u(st.rmr_m, out, cap);
  if (n == "rmr_n") return put_u(st.rmr_n, out, cap);
  if (n == "ldh") return put_u({st.ldh.max, st.ldh.min}, out, cap);
  if (n == "stranded_round_count" || n == "stranded_round_max" || n == "stranded_round_min") {
    std::vector<uint64_t> v;
    for (auto& x : st.stranded.per_iter)
      v.push_back(n == "stranded_round_count" ? x.count : n == "stranded_round_max" ? x.max : x.min);
    return put_u(v, out, cap);
  }
  if (n == "stranded") {
    auto& s = st.stranded;
    return put_u({s.total_stranded_iterations, (uint64_t)s.stranded_nodes.size(), s.max_stake, s.min_stake}, out, cap);
  }
  if (n == "stranded_times") {  // (node index, times) sorted by index
    std::vector<std::pair<uint64_t, uint64_t>> v;
    for (auto& kv : st.stranded.stranded_nodes) v.push_back({h->index.at(kv.first), kv.second.second});
    std::sort(v.begin(), v.end());
    std::vector<uint64_t> f;
    for (auto& p : v) { f.push_back(p.first); f.push_back(p.second); }
    return put_u(f, out, cap);
  }
  if (n == "hops_hist") return put_u(hist_kv(st.hops_histogram), out, cap);
  if (n == "stranded_hist") return put_u(hist_kv(st.stranded.histogram), out, cap);
  if (n == "validator_hist") return put_u(hist_kv(st.validator_stake_distribution), out, cap);
  if (n == "egress_hist") return put_u(hist_kv(st.egress.histogram), out, cap);
  if (n == "ingress_hist") return put_u(hist_kv(st.ingress.histogram), out, cap);
  if (n == "prune_hist") return put_u(hist_kv(st.prune.histogram), out, cap);
  if (n == "egress_cpb") return put_u(st.egress.count_per_bucket, out, cap);
  if (n == "hist_errors")
    return put_u({(uint64_t)st.hops_histogram.errors, (uint64_t)st.stranded.histogram.errors}, out, cap);
  if (n == "failed_count") return put_u({(uint64_t)st.failed_count}, out, cap);
  return (size_t)-1;
}

// CPU baseline on all host cores (bench.py's cpu_baseline leg; test infrastructure):
// n_sims independent reference-structure simulations (one origin each, as
// gossip_main.rs runs them), dealt round-robin over `threads` std::threads. Every sim
// is initialised first (init_s, wall); then every thread runs rounds [0, rounds) of
// its sims (gossip_main.rs:449-473) and the wall time of that parallel region is
// run_s. Returns the pushes to non-failed peers summed over sims and rounds.
uint64_t or_bench_parallel(uint64_t seed, const uint8_t* pks, const uint64_t* stakes, size_t n, size_t fanout,
                           size_t asz, const uint32_t* origins, size_t n_sims, double thr, size_t min_ingress, double p,
                           uint32_t rounds, uint32_t threads, double* init_s, double* run_s) {
  using clk = std::chrono::steady_clock;
  if (threads < 1) threads = 1;
  std::vector<std::unique_ptr<Sim>> sims(n_sims);
  auto par = [&](auto&& body) {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t)
      th.emplace_back([&, t]() {
        for (size_t i = t; i < n_sims; i += threads) body(i);
      });
    for (auto& x : th) x.join();
  };
  const auto t0 = clk::now();
  par([&](size_t i) {
    sims[i].reset(new Sim(PHILOX, seed, pk_vec(pks, n), std::vector<uint64_t>(stakes, stakes + n), fanout));
    sims[i]->init_philox(asz);
  });
  const auto t1 = clk::now();
  std::vector<uint64_t> edges(n_sims, 0);
  par([&](size_t i) {
    Sim* s = sims[i].get();
    const Pubkey org = s->nodes[origins[i]].pk;
    for (uint32_t r = 0; r < rounds; ++r) {
      s->round_steps(org, thr, min_ingress, asz, p, r, nullptr);
      for (auto& kv : s->cluster.ingress_message_count) edges[i] += kv.second;
    }
  });
  const auto t2 = clk::now();
  *init_s = std::chrono::duration<double>(t1 - t0).count();
  *run_s = std::chrono::duration<double>(t2 - t1).count();
  uint64_t e = 0;
  for (uint64_t x : edges) e += x;
  return e;
}

}  // extern "C"
