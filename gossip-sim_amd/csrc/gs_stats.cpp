// gs_stats.cpp -- host half of the statistics path (gossip_stats.rs) and the
// run_simulation driver (gossip_main.rs:292-647) on top of the engine ABI.
//
// The device reduces each recorded round to integers (gs_round_summary, the
// hop histogram, per-node accumulators); the f64 summaries are formed here in
// the reference's operation order so they are bit-identical to it:
//   HopsStat::new                 gossip_stats.rs:47-98
//   StatCollection::calculate     gossip_stats.rs:266-295 (mean = fold over the sorted values)
//   StrandedNodeStats::new        gossip_stats.rs:767-819
//   StrandedNodeCollection::calc  gossip_stats.rs:964-1038
//   Histogram::build/_from_map    gossip_stats.rs:575-682
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/gossip_hip.h"

namespace {

struct Hops {
  double mean = 0, median = 0;
  uint64_t max = 0, min = 0;
};

// HopsStat over a value->count histogram (values 0 and u64::MAX excluded by the caller).
Hops hops_from_counts(const std::map<uint64_t, uint64_t>& h) {
  Hops s;
  uint64_t count = 0, sum = 0;
  for (auto& kv : h) { count += kv.second; sum += kv.first * kv.second; }
  s.mean = (double)sum / (double)count;
  auto kth = [&](uint64_t k) {
    uint64_t run = 0;
    for (auto& kv : h) {
      if (k < run + kv.second) return kv.first;
      run += kv.second;
    }
    return (uint64_t)0;
  };
  if (count == 0) s.median = 0.0;
  else if (count == 1) s.median = (double)kth(0);
  else if (count % 2 == 0) s.median = (double)(kth(count / 2 - 1) + kth(count / 2)) / 2.0;
  else s.median = (double)kth(count / 2);
  s.max = count ? h.rbegin()->first : 0;
  s.min = count ? h.begin()->first : 0;
  return s;
}

void stat4(const std::vector<double>& in, double out[4]) {
  std::vector<double> v = in;
  std::sort(v.begin(), v.end());
  const size_t len = v.size();
  double sum = 0.0;
  for (double x : v) sum += x;
  out[0] = sum / (double)len;
  out[1] = len == 0 ? std::nan("") : (len % 2 == 0 ? (v[len / 2 - 1] + v[len / 2]) / 2.0 : v[len / 2]);
  out[2] = len ? v.back() : 0.0;
  out[3] = len ? v.front() : 0.0;
}

struct Hist {
  std::map<uint64_t, uint64_t> entries;
  uint64_t min_entry = 0, max_entry = 0, range = 0, nb = 0, errors = 0;
  bool ok = true;
  // Histogram::build over a value->multiplicity map
  void build(uint64_t upper, uint64_t lower, uint64_t n_buckets, const std::map<uint64_t, uint64_t>& values) {
    min_entry = lower; max_entry = upper; nb = n_buckets;
    range = (upper == lower || lower + 1 == upper) ? 1 : (upper - lower) / n_buckets;
    entries.clear();
    for (uint64_t b = 0; b < nb; ++b) entries[b] = 0;
    for (auto& kv : values) {
      if (kv.first >= min_entry && kv.first <= max_entry) {
        if (range == 0) { ok = false; return; }
        uint64_t b = (kv.first - min_entry) / range;
        if (b == nb) b -= 1;
        entries[b] += kv.second;
      } else {
        errors += kv.second;
      }
    }
  }
};

// EgressIngressMessageTracker::build_histogram + normalize (gossip_stats.rs:399-431,621-682)
struct Tracker {
  Hist h;
  std::vector<uint64_t> cpb;
  void build(uint64_t nb, const uint64_t* stakes, const std::vector<uint64_t>& counts, uint64_t max_stake) {
    h.min_entry = 0; h.max_entry = max_stake; h.nb = nb;
    h.range = (max_stake == 0) ? 1 : max_stake / nb;
    h.entries.clear();
    for (uint64_t b = 0; b < nb; ++b) h.entries[b] = 0;
    cpb.assign(nb, 0);
    for (size_t v = 0; v < counts.size(); ++v) {
      const uint64_t s = stakes[v];
      if (h.range == 0) { h.ok = false; return; }
      uint64_t b = s / h.range;
      if (b == nb) b -= 1;
      h.entries[b] += counts[v];
      if (b >= cpb.size()) { h.ok = false; return; }  // the reference panics here
      cpb[b] += 1;
    }
    for (auto& kv : h.entries) {
      const uint64_t n = cpb[kv.first];
      if (n) kv.second /= n;
    }
  }
};

std::vector<uint64_t> kv_flat(const std::map<uint64_t, uint64_t>& m) {
  std::vector<uint64_t> v;
  for (auto& kv : m) { v.push_back(kv.first); v.push_back(kv.second); }
  return v;
}

double median_of_sorted_counts(const std::vector<std::pair<uint64_t, uint64_t>>& sorted_vc) {
  // median of a multiset given as ascending (value, multiplicity)
  uint64_t n = 0;
  for (auto& p : sorted_vc) n += p.second;
  if (n == 0) return 0.0;
  auto kth = [&](uint64_t k) {
    uint64_t run = 0;
    for (auto& p : sorted_vc) {
      if (k < run + p.second) return p.first;
      run += p.second;
    }
    return (uint64_t)0;
  };
  if (n % 2 == 0) return (double)(kth(n / 2 - 1) + kth(n / 2)) / 2.0;
  return (double)kth(n / 2);
}

}  // namespace

struct SimStats {
  std::map<std::string, std::vector<double>> f;
  std::map<std::string, std::vector<uint64_t>> u;
};

struct gs_sim_result {
  std::vector<SimStats> sims;
};

static thread_local std::string g_sim_err;

extern "C" {

int gs_hops_stat_new(const uint64_t* hops, size_t n, gs_hops_stat* out) {
  if (!out || (n && !hops)) return GS_EINVAL;
  std::map<uint64_t, uint64_t> h;
  for (size_t i = 0; i < n; ++i)
    if (hops[i] != UINT64_MAX && hops[i] != 0) h[hops[i]] += 1;
  Hops s = hops_from_counts(h);
  out->mean = s.mean; out->median = s.median; out->max = s.max; out->min = s.min;
  return GS_OK;
}

int gs_stat_collection_calculate(const double* values, size_t n, gs_stat4* out) {
  if (!out || (n && !values)) return GS_EINVAL;
  double r[4];
  stat4(std::vector<double>(values, values + n), r);
  out->mean = r[0]; out->median = r[1]; out->max = r[2]; out->min = r[3];
  return GS_OK;
}

void gs_result_free(gs_sim_result* r) { delete r; }

size_t gs_result_f64(const gs_sim_result* r, uint32_t sim, const char* name, double* out, size_t cap) {
  if (!r || sim >= r->sims.size() || !name) return SIZE_MAX;
  auto it = r->sims[sim].f.find(name);
  if (it == r->sims[sim].f.end()) return SIZE_MAX;
  for (size_t i = 0; i < it->second.size() && i < cap; ++i) out[i] = it->second[i];
  return it->second.size();
}

size_t gs_result_u64(const gs_sim_result* r, uint32_t sim, const char* name, uint64_t* out, size_t cap) {
  if (!r || sim >= r->sims.size() || !name) return SIZE_MAX;
  auto it = r->sims[sim].u.find(name);
  if (it == r->sims[sim].u.end()) return SIZE_MAX;
  for (size_t i = 0; i < it->second.size() && i < cap; ++i) out[i] = it->second[i];
  return it->second.size();
}

// find_nth_largest_node (gossip_main.rs:279-290): the n-th largest stake value of
// the multiset; among nodes holding it, the lowest id.
static int64_t nth_largest(const uint64_t* stakes, uint32_t n, uint32_t rank) {
  if (rank == 0 || rank > n) return -1;
  std::vector<uint64_t> v(stakes, stakes + n);
  std::nth_element(v.begin(), v.begin() + (rank - 1), v.end(), std::greater<uint64_t>());
  const uint64_t s = v[rank - 1];
  for (uint32_t i = 0; i < n; ++i)
    if (stakes[i] == s) return i;
  return -1;
}

int gs_run_simulations(const gs_sim_config* cfg, const uint64_t* stakes, uint32_t n, uint32_t n_sims,
                       const uint32_t* origin_ranks, const uint32_t* min_ingress, const double* thresholds,
                       const double* fractions, gs_sim_result** out) {
  if (!cfg || !stakes || !out || n_sims == 0) return GS_EINVAL;
  *out = nullptr;
  gs_params prm{};
  prm.push_fanout = cfg->push_fanout;
  prm.active_set_size = cfg->active_set_size;
  prm.rotation_probability = cfg->rotation_probability;
  prm.seed = cfg->seed;
  prm.device = cfg->device;
  prm.bfs_mode = cfg->bfs_mode;
  gs_engine* e = nullptr;
  int r = gs_create(&prm, stakes, n, n_sims, &e);
  if (r) return r;
  std::vector<gs_slot> slots(n_sims);
  for (uint32_t i = 0; i < n_sims; ++i) {
    const int64_t o = nth_largest(stakes, n, origin_ranks ? origin_ranks[i] : 1);
    if (o < 0) { gs_destroy(e); return GS_EINVAL; }
    slots[i].origin = (uint32_t)o;
    slots[i].min_ingress_nodes = min_ingress ? min_ingress[i] : cfg->min_ingress_nodes;
    slots[i].prune_stake_threshold = thresholds ? thresholds[i] : cfg->prune_stake_threshold;
  }
  std::vector<double> frac(n_sims, cfg->fraction_to_fail);
  if (fractions) frac.assign(fractions, fractions + n_sims);
#define CK(x) do { r = (x); if (r) { gs_destroy(e); return r; } } while (0)
  CK(gs_set_slots(e, slots.data(), n_sims));
  CK(gs_init_active_sets(e));
  for (uint32_t it = 0; it < cfg->iterations; ++it) {
    if (cfg->test_type == 5 && it == cfg->when_to_fail) CK(gs_fail_nodes(e, frac.data()));
    CK(gs_round(e, it, it >= cfg->warm_up_rounds));
  }
  CK(gs_sync(e));
  const uint32_t rounds = cfg->iterations > cfg->warm_up_rounds ? cfg->iterations - cfg->warm_up_rounds : 0;
  std::vector<gs_round_summary> sums((size_t)rounds * n_sims + 1);
  size_t nsum = 0;
  CK(gs_read_round_summaries(e, sums.data(), sums.size(), &nsum));
  std::unique_ptr<gs_sim_result> res(new gs_sim_result());  // released to *out only on success
  res->sims.resize(n_sims);
  uint64_t max_stake = 0;
  for (uint32_t v = 0; v < n; ++v) max_stake = std::max(max_stake, stakes[v]);
  std::vector<uint64_t> eg(n), in(n), pr(n), hh(256);
  std::vector<uint32_t> st(n);
  std::vector<uint8_t> failed(n);
  for (uint32_t s = 0; s < n_sims; ++s) {
    SimStats& o = res->sims[s];
    CK(gs_read_accumulators(e, s, eg.data(), in.data(), pr.data(), st.data(), hh.data()));
    CK(gs_read_failed(e, s, failed.data()));
    std::vector<double> cov, rmr, br, hmean, hmed, smean, smed;
    std::vector<uint64_t> hmax, hmin, scnt, smax, smin, rm, rn;
    for (uint32_t k = 0; k < rounds; ++k) {
      const gs_round_summary& q = sums[(size_t)k * n_sims + s];
      cov.push_back((double)q.visited / (double)n);
      const uint64_t m = (uint64_t)q.pushes + q.prunes;
      rmr.push_back((double)m / (double)(q.visited - 1) - 1.0);
      rm.push_back(m);
      rn.push_back(q.visited);
      br.push_back(q.visited ? (double)q.pushes / (double)q.visited : 0.0);
      // per-round HopsStat
      double mean = (double)q.hop_sum / (double)q.hop_count, med = 0.0;
      if (q.hop_count == 1 || (q.hop_count && q.hop_count % 2)) med = (double)q.hop_med_lo;
      else if (q.hop_count) med = (double)((uint64_t)q.hop_med_lo + q.hop_med_hi) / 2.0;
      hmean.push_back(mean); hmed.push_back(med);
      hmax.push_back(q.hop_count ? q.hop_max : 0); hmin.push_back(q.hop_count ? q.hop_min : 0);
      // per-round StrandedNodeStats
      scnt.push_back(q.stranded);
      if (q.stranded == 0) { smean.push_back(0.0); smed.push_back(0.0); smax.push_back(0); smin.push_back(0); }
      else if (q.stranded == 1) {
        smean.push_back((double)q.stranded_stake_min); smed.push_back((double)q.stranded_stake_min);
        smax.push_back(q.stranded_stake_min); smin.push_back(q.stranded_stake_min);
      } else {
        smean.push_back((double)q.stranded_stake_sum / (double)q.stranded);
        smed.push_back(q.stranded % 2 ? (double)q.stranded_med_lo
                                      : (double)(q.stranded_med_lo + q.stranded_med_hi) / 2.0);
        smax.push_back(q.stranded_stake_max); smin.push_back(q.stranded_stake_min);
      }
    }
    o.f["coverage"] = cov; o.f["rmr"] = rmr; o.f["branching"] = br;
    o.u["rmr_m"] = rm; o.u["rmr_n"] = rn;  // the rmr datapoint's m, n (influx_db.rs:346-360)
    o.f["hop_mean"] = hmean; o.f["hop_median"] = hmed;
    o.u["hop_max"] = hmax; o.u["hop_min"] = hmin;
    o.u["stranded_round_count"] = scnt; o.u["stranded_round_max"] = smax; o.u["stranded_round_min"] = smin;
    o.f["stranded_round_mean"] = smean; o.f["stranded_round_median"] = smed;
    o.u["origin"] = {slots[s].origin};
    if (rounds == 0) continue;
    double c4[4];
    stat4(cov, c4); o.f["coverage_stats"] = {c4[0], c4[1], c4[2], c4[3]};
    stat4(rmr, c4); o.f["rmr_stats"] = {c4[0], c4[1], c4[2], c4[3]};
    stat4(br, c4); o.f["branching_stats"] = {c4[0], c4[1], c4[2], c4[3]};
    // aggregate hops over raw_hop_collection (0s kept in the histogram, dropped by HopsStat)
    std::map<uint64_t, uint64_t> raw, raw_nz;
    for (int h = 0; h < 255; ++h)
      if (hh[h]) { raw[h] = hh[h]; if (h) raw_nz[h] = hh[h]; }
    Hops ag = hops_from_counts(raw_nz);
    o.f["aggregate_hops"] = {ag.mean, ag.median}; o.u["aggregate_hops"] = {ag.max, ag.min};
    std::map<uint64_t, uint64_t> maxes;
    for (auto x : hmax) if (x) maxes[x] += 1;
    Hops ldh = hops_from_counts(maxes);
    o.f["ldh"] = {ldh.mean, ldh.median}; o.u["ldh"] = {ldh.max, ldh.min};
    Hist hops_hist;
    uint64_t hb = 30;
    if (cfg->test_type == 5) hb = (uint64_t)(40.0 * (1.0 + frac[s]));
    else if (cfg->test_type == 2) hb = 50;
    hops_hist.build(hb, 0, cfg->num_buckets_hops, raw);
    o.u["hops_hist"] = kv_flat(hops_hist.entries);
    // StrandedNodeCollection::calculate_stats
    uint64_t tot_it = 0, tot_stake = 0, wtot = 0, cnt = 0;
    std::vector<uint64_t> times_v, stakes_v;
    std::map<uint64_t, uint64_t> wstakes, times_hist_in;
    std::vector<uint64_t> stimes;
    for (uint32_t v = 0; v < n; ++v) {
      if (!st[v]) continue;
      ++cnt;
      tot_it += st[v];
      tot_stake += stakes[v];
      wtot += stakes[v] * (uint64_t)st[v];
      times_v.push_back(st[v]);
      stakes_v.push_back(stakes[v]);
      wstakes[stakes[v]] += st[v];
      times_hist_in[st[v]] += 1;
      stimes.push_back(v); stimes.push_back(st[v]);
    }
    std::sort(times_v.begin(), times_v.end());
    std::sort(stakes_v.begin(), stakes_v.end());
    auto med = [](const std::vector<uint64_t>& x) {
      if (x.empty()) return 0.0;
      size_t k = x.size();
      return k % 2 == 0 ? (double)(x[k / 2 - 1] + x[k / 2]) / 2.0 : (double)x[k / 2];
    };
    std::vector<std::pair<uint64_t, uint64_t>> wv(wstakes.begin(), wstakes.end());
    const double dc = (double)cnt;
    o.u["stranded"] = {tot_it, cnt, stakes_v.empty() ? 0 : stakes_v.back(), stakes_v.empty() ? 0 : stakes_v.front()};
    o.f["stranded"] = {(double)tot_it / (double)n, (double)tot_it / (double)rounds, (double)tot_it / dc,
                       med(times_v), (double)tot_stake / dc, med(stakes_v), (double)wtot / (double)tot_it,
                       median_of_sorted_counts(wv)};
    o.u["stranded_times"] = stimes;
    Hist sh;
    sh.build(rounds, 0, cfg->num_buckets_stranded, times_hist_in);
    o.u["stranded_hist"] = kv_flat(sh.entries);
    Tracker te, ti, tp;
    te.build(cfg->num_buckets_message, stakes, eg, max_stake);
    ti.build(cfg->num_buckets_message, stakes, in, max_stake);
    tp.build(cfg->num_buckets_message, stakes, pr, max_stake);
    o.u["egress_hist"] = kv_flat(te.h.entries); o.u["egress_cpb"] = te.cpb;
    o.u["ingress_hist"] = kv_flat(ti.h.entries);
    o.u["prune_hist"] = kv_flat(tp.h.entries);
    std::map<uint64_t, uint64_t> sv;
    for (uint32_t v = 0; v < n; ++v) sv[stakes[v]] += 1;
    Hist vh;
    vh.build(max_stake, 0, 50, sv);
    o.u["validator_hist"] = kv_flat(vh.entries);
    o.u["hist_errors"] = {hops_hist.errors, sh.errors};
    uint64_t nf = 0;
    for (uint32_t v = 0; v < n; ++v) nf += failed[v];
    o.u["failed_count"] = {nf};
  }
#undef CK
  gs_destroy(e);
  *out = res.release();
  return GS_OK;
}

}  // extern "C"
