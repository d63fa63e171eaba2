// oracle/oracle_core.cpp -- TEST INFRASTRUCTURE ONLY (see oracle_core.h).
#include "oracle_core.h"
#include <algorithm>
#include <stdexcept>

namespace orc {

// ------------------------------------------------------------- base58 ----
static const char* B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz";

std::string base58(const Pubkey& p) {
  // Big-number base conversion; each leading zero byte becomes a leading '1'.
  int zeros = 0;
  while (zeros < 32 && p.b[zeros] == 0) ++zeros;
  std::vector<uint8_t> digits;  // base-58 digits, little-endian
  for (int i = zeros; i < 32; ++i) {
    uint32_t carry = p.b[i];
    for (auto& d : digits) {
      carry += (uint32_t)d << 8;
      d = (uint8_t)(carry % 58);
      carry /= 58;
    }
    while (carry) { digits.push_back((uint8_t)(carry % 58)); carry /= 58; }
  }
  std::string s(zeros, '1');
  for (auto it = digits.rbegin(); it != digits.rend(); ++it) s.push_back(B58[*it]);
  return s;
}

Pubkey pubkey_from_counter(uint64_t i) {
  Pubkey p{};
  for (int k = 0; k < 8; ++k) p.b[k] = (uint8_t)(i >> (56 - 8 * k));
  return p;
}

// ------------------------------------------------------------- ChaCha ----
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define QR(a, b, c, d)              \
  a += b; d ^= a; d = rotl32(d, 16); \
  c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  \
  c += d; b ^= c; b = rotl32(b, 7);

ChaCha20Rng::ChaCha20Rng(const uint8_t seed[32]) {
  for (int i = 0; i < 8; ++i)
    key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
             ((uint32_t)seed[4 * i + 3] << 24);
}

uint32_t ChaCha20Rng::next_u32() {
  if (idx >= 16) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                      key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                      (uint32_t)counter, (uint32_t)(counter >> 32), 0u, 0u};
    uint32_t x[16];
    std::memcpy(x, s, sizeof x);
    for (int r = 0; r < 10; ++r) {
      QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
      QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
      QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
      QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) buf[i] = x[i] + s[i];
    ++counter;
    idx = 0;
  }
  return buf[idx++];
}

uint64_t ChaCha20Rng::next_u64() {
  uint64_t lo = next_u32();
  uint64_t hi = next_u32();
  return lo | (hi << 32);
}

// ------------------------------------------------------------- Philox ----
void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

PhiloxStream::PhiloxStream(uint64_t seed, uint32_t purpose_, uint32_t a_, uint32_t b_)
    : a(a_), b(b_), purpose(purpose_) {
  key[0] = (uint32_t)seed;
  key[1] = (uint32_t)(seed >> 32);
}

uint64_t PhiloxStream::next_u64() {
  if (idx >= 4) {
    uint32_t ctr[4] = {block, a, b, purpose};
    philox4x32_10(ctr, key, out);
    ++block;
    idx = 0;
  }
  uint64_t v = (uint64_t)out[idx] | ((uint64_t)out[idx + 1] << 32);
  idx += 2;
  return v;
}

// ------------------------------------------------------- rand 0.7 bits ----
uint64_t sample_single_u64(uint64_t low, uint64_t high, Rng& rng) {
  if (!(low < high)) throw std::runtime_error("sample_single: low >= high");
  uint64_t range = high - low;
  int lz = __builtin_clzll(range);
  uint64_t zone = (range << lz) - 1;
  for (;;) {
    uint64_t v = rng.next_u64();
    unsigned __int128 m = (unsigned __int128)v * range;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    if (lo <= zone) return low + hi;
  }
}

double gen_f64(Rng& rng) {
  uint64_t v = rng.next_u64() >> 11;
  return (double)v * (1.0 / 9007199254740992.0);
}

// ------------------------------------------------------------ buckets ----
int get_stake_bucket(const uint64_t* stake) {
  uint64_t s = (stake ? *stake : 0) / LAMPORTS_PER_SOL;
  int bits = s ? 64 - __builtin_clzll(s) : 0;
  return std::min(bits, NUM_PUSH_ACTIVE_SET_ENTRIES - 1);
}

const uint64_t* opt_min(const uint64_t* a, const uint64_t* b) {
  if (!a || !b) return nullptr;
  return *b < *a ? b : a;
}

// -------------------------------------------------- WeightedShuffle ----
WeightedShuffle::WeightedShuffle(const std::vector<uint64_t>& weights) : w(weights) {
  for (size_t k = 0; k < w.size(); ++k) {
    if (w[k] == 0) { zeros.push_back(k); continue; }
    if (sum + w[k] < sum) { zeros.push_back(k); w[k] = 0; continue; }  // checked_add overflow
    sum += w[k];
  }
}

std::optional<size_t> WeightedShuffle::next(Rng& rng) {
  if (sum > 0) {
    uint64_t v = sample_single_u64(0, sum, rng);
    uint64_t acc = 0;
    for (size_t i = 0; i < w.size(); ++i) {
      acc += w[i];
      if (acc > v) {
        sum -= w[i];
        w[i] = 0;
        return i;
      }
    }
    throw std::runtime_error("WeightedShuffle: search fell off the end");
  }
  if (zeros.empty()) return std::nullopt;
  size_t i = (size_t)sample_single_u64(0, zeros.size(), rng);
  size_t r = zeros[i];
  zeros[i] = zeros.back();
  zeros.pop_back();
  return r;
}

// --------------------------------------------------- PushActiveSet ----
long PushActiveSetEntry::index_of(const Pubkey& node) const {
  for (size_t i = 0; i < keys.size(); ++i)
    if (keys[i] == node) return (long)i;
  return -1;
}

bool PushActiveSetEntry::filter_contains(size_t i, const Pubkey& x) const {
  if (x == keys[i]) return true;
  for (const auto& pr : pruned)
    if (pr.first == i && pr.second == x) return true;
  return false;
}

std::vector<Pubkey> PushActiveSetEntry::get_nodes(const Pubkey& origin,
                                                  const std::function<bool(const Pubkey&)>& force) const {
  std::vector<Pubkey> out;
  for (size_t i = 0; i < keys.size(); ++i)
    if (!filter_contains(i, origin) || force(keys[i])) out.push_back(keys[i]);
  return out;
}

void PushActiveSetEntry::prune(const Pubkey& node, const Pubkey& origin) {
  const long i = index_of(node);  // push_active_set.rs:56-71: only a present key's filter
  if (i >= 0 && !filter_contains((size_t)i, origin)) pruned.push_back({(uint32_t)i, origin});
}

void PushActiveSetEntry::rotate(Rng& rng, size_t size, const std::vector<Pubkey>& nodes,
                                const std::vector<uint64_t>& weights) {
  WeightedShuffle sh(weights);
  for (;;) {
    auto k = sh.next(rng);  // the draw happens before the length check (push_active_set.rs:165-168)
    if (!k) break;
    if (keys.size() > size) break;
    const Pubkey& node = nodes[*k];
    if (index_of(node) >= 0) continue;
    keys.push_back(node);  // with a fresh filter holding the node itself: a peer never receives its own origin
  }
  while (keys.size() > size) {  // shift_remove_index(0): the front key and its filter go, indices shift down
    keys.erase(keys.begin());
    std::vector<std::pair<uint32_t, Pubkey>> kept;
    for (const auto& pr : pruned)
      if (pr.first > 0) kept.push_back({pr.first - 1, pr.second});
    pruned.swap(kept);
  }
}

std::vector<Pubkey> PushActiveSet::get_nodes(const Pubkey& self, const Pubkey& origin, const Stakes& stakes) const {
  const uint64_t* s = opt_min(stake_of(stakes, self), stake_of(stakes, origin));
  return e[get_stake_bucket(s)].get_nodes(origin, [](const Pubkey&) { return false; });
}

void PushActiveSet::prune(const Pubkey& self, const Pubkey& node, const std::vector<Pubkey>& origins,
                          const Stakes& stakes) {
  const uint64_t* s = stake_of(stakes, self);
  for (const auto& origin : origins) {
    if (origin == self) continue;
    const uint64_t* m = opt_min(s, stake_of(stakes, origin));
    e[get_stake_bucket(m)].prune(node, origin);
  }
}

void PushActiveSet::rotate(const std::function<Rng&(int)>& rng_for_k, size_t size, const std::vector<Pubkey>& nodes,
                           const Stakes& stakes) {
  std::vector<int> buckets(nodes.size());
  for (size_t i = 0; i < nodes.size(); ++i) buckets[i] = get_stake_bucket(stake_of(stakes, nodes[i]));
  std::vector<uint64_t> weights(nodes.size());
  for (int k = 0; k < NUM_PUSH_ACTIVE_SET_ENTRIES; ++k) {
    for (size_t i = 0; i < nodes.size(); ++i) {
      uint64_t b = (uint64_t)std::min(buckets[i], k);
      weights[i] = (b + 1) * (b + 1);
    }
    e[k].rotate(rng_for_k(k), size, nodes, weights);
  }
}

// --------------------------------------------------- ReceivedCache ----
void ReceivedCacheEntry::record(const Pubkey& node, size_t num_dups) {
  if (num_dups == 0) num_upserts += 1;
  if (num_dups < NUM_DUPS_THRESHOLD) {
    nodes[node] += 1;
  } else if (nodes.size() < CAPACITY) {
    nodes.emplace(node, 0);
  }
}

void ReceivedCache::record(const Pubkey& origin, const Pubkey& node, size_t num_dups) {
  m[origin].record(node, num_dups);
}

std::vector<Pubkey> ReceivedCache::prune(const Pubkey& self, const Pubkey& origin, double stake_threshold,
                                         size_t min_ingress_nodes, const Stakes& stakes,
                                         const std::function<uint64_t(const Pubkey&)>& tie_rank) {
  std::vector<Pubkey> out;
  auto it = m.find(origin);  // peek_mut: no LRU promotion
  if (it == m.end() || it->second.num_upserts < MIN_NUM_UPSERTS) return out;
  ReceivedCacheEntry entry = std::move(it->second);
  it->second = ReceivedCacheEntry{};  // std::mem::take
  const uint64_t* ms = opt_min(stake_of(stakes, self), stake_of(stakes, origin));
  uint64_t min_ingress_stake = (uint64_t)((double)(ms ? *ms : 0) * stake_threshold);
  struct Item { Pubkey node; uint64_t score, stake, rank; };
  std::vector<Item> items;
  for (auto& kv : entry.nodes) {
    const uint64_t* st = stake_of(stakes, kv.first);
    items.push_back({kv.first, kv.second, st ? *st : 0, tie_rank(kv.first)});
  }
  std::sort(items.begin(), items.end(), [](const Item& a, const Item& b) {
    if (a.score != b.score) return a.score > b.score;
    if (a.stake != b.stake) return a.stake > b.stake;
    return a.rank < b.rank;
  });
  uint64_t acc = 0;
  bool skipping = true;
  for (size_t i = 0; i < items.size(); ++i) {
    uint64_t old = acc;
    acc = (acc + items[i].stake < acc) ? UINT64_MAX : acc + items[i].stake;  // saturating_add
    if (i < min_ingress_nodes) continue;                                    // skip(min_ingress_nodes)
    if (skipping && old < min_ingress_stake) continue;                      // skip_while(stake < min)
    skipping = false;
    if (items[i].node != origin) out.push_back(items[i].node);
  }
  return out;
}

}  // namespace orc
