// oracle/oracle_core.h -- TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of gregcusack/gossip-sim's push-propagation path, used as the
// parity checker for the HIP engine (tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg only). Nothing in the product links this code.
//
// The reference is Rust and cannot be built in this image (no cargo/rustc, the
// solana-* git dependencies are not vendored). This file
// restates, with the same data-structure shapes as the reference (maps keyed by
// 32-byte pubkeys, insertion-ordered active-set entries, per-origin received
// caches), the following reference code:
//   push_active_set.rs:38-196   PushActiveSet / PushActiveSetEntry / get_stake_bucket
//   received_cache.rs:19-131    ReceivedCache / ReceivedCacheEntry
//   gossip.rs:483-771, 805-842  Cluster::{run_gossip, consume_messages, send_prunes,
//                               prune_connections, chance_to_rotate, fail_nodes}, Node
//   gossip_stats.rs             HopsStat, StatCollection, Histogram, trackers, stranded stats
//   gossip_main.rs:263-290,425-647  init, origin rank, the per-iteration loop, finalize
// plus the third-party semantics the reference calls into (pinned versions in
// Cargo.lock): rand_chacha 0.2.2 ChaChaRng, rand 0.7.3 UniformInt<u64>::sample_single
// and Standard f64, solana-gossip 1.16 (fdf7bdae) WeightedShuffle, indexmap 1.9
// insertion order / shift_remove_index(0), solana-bloom AtomicBloom replaced by an
// exact set (bloom false positives: parity unpinned), solana-sdk Pubkey ordering
// and new_unique().
//
// Two RNG modes:
//   COMPAT  -- ChaCha20 stream shared across nodes, candidates sorted by Pubkey bytes
//              (the reference's test=true path). Pinned by the reference's own KATs.
//   PHILOX  -- the build's deterministic contract (DESIGN.md "Determinism contract"):
//              Philox4x32-10 substreams keyed by (seed, purpose, node, round/bucket),
//              candidates in node-id (= base58 rank) order.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>
#include <array>
#include <unordered_map>
#include <unordered_set>
#include <deque>
#include <map>
#include <optional>
#include <functional>

namespace orc {

// ---------------------------------------------------------------- Pubkey ----
struct Pubkey {
  uint8_t b[32];
  bool operator==(const Pubkey& o) const { return std::memcmp(b, o.b, 32) == 0; }
  bool operator!=(const Pubkey& o) const { return !(*this == o); }
  // solana_sdk::Pubkey derives Ord over its [u8; 32]: lexicographic bytes.
  bool operator<(const Pubkey& o) const { return std::memcmp(b, o.b, 32) < 0; }
};
struct PubkeyHash {  // (iteration order of these maps never decides a result: the reference's is random)
  static uint64_t mix(uint64_t x) {  // splitmix64 finalizer
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
  }
  size_t operator()(const Pubkey& p) const {
    uint64_t w[4];
    std::memcpy(w, p.b, 32);
    return (size_t)mix(w[0] ^ mix(w[1] ^ mix(w[2] ^ mix(w[3]))));
  }
};
template <class V> using PkMap = std::unordered_map<Pubkey, V, PubkeyHash>;
using PkSet = std::unordered_set<Pubkey, PubkeyHash>;

std::string base58(const Pubkey& p);   // bs58 encoding of the 32 bytes (Pubkey Display)
Pubkey pubkey_from_counter(uint64_t i); // Pubkey::new_unique(): BE counter in bytes 0..8

// ------------------------------------------------------------------- RNG ----
struct Rng {
  virtual uint64_t next_u64() = 0;
  virtual ~Rng() {}
};

// rand_chacha 0.2.2 ChaChaRng::from_seed: ChaCha20, 64-bit block counter in state
// words 12-13 starting at 0, 64-bit stream id (words 14-15) = 0; output words in
// order, next_u64 = lo | hi << 32.
struct ChaCha20Rng : Rng {
  uint32_t key[8];
  uint64_t counter = 0;
  uint32_t buf[16];
  int idx = 16;
  explicit ChaCha20Rng(const uint8_t seed[32]);
  uint32_t next_u32();
  uint64_t next_u64() override;
};

// Philox4x32-10 (Random123). Stream (seed, purpose, a, b): key = seed split in two
// 32-bit halves, counter = {block j, a, b, purpose}; block j yields the u64s
// x0|x1<<32 then x2|x3<<32.
void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]);
struct PhiloxStream : Rng {
  uint32_t key[2];
  uint32_t a, b, purpose;
  uint32_t block = 0;
  uint32_t out[4];
  int idx = 4;
  PhiloxStream(uint64_t seed, uint32_t purpose, uint32_t a, uint32_t b);
  uint64_t next_u64() override;
};
enum Purpose : uint32_t {
  P_INIT = 1, P_ROTATE = 2, P_DECIDE = 3, P_FAIL = 4, P_STAKE = 5, P_PUBKEY = 6
};

// rand 0.7.3 UniformInt<u64>::sample_single(low, high): widening-multiply rejection.
uint64_t sample_single_u64(uint64_t low, uint64_t high, Rng& rng);
// rand 0.7.3 Standard for f64: (next_u64 >> 11) * 2^-53.
double gen_f64(Rng& rng);

// --------------------------------------------------------------- buckets ----
constexpr int NUM_PUSH_ACTIVE_SET_ENTRIES = 25;
constexpr uint64_t LAMPORTS_PER_SOL = 1000000000ull;
// push_active_set.rs:190-196; None -> 0.
int get_stake_bucket(const uint64_t* stake);

using Stakes = PkMap<uint64_t>;
// Option<&u64>::min(Option<&u64>) as used at push_active_set.rs:48,68 and
// received_cache.rs:113 (None < Some).
const uint64_t* opt_min(const uint64_t* a, const uint64_t* b);
inline const uint64_t* stake_of(const Stakes& s, const Pubkey& k) {
  auto it = s.find(k);
  return it == s.end() ? nullptr : &it->second;
}

// ------------------------------------------------------ WeightedShuffle ----
// solana-gossip 1.16 WeightedShuffle semantics: each step draws
// v = sample_single(0, sum of remaining weights) and yields the smallest index
// whose running prefix of remaining weights exceeds v, removing it; zero weights
// are yielded last in swap_remove order.
struct WeightedShuffle {
  std::vector<uint64_t> w;
  uint64_t sum = 0;
  std::vector<size_t> zeros;
  explicit WeightedShuffle(const std::vector<uint64_t>& weights);
  std::optional<size_t> next(Rng& rng);
};

// ------------------------------------------------------- PushActiveSet ----
struct PushActiveSetEntry {
  std::vector<Pubkey> keys;        // IndexMap insertion order
  // Exact stand-in for each key's AtomicBloom<Pubkey>: the key itself (bloom.add(node),
  // push_active_set.rs:179) plus the origins pruned for it, kept as (key index, origin)
  // pairs (a per-key set cost ~2 KB per entry, which 1M-node checks cannot afford).
  std::vector<std::pair<uint32_t, Pubkey>> pruned;
  long index_of(const Pubkey& node) const;  // IndexMap::get_index_of
  bool filter_contains(size_t i, const Pubkey& x) const;
  std::vector<Pubkey> get_nodes(const Pubkey& origin, const std::function<bool(const Pubkey&)>& force) const;
  void prune(const Pubkey& node, const Pubkey& origin);
  void rotate(Rng& rng, size_t size, const std::vector<Pubkey>& nodes, const std::vector<uint64_t>& weights);
};

struct PushActiveSet {
  std::array<PushActiveSetEntry, NUM_PUSH_ACTIVE_SET_ENTRIES> e;
  std::vector<Pubkey> get_nodes(const Pubkey& self, const Pubkey& origin, const Stakes& stakes) const;
  void prune(const Pubkey& self, const Pubkey& node, const std::vector<Pubkey>& origins, const Stakes& stakes);
  // rng_for_k(k) returns the generator used for entry k: the same shared stream in
  // COMPAT mode (as the reference), a fresh Philox substream in PHILOX mode.
  void rotate(const std::function<Rng&(int)>& rng_for_k, size_t size, const std::vector<Pubkey>& nodes,
              const Stakes& stakes);
};

// ------------------------------------------------------- ReceivedCache ----
struct ReceivedCacheEntry {
  PkMap<uint64_t> nodes;  // node -> score
  uint64_t num_upserts = 0;
  static constexpr size_t CAPACITY = 50;
  static constexpr size_t NUM_DUPS_THRESHOLD = 2;
  void record(const Pubkey& node, size_t num_dups);
};
struct ReceivedCache {
  static constexpr uint64_t MIN_NUM_UPSERTS = 20;
  PkMap<ReceivedCacheEntry> m;  // LRU capacity 16384 (gossip.rs:906) is never reached
  void record(const Pubkey& origin, const Pubkey& node, size_t num_dups);
  // Tie order among equal (score, stake) is unspecified in the reference
  // (sorted_unstable over HashMap order); canonical order here: ascending rank(),
  // i.e. base58 order, supplied by the caller.
  std::vector<Pubkey> prune(const Pubkey& self, const Pubkey& origin, double stake_threshold,
                            size_t min_ingress_nodes, const Stakes& stakes,
                            const std::function<uint64_t(const Pubkey&)>& tie_rank);
};

}  // namespace orc
