// gs_device.h -- device-side building blocks of the push-propagation engine.
//
// Philox4x32-10 substreams, rand-0.7-compatible u64 sampling and the exact
// weighted-shuffle draw used by active-set rotation (push_active_set.rs:153-187
// with solana-gossip's WeightedShuffle). Everything here is integer arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

constexpr int NB = 25;  // NUM_PUSH_ACTIVE_SET_ENTRIES (push_active_set.rs:11)
constexpr uint32_t P_INIT = 1, P_ROTATE = 2, P_DECIDE = 3, P_FAIL = 4;
constexpr uint32_t ERR_INBOUND = 1u, ERR_CACHE = 2u, ERR_DEPTH = 4u, ERR_MV_CAP = 8u, ERR_SYNC = 16u;
// which multi-source BFS capacity ERR_MV_CAP hit (reported with it)
constexpr uint32_t ERR_MVD_ROWS = 0x1000u, ERR_MVD_AREA = 0x2000u, ERR_MVD_POOL = 0x4000u, ERR_MVD_Q = 0x8000u,
                   ERR_MVD_CSR = 0x10000u;
// a frontier-exchange message outgrew its fixed-capacity slot (the asynchronous level loop:
// not an error of the engine -- gs_part_xbfs_async_status reports and clears it, and the
// group's BFS is redone with exact sizes)
constexpr uint32_t ERR_MVX_CAP = 0x20000u;
constexpr uint32_t CACHE_CAP = 96;   // >= 50 zero-score + 2 timely keys x 20 rounds (received_cache.rs:78-97)
constexpr uint32_t CACHE_LIMIT = 50; // ReceivedCacheEntry::CAPACITY
constexpr uint32_t MIN_NUM_UPSERTS = 20;
constexpr uint32_t PRUNED_FLAG = 0x80u;

// A received-cache slot is one u32 word: node id (24 bits) | score (7 bits) << 24 |
// pruned flag << 31. Key and score travel in one load and one store, so a score
// increment is a plain store of a word the lookup already holds.
constexpr uint32_t CK_ID = 0xFFFFFFu;
__host__ __device__ inline uint32_t ck_id(uint32_t w) { return w & CK_ID; }
__host__ __device__ inline uint32_t ck_score(uint32_t w) { return (w >> 24) & 0x7Fu; }
__host__ __device__ inline bool ck_pruned(uint32_t w) { return (w >> 31) != 0; }
// score_flag: score (<= 0x7F) | PRUNED_FLAG
__host__ __device__ inline uint32_t ck_make(uint32_t id, uint32_t score_flag) { return id | (score_flag << 24); }
// the slot with score + 1, saturating at 0x7F (received_cache.rs:88-90); clears the pruned flag
__host__ __device__ inline uint32_t ck_bump(uint32_t w) {
  const uint32_t s = ck_score(w);
  return ck_make(ck_id(w), s < 0x7Fu ? s + 1 : 0x7Fu);
}

// Debug builds (make DEBUG_BOUNDS=1): every guarded index is checked; a violation
// prints, raises ERR_BOUNDS and the access is skipped instead of faulting.
constexpr uint32_t ERR_BOUNDS = 0x100u;
#ifdef GS_DEBUG_BOUNDS
#define GS_OOB(idx, size, err, tag)                                                                     \
  ((size_t)(idx) >= (size_t)(size)                                                                      \
       ? (printf("GS_OOB %s: %llu >= %llu\n", tag, (unsigned long long)(idx), (unsigned long long)(size)), \
          atomicOr((err), ERR_BOUNDS), true)                                                            \
       : false)
#else
#define GS_OOB(idx, size, err, tag) false
#endif

__host__ __device__ inline uint64_t weight(int k, int bucket) {
  // (min(bucket, k) + 1)^2 (push_active_set.rs:97-111)
  uint64_t b = (uint64_t)(bucket < k ? bucket : k) + 1;
  return b * b;
}

__host__ __device__ inline int stake_bucket(uint64_t stake) {  // push_active_set.rs:190-196
  uint64_t s = stake / 1000000000ull;
  int bits = 0;
  while (s) { ++bits; s >>= 1; }
  return bits < NB - 1 ? bits : NB - 1;
}

// Philox4x32-10 substream: key = seed halves, counter = {block, a, b, purpose}.
struct Philox {
  uint32_t k0, k1, a, b, p, blk;
  uint32_t o0, o1, o2, o3;
  int idx;
  __host__ __device__ Philox(uint64_t seed, uint32_t purpose, uint32_t a_, uint32_t b_)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), a(a_), b(b_), p(purpose), blk(0), o0(0), o1(0), o2(0),
        o3(0), idx(4) {}
  __host__ __device__ void refill() {
    uint32_t c0 = blk, c1 = a, c2 = b, c3 = p, x0 = k0, x1 = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      if (r) { x0 += 0x9E3779B9u; x1 += 0xBB67AE85u; }
      uint64_t m0 = (uint64_t)0xD2511F53u * c0;
      uint64_t m1 = (uint64_t)0xCD9E8D57u * c2;
      uint32_t n0 = (uint32_t)(m1 >> 32) ^ c1 ^ x0;
      uint32_t n2 = (uint32_t)(m0 >> 32) ^ c3 ^ x1;
      c0 = n0; c1 = (uint32_t)m1; c2 = n2; c3 = (uint32_t)m0;
    }
    o0 = c0; o1 = c1; o2 = c2; o3 = c3;
    ++blk;
    idx = 0;
  }
  __host__ __device__ uint64_t next() {
    if (idx >= 4) refill();
    uint64_t v = idx == 0 ? ((uint64_t)o0 | ((uint64_t)o1 << 32)) : ((uint64_t)o2 | ((uint64_t)o3 << 32));
    idx += 2;
    return v;
  }
};

__device__ inline uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// rand 0.7 UniformInt<u64>::sample_single(0, range).
__device__ inline uint64_t sample_below(uint64_t range, Philox& s) {
  int lz = __clzll((long long)range);
  uint64_t zone = (range << lz) - 1;
  for (;;) {
    uint64_t v = s.next();
    uint64_t lo = v * range;
    if (lo <= zone) return mulhi64(v, range);
  }
}

// rand 0.7 Standard f64.
__host__ __device__ inline double unit_f64(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

// Smallest c in [0, n) with P[c + 1] > x (P = prefix sums of weights, P[0] = 0).
__device__ inline uint32_t prefix_search(const uint64_t* __restrict__ P, uint32_t n, uint64_t x) {
  uint32_t lo = 0, hi = n - 1;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (P[mid + 1] > x) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// prefix_search through an index table: IX[j] = the answer for x_j = floor(total * j / 2^L)
// (j <= 2^L), so the answer for x lies in [IX[j], IX[j + 1]] with j = floor(x * 2^L / total)
// (answers are monotone in x and x_j <= x <= x_{j+1}): one table load, then a short
// search of P instead of a search of the whole prefix array.
__host__ __device__ inline uint32_t ix_log(uint32_t n) {
  uint32_t l = 0;
  while ((1u << l) < n) ++l;
  l = l > 3 ? l - 3 : 0;  // ~8 candidates per table entry: ~3 steps of the search in P
  return l < 4 ? 4 : (l > 20 ? 20 : l);
}
__host__ __device__ inline uint32_t ix_count(uint32_t n) { return (1u << ix_log(n)) + 1; }
__device__ inline uint32_t prefix_search_ix(const uint64_t* __restrict__ P, const uint32_t* __restrict__ IX,
                                            uint32_t L, uint64_t total, uint64_t x) {
  const uint32_t j = (uint32_t)((x << L) / total);  // x < total <= 625 * 2^24, L <= 20: no overflow
  uint32_t lo = IX[j], hi = IX[j + 1];
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (P[mid + 1] > x) hi = mid; else lo = mid + 1;
  }
  return lo;
}

// One WeightedShuffle step over the remaining candidates: given v uniform in
// [0, sum of remaining weights), return the smallest remaining index whose
// running prefix exceeds v. `rem` (ascending) lists excluded ids with weights;
// walking them in order shifts v past each excluded weight lying before the
// answer, so a single search over the full prefix array finds it.
template <int R>
__device__ inline uint32_t shuffle_pick(const uint64_t* __restrict__ P, const uint32_t* __restrict__ IX, uint32_t L,
                                        uint64_t total, uint64_t v, const uint32_t (&rem)[R],
                                        const uint64_t (&remw)[R], int nr) {
  uint64_t x = v;
  for (int i = 0; i < nr; ++i) {
    if (P[rem[i]] <= x) x += remw[i];
    else break;
  }
  return prefix_search_ix(P, IX, L, total, x);
}

template <int R>
__device__ inline void rem_insert(uint32_t (&rem)[R], uint64_t (&remw)[R], int& nr, uint32_t id, uint64_t w) {
  int i = nr;
  while (i > 0 && rem[i - 1] > id) { rem[i] = rem[i - 1]; remw[i] = remw[i - 1]; --i; }
  rem[i] = id; remw[i] = w;
  ++nr;
}

// ------------------------------------------------ shared kernel helpers ----
template <int ASZP>
__device__ inline void load_row(const uint32_t* __restrict__ src, uint32_t (&row)[ASZP]) {
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int q = 0; q < ASZP / 4; ++q) {
    const uint4 x = s4[q];
    row[4 * q] = x.x; row[4 * q + 1] = x.y; row[4 * q + 2] = x.z; row[4 * q + 3] = x.w;
  }
}

// Own-bucket entry row of node u (the entry it uses for every origin whose bucket is at
// least its own, push_active_set.rs:38-52): own[u] = peers[u][bucket[u]] and, in word
// ASZP, hl | bucket << 16; with fcls (the multi-source BFS) words ASZP + 1 .. hold the
// peers' failure classes, one byte each, so a row and its failure test are one line.
template <int ASZP>
__device__ inline void own_row(const uint8_t* __restrict__ bucket, const uint32_t* __restrict__ peers,
                               const uint16_t* __restrict__ hl, uint32_t ORW, const uint8_t* __restrict__ fcls,
                               uint32_t* __restrict__ own, uint32_t u) {
  const uint32_t b = bucket[u];
  const uint32_t ent = u * NB + b;
  uint32_t row[ASZP];
  load_row<ASZP>(peers + (size_t)ent * ASZP, row);
  uint32_t* dst = own + (size_t)u * ORW;
  uint4* d4 = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int q = 0; q < ASZP / 4; ++q) d4[q] = make_uint4(row[4 * q], row[4 * q + 1], row[4 * q + 2], row[4 * q + 3]);
  dst[ASZP] = (uint32_t)hl[ent] | (b << 16);
  if (fcls) {
#pragma unroll
    for (int q = 0; q < ASZP / 4; ++q)
      dst[ASZP + 1 + q] = (uint32_t)fcls[row[4 * q]] | ((uint32_t)fcls[row[4 * q + 1]] << 8) |
                          ((uint32_t)fcls[row[4 * q + 2]] << 16) | ((uint32_t)fcls[row[4 * q + 3]] << 24);
  }
}

// PushActiveSet::get_nodes(..).take(fanout) (gossip.rs:527-536, push_active_set.rs:128-141):
// the first `fanout` peers in FIFO order whose filter lacks the origin -- i.e.
// not pruned for this slot and not the origin itself. Returns physical ring slots.
template <int ASZP>
__device__ inline uint32_t taken_slots(const uint32_t (&row)[ASZP], uint32_t head, uint32_t len, uint32_t S,
                                       uint32_t pmask, uint32_t origin, uint32_t fanout) {
  if constexpr (ASZP < 32) {  // S < 32: every ring mask fits a u32, with few VALU ops
    const uint32_t full = (1u << S) - 1u;
    const uint32_t lm = len >= S ? full : (1u << len) - 1u;            // ring positions [0, len)
    const uint32_t valid = ((lm << head) | (lm >> (S - head))) & full;  // their physical slots
    uint32_t om = 0;
#pragma unroll
    for (int s = 0; s < ASZP; ++s) om |= (uint32_t)(row[s] == origin) << s;
    const uint32_t elig = valid & ~pmask & ~om;
    uint32_t fifo = ((elig >> head) | (elig << (S - head))) & full;  // bit = ring position (FIFO order)
    if ((uint32_t)__popc(fifo) > fanout) {
      uint32_t sel = 0;
      for (uint32_t t = 0; t < fanout; ++t) {
        const uint32_t low = fifo & (~fifo + 1u);
        sel |= low;
        fifo ^= low;
      }
      fifo = sel;
    }
    return ((fifo << head) | (fifo >> (S - head))) & full;
  }
  uint32_t elig = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    const uint32_t pos = (uint32_t)s >= head ? (uint32_t)s - head : (uint32_t)s + S - head;
    const bool ok = (uint32_t)s < S && pos < len && !((pmask >> s) & 1u) && row[s] != origin;
    elig |= (uint32_t)ok << s;
  }
  const uint64_t full = (S == 64) ? ~0ull : ((1ull << S) - 1);
  const uint64_t e64 = elig;
  uint64_t fifo = ((e64 >> head) | (e64 << (S - head))) & full;
  if ((uint32_t)__popcll(fifo) > fanout) {
    uint64_t sel = 0;
    for (uint32_t t = 0; t < fanout; ++t) {
      const uint64_t low = fifo & (~fifo + 1);
      sel |= low;
      fifo ^= low;
    }
    fifo = sel;
  }
  return (uint32_t)(((fifo << head) | (fifo >> (S - head))) & full);
}

__device__ inline uint32_t lane_id() { return __lane_id(); }

// Atomics for words that only ONE workgroup touches during the kernel (the single-
// workgroup level kernels): workgroup scope, so they execute in the XCD's L2 instead of
// at the memory side (a device-scope returning atomic is a fabric round trip: the small
// levels' atomics at C4 took ~10 us per level). Data from earlier kernels is visible and
// the results reach later kernels through the kernel-boundary write-back as usual.
__device__ inline uint32_t atomic_or_wg(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ inline uint32_t atomic_add_wg(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Inclusive prefix sum over the 64 lanes of a wave (all lanes must be active).
__device__ inline uint32_t wave_incl_scan(uint32_t x) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, off);
    if (lane >= (uint32_t)off) x += y;
  }
  return x;
}

// u64 -> f64 -> u64 of received_cache.rs:114, saturating like Rust's `as u64`.
__device__ inline uint64_t min_ingress_stake(uint64_t stake, double thr) {
  const double x = (double)stake * thr;
  if (!(x > 0.0)) return 0;
  if (x >= 18446744073709551616.0) return ~0ull;
  return (uint64_t)x;
}

__device__ inline uint64_t sat_add(uint64_t a, uint64_t b) { return a + b < a ? ~0ull : a + b; }

// Maximum of x (< 2^BITS) over the wave's ACTIVE lanes, wave-uniform. Built from
// ballots, which see exactly the active lanes; a shuffle butterfly would read
// stale registers of lanes switched off by an enclosing divergent branch.
template <int BITS = 5>
__device__ inline uint32_t active_max(uint32_t x) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t b = 1u << (BITS - 1); b; b >>= 1)
    if (__ballot(x >= m + b)) m += b;
  return __builtin_amdgcn_readfirstlane(m);
}
__device__ inline uint32_t active_max_small(uint32_t x) { return active_max<5>(x); }

__device__ inline void cswap(uint32_t& x, uint32_t& y) {
  const uint32_t lo = min(x, y), hi = max(x, y);
  x = lo;
  y = hi;
}

// Batcher odd-even merge sort of r[0, NS) (NS a power of two), register-resident:
// 63 comparators for 16 keys, 191 for 32. W < NS: r[W, NS) hold ~0 (the largest key), which
// no comparator moves, so the comparators reaching past W are dropped (the first W keys
// are sorted with fewer).
template <int NS, int M, int W = NS>
__device__ inline void sort_net(uint32_t (&r)[M]) {
  static_assert(NS <= M && (NS & (NS - 1)) == 0 && W <= NS, "power-of-two prefix");
#pragma unroll
  for (int p = 1; p < NS; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j + k < NS; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k; ++i)
          if (i + j + k < W && (i + j) / (2 * p) == (i + j + k) / (2 * p)) cswap(r[i + j], r[i + j + k]);
}
__device__ inline void sort16(uint32_t (&r)[16]) { sort_net<16>(r); }

// One thread per (rotating node, entry k). On a full entry the reference's loop
// appends the first drawn peer that is not present, draws once more and breaks,
// then drops the oldest: the ring's head slot is overwritten.
// (rotating node rot_list[gid / NB], entry gid % NB): PushActiveSetEntry::rotate.
template <int ASZP>
__device__ inline void rotate_entry(const uint8_t* __restrict__ bucket, const uint64_t* __restrict__ P,
                                    const uint32_t* __restrict__ IX, uint32_t* __restrict__ peers,
                                    uint16_t* __restrict__ hl, const uint32_t* __restrict__ rot_list,
                                    uint32_t* __restrict__ rot_changed, uint32_t N, uint32_t size, uint64_t seed,
                                    uint32_t round, uint32_t gid) {
    const uint32_t i = gid / NB, k = gid % NB;
  const uint32_t u = rot_list[i];
  const uint32_t ent = u * NB + k;
  const uint16_t hv = hl[ent];
  uint32_t head = hv & 0xFF, L = hv >> 8;
  const uint32_t S = size;
  uint32_t* row = peers + (size_t)ent * ASZP;
  const uint64_t* Pk = P + (size_t)k * (N + 1);
  const uint32_t LX = ix_log(N);
  const uint32_t* IXk = IX + (size_t)k * ix_count(N);
  constexpr int R = ASZP + 2;
  uint32_t rem[R];
  uint64_t remw[R];
  int nr = 0;
  const uint64_t wself = weight(k, bucket[u]);
  rem_insert(rem, remw, nr, u, wself);
  const uint64_t total = Pk[N];
  uint64_t left = total - wself;
  Philox s(seed, P_ROTATE, u, (round << 5) | k);
  uint32_t changed = 0;
  for (uint32_t drawn = 0; drawn + 1 < N; ++drawn) {
    const uint64_t v = sample_below(left, s);
    const uint32_t c = shuffle_pick(Pk, IXk, LX, total, v, rem, remw, nr);
    const uint64_t wc = weight(k, bucket[c]);
    left -= wc;
    if (nr < R) rem_insert(rem, remw, nr, c, wc);
    bool present = false;
    for (uint32_t j = 0; j < L; ++j) {
      uint32_t slot = head + j;
      if (slot >= S) slot -= S;
      present |= row[slot] == c;
    }
    if (present) continue;
    if (L < S) {
      uint32_t slot = head + L;
      if (slot >= S) slot -= S;
      row[slot] = c;
      ++L;
      changed |= 1u << slot;
      continue;
    }
    row[head] = c;
    changed |= 1u << head;
    head = head + 1 == S ? 0 : head + 1;
    break;
  }
  hl[ent] = (uint16_t)((L << 8) | head);
  rot_changed[ent] = changed;
}


}  // namespace gs
