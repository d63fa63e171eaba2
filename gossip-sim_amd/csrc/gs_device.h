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
constexpr uint32_t ERR_INBOUND = 1u, ERR_CACHE = 2u, ERR_DEPTH = 4u;
constexpr uint32_t CACHE_CAP = 96;   // >= 50 zero-score + 2 timely keys x 20 rounds (received_cache.rs:78-97)
constexpr uint32_t CACHE_LIMIT = 50; // ReceivedCacheEntry::CAPACITY
constexpr uint32_t MIN_NUM_UPSERTS = 20;
constexpr uint32_t PRUNED_FLAG = 0x80u;

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

// One WeightedShuffle step over the remaining candidates: given v uniform in
// [0, sum of remaining weights), return the smallest remaining index whose
// running prefix exceeds v. `rem` (ascending) lists excluded ids with weights;
// walking them in order shifts v past each excluded weight lying before the
// answer, so a single search over the full prefix array finds it.
template <int R>
__device__ inline uint32_t shuffle_pick(const uint64_t* __restrict__ P, uint32_t n, uint64_t v,
                                        const uint32_t (&rem)[R], const uint64_t (&remw)[R], int nr) {
  uint64_t x = v;
  for (int i = 0; i < nr; ++i) {
    if (P[rem[i]] <= x) x += remw[i];
    else break;
  }
  return prefix_search(P, n, x);
}

template <int R>
__device__ inline void rem_insert(uint32_t (&rem)[R], uint64_t (&remw)[R], int& nr, uint32_t id, uint64_t w) {
  int i = nr;
  while (i > 0 && rem[i - 1] > id) { rem[i] = rem[i - 1]; remw[i] = remw[i - 1]; --i; }
  rem[i] = id; remw[i] = w;
  ++nr;
}

}  // namespace gs
