// gs_consume_dev.h -- the received-cache update of one (slot, node) pair:
// consume_messages + ReceivedCache::record (gossip.rs:618-653, received_cache.rs:27-36,
// 83-98) given the pair's inbound records (hop << 24 | src) in rank order. Shared by the
// level-synchronous consume (gs_consume_g.hip, records from inbound rows in HBM) and the
// multi-source BFS's fused gather + consume (gs_bfs_multi.hip, records from an LDS CSR).
//
// Cache rows are ckey[i * PAIRS + q] (i < len), coalesced across the lanes' pairs q.
#pragma once
#include "gs_device.h"

namespace gs {

template <class T>
__device__ inline T ntl(const T* p) { return __builtin_nontemporal_load(p); }

// The first 8 cache rows of the lane's pair (rows >= len are not loaded and read as ~0,
// whose id CK_ID is no node's: n_nodes <= 2^24 - 1): issued before the records are
// sorted, so the sort hides their latency.
__device__ inline void cache_prefetch(const uint32_t* __restrict__ ckey, size_t PAIRS, size_t q, uint32_t len,
                                      uint32_t (&kc)[8]) {
#pragma unroll
  for (int t = 0; t < 8; ++t) kc[t] = (uint32_t)t < len ? ntl(&(ckey + (size_t)t * PAIRS)[q]) : 0xFFFFFFFFu;
}

template <int NC>
__device__ inline void cache_match(uint32_t* __restrict__ ckey, size_t PAIRS, size_t q, const uint32_t (&rid)[16],
                                   uint32_t len, uint32_t wl, const uint32_t (&kc0)[8], bool (&pr)[16], int& idx0,
                                   int& idx1, uint32_t& w0, uint32_t& w1) {
  for (uint32_t i0 = 0; i0 < wl; i0 += 8) {
    uint32_t kc[8];
    if (i0 == 0) {
#pragma unroll
      for (int t = 0; t < 8; ++t) kc[t] = kc0[t];
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) kc[t] = i0 + t < len ? ntl(&(ckey + (size_t)(i0 + t) * PAIRS)[q]) : 0xFFFFFFFFu;
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t i = i0 + t;
      const uint32_t k = ck_id(kc[t]);  // CK_ID past len: matches no record id
#pragma unroll
      for (int j = 0; j < NC; ++j) pr[j] = pr[j] || rid[j] == k;
      if (rid[0] == k) { idx0 = (int)i; w0 = kc[t]; }
      if (rid[1] == k) { idx1 = (int)i; w1 = kc[t]; }
    }
  }
}

// Register path: rk[0..c) sorted ascending, rk[c..16) = ~0 (1 <= c <= 16); wc = the
// wave's largest c (selects the match width); kc0 = cache_prefetch of the pair. Rank 0
// and 1 are timely (score += 1, inserted regardless of the 50-key cap); later ranks are
// inserted while len < 50. Presence is kept as per-rank lane masks (bool: one compare
// per (key, rank), the OR runs on the scalar unit), the cache rows are streamed 8 at a time.
__device__ inline void cache_update_lane(uint32_t* __restrict__ ckey, size_t PAIRS, size_t q,
                                         const uint32_t (&rk)[16], uint32_t c, uint32_t wc,
                                         const uint32_t (&kc0)[8], uint32_t& len, uint32_t& up, uint32_t& errf) {
  uint32_t rid[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rid[j] = (uint32_t)j < c ? rk[j] & CK_ID : 0xFFFFFFFEu;  // never a cache id
  bool pr[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) pr[j] = false;
  uint32_t w0 = 0, w1 = 0;
  int idx0 = -1, idx1 = -1;
  const uint32_t wl = active_max<7>(len);
  if (wc <= 4) cache_match<4>(ckey, PAIRS, q, rid, len, wl, kc0, pr, idx0, idx1, w0, w1);
  else if (wc <= 8) cache_match<8>(ckey, PAIRS, q, rid, len, wl, kc0, pr, idx0, idx1, w0, w1);
  else if (wc <= 12) cache_match<12>(ckey, PAIRS, q, rid, len, wl, kc0, pr, idx0, idx1, w0, w1);
  else cache_match<16>(ckey, PAIRS, q, rid, len, wl, kc0, pr, idx0, idx1, w0, w1);
  up = up < 255 ? up + 1 : 255;  // rank 0 (received_cache.rs:84-86)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if ((uint32_t)j >= c) break;
    const int idx = j == 0 ? idx0 : idx1;
    if (idx >= 0) {
      (ckey + (size_t)idx * PAIRS)[q] = ck_bump(j == 0 ? w0 : w1);
    } else if (len < CACHE_CAP) {
      (ckey + (size_t)len * PAIRS)[q] = ck_make(rid[j], 1u);
      ++len;
    } else {
      errf |= ERR_CACHE;
    }
  }
#pragma unroll
  for (int j = 2; j < 16; ++j)  // rank order (received_cache.rs:91-97)
    if ((uint32_t)j < c && !pr[j] && len < CACHE_LIMIT) {
      (ckey + (size_t)len * PAIRS)[q] = ck_make(rid[j], 0u);
      ++len;
    }
}

// Sorts rk[0..16) ascending with the narrowest network that covers wc keys (rk[wc..16)
// are ~0). (C5's waves: the largest in-degree of 64 lanes averages 12.5.)
__device__ inline void sort_ranked(uint32_t (&rk)[16], uint32_t wc) {
  if (wc <= 4) sort_net<4>(rk);
  else if (wc <= 8) sort_net<8>(rk);
  else if (wc <= 12) sort_net<16, 16, 12>(rk);
  else sort_net<16>(rk);
}

// Bitonic sort of one key per lane across the wave, ascending by lane.
__device__ inline uint32_t wave_sort(uint32_t key) {
  const uint32_t l = lane_id();
#pragma unroll
  for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t other = (uint32_t)__shfl_xor((int)key, (int)j);
      const bool asc = (l & k) == 0;
      const bool lower = (l & j) == 0;
      key = (lower == asc) ? min(key, other) : max(key, other);
    }
  return key;
}

// Wave path (all lanes on pair q; len/up wave-uniform): lane l holds the rank-l record
// (l < c <= 64, ~0 beyond). scr: >= CACHE_CAP words of this wave's LDS.
__device__ inline void cache_update_wave(uint32_t* __restrict__ ckey, size_t PAIRS, size_t q, uint32_t key,
                                         uint32_t c, uint32_t& len, uint32_t& up, uint32_t* scr, uint32_t& errf) {
  const uint32_t l = lane_id();
  const uint32_t src = key & CK_ID;
  const uint32_t L0 = len;
  for (uint32_t i = l; i < L0; i += 64) scr[i] = (ckey + (size_t)i * PAIRS)[q];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int found = -1;
  if (l < c)
    for (uint32_t i = 0; i < L0; ++i)
      if (ck_id(scr[i]) == src) found = (int)i;
  const bool isnew = l < c && found < 0;
  const uint64_t nb = __ballot(isnew);
  const uint32_t n0 = (uint32_t)(nb & 1u), n1 = (uint32_t)((nb >> 1) & 1u);
  up = up < 255 ? up + 1 : 255;
  if (l < 2 && l < c) {
    if (found >= 0) {
      (ckey + (size_t)found * PAIRS)[q] = ck_bump(scr[found]);
    } else {
      const uint32_t pos = L0 + (l == 1 ? n0 : 0u);
      if (pos < CACHE_CAP) (ckey + (size_t)pos * PAIRS)[q] = ck_make(src, 1u);
      else errf |= ERR_CACHE;
    }
  }
  const uint32_t L1 = min(L0 + n0 + n1, CACHE_CAP);
  const uint64_t rest = nb & ~3ull;
  if (l >= 2 && isnew) {
    const uint32_t pos = L1 + (uint32_t)__popcll(rest & ((1ull << l) - 1));
    if (pos < CACHE_LIMIT) (ckey + (size_t)pos * PAIRS)[q] = ck_make(src, 0u);
  }
  const uint32_t nrest = (uint32_t)__popcll(rest);
  len = L1 + (L1 < CACHE_LIMIT ? min(nrest, CACHE_LIMIT - L1) : 0u);
  __builtin_amdgcn_wave_barrier();  // scr is reused by the wave's next pair
}

// Any c (lane 0 of the wave): next(k, prev) returns the rank-k record (the smallest
// record above prev for k > 0). len/up are broadcast from lane 0.
template <class Next>
__device__ inline void cache_update_serial(uint32_t* __restrict__ ckey, size_t PAIRS, size_t q, uint32_t c,
                                           uint32_t& len, uint32_t& up, uint32_t& errf, Next next) {
  uint32_t ln = len, u = up;
  if (lane_id() == 0) {
    uint32_t prev = 0;
    u = u < 255 ? u + 1 : 255;
    for (uint32_t k = 0; k < c; ++k) {
      const uint32_t best = next(k, prev);
      prev = best;
      const uint32_t src = best & CK_ID;
      int found = -1;
      for (uint32_t i = 0; i < ln; ++i)
        if (ck_id(ckey[(size_t)i * PAIRS + q]) == src) { found = (int)i; break; }
      if (k < 2) {
        if (found >= 0) {
          uint32_t* sp = ckey + (size_t)found * PAIRS + q;
          *sp = ck_bump(*sp);
        } else if (ln < CACHE_CAP) {
          ckey[(size_t)ln * PAIRS + q] = ck_make(src, 1u);
          ++ln;
        } else {
          errf |= ERR_CACHE;
        }
      } else if (found < 0 && ln < CACHE_LIMIT) {
        ckey[(size_t)ln * PAIRS + q] = ck_make(src, 0u);
        ++ln;
      }
    }
  }
  len = (uint32_t)__shfl((int)ln, 0);
  up = (uint32_t)__shfl((int)u, 0);
}

}  // namespace gs
