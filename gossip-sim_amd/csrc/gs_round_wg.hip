// gs_round_wg.hip -- one whole gossip round of one origin slot inside one workgroup.
//
// The per-slot state of a round fits in LDS for clusters up to a few thousand
// nodes (C2: 3,000 nodes -> ~80 KB), so a single kernel runs, per slot:
//   A  Cluster::run_gossip BFS (gossip.rs:494-615): frontier queues, in-degree
//      counters, hop table and each node's push mask in LDS;
//   B  the inbound lists ("orders", gossip.rs:601-607) as an LDS CSR: segment
//      offsets from a wave-aggregated scan of the in-degrees, then every visited
//      node scatters its id into its peers' segments -- the records never touch
//      HBM; per-pair hops/in-degree/egress and the measured-round statistics are
//      written in the same pass;
//   C  consume_messages + ReceivedCache::record (gossip.rs:618-653,
//      received_cache.rs:27-36,83-98): per receiving node, its records sorted by
//      (hop, id) in registers, looked up in the node's cache entry (HBM,
//      slot-major rows, coalesced across lanes);
//   D  send_prunes + ReceivedCache::prune + prune_connections (gossip.rs:657-737,
//      received_cache.rs:38-63,100-131) for the entries that reached 20 upserts:
//      (score, stake) order as one 31-bit key ((127 - score) << 24 | stake rank)
//      sorted in registers, pre-add cumulative stake, prune bits set in the
//      prunees' masks;
//   E  the round summary (gossip_main.rs:480-514): hop histogram, stranded
//      count/stake order statistics from an LDS bitmap over stake rank.
// In-degree > 16 or cache entries > 32 keys take a wave-cooperative path
// (one wave per node) so a few heavy nodes do not serialize their wave.
#include <type_traits>

#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

#ifndef RWG_THREADS_N
#define RWG_THREADS_N 768  // 12 waves: 2 workgroups per CU (LDS) = 6 waves per SIMD (VGPR budget 80)
#endif
#ifndef RWG_MIN_WAVES
#define RWG_MIN_WAVES (RWG_THREADS_N / 128)  // waves per SIMD at 2 workgroups per CU (the LDS limit at C2)
#endif
#ifndef GS_NT_STORES
#define GS_NT_STORES 1
#endif
constexpr uint32_t RWG_THREADS = RWG_THREADS_N;
constexpr uint32_t RWG_WAVES = RWG_THREADS / 64;
// Largest N whose consume CSR is staged in registers (BASELINE C2's 3,000 nodes fit);
// larger N take the LDS-staged path. tests/test_gpu_parity.py (fused_vs_split at
// n = 3500) covers both sides of it. Only the default 768-thread build is parity-checked.
constexpr uint32_t RWG_CSR_REG_NODES = 3072;
constexpr uint32_t CSR_NPT = (RWG_CSR_REG_NODES + RWG_THREADS - 1) / RWG_THREADS;  // nodes per thread
static_assert(CSR_NPT * RWG_THREADS >= RWG_CSR_REG_NODES, "register-staged CSR covers its node bound");
constexpr uint32_t RWG_SCR = 128;  // per-wave LDS scratch (u32): staged cache keys / prune keys
constexpr uint32_t LANE_C = 16;    // register path: in-degree <= 16
#ifndef RWG_IN
#define RWG_IN 4  // nodes per trip of the setup loop (C2: 3,000 nodes = 4 per thread)
#endif
constexpr int LANE_L = 16;         // register prune path: cache entry <= 16 keys (the wave path
                                   // takes longer entries; at prune time they are rare)

struct RoundArgs {
  const uint64_t* stake;
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
  const uint32_t* frank;
  const uint32_t* srank;
  const uint32_t* by_srank;
  const uint32_t* prank;     // rank by (stake desc, id asc): the prune order's tie-broken stake key
  const uint32_t* by_prank;
  const uint64_t* pstake;    // stake by prune rank
  const uint4* rinfo;        // by prune rank: {node id, 0, stake lo, stake hi}
  const uint32_t* origin;
  const uint8_t* obkt;
  const uint32_t* nfail;
  const uint32_t* min_ingress;
  const double* thr;
  uint32_t* slot_prunes;
  uint8_t* hops;
  uint32_t* cnt;
  uint32_t* mask;
  uint32_t* cmeta;
  uint32_t* ckey;  // [CACHE_CAP][PAIRS] slot words (ck_make)
  uint8_t* egress;
  uint8_t* prune_round;
  uint32_t* egress_acc;
  uint32_t* ingress_acc;
  uint32_t* prune_acc;
  uint32_t* strand;
  uint64_t* hist_acc;
  gs_round_summary* sum;  // this round's row [S] of the summary ring (record only)
  // the last rotation's pending prune-bit clear (null when none): replaced ring slots
  // of rotated node u's entry k are rot_changed[u * 25 + k]
  const uint32_t* rot_list;
  const uint32_t* rot_count;
  const uint32_t* rot_changed;
  // rotation ahead (rot_on): workgroup 0 runs Cluster::chance_to_rotate of round rround on
  // the other row buffer (rpeers / rhl), after copying the previous ahead rotation's
  // entries (plist / pcount) into it from the current one
  uint32_t rot_on;
  const uint64_t* P;
  const uint32_t* IX;
  uint32_t* rpeers;
  uint16_t* rhl;
  uint32_t* rlist;
  uint32_t* rcount;
  uint32_t* rchanged;
  const uint32_t* plist;
  const uint32_t* pcount;
  uint64_t seed;
  double rp;
  uint32_t rround;
  uint32_t* err;
  unsigned long long* phase_clk;  // optional: per-phase clock sums (thread 0 of each workgroup)
  uint32_t wave_c_max;            // in-degree bound of the wave consume path (64; 24 for path coverage)
  uint32_t N, S, ASZ, fanout, fcap;
  size_t PAIRS;
  int record;
};

// Phase clock: thread 0 adds the time since the last mark to phase_clk[ph].
#define RWG_MARK(ph)                                                              \
  do {                                                                            \
    if (PROF && a.phase_clk && tid == 0) {                                        \
      const unsigned long long now_ = wall_clock64();                             \
      atomicAdd(&a.phase_clk[ph], now_ - t_mark);                                 \
      t_mark = now_;                                                              \
    }                                                                             \
  } while (0)

// LDS carve-up (byte offsets), shared by the host's size query and the kernel.
struct RwgLayout {
  uint32_t ctrl, hist, scr, cnt, qo, pm, mk, eg, nl, hops, bm, rec, total;
};
// pmw: bytes per push mask (2 when the ring has <= 16 slots); offw: bytes per segment
// offset (2 when every round's inbound records, <= fcap * N, fit in a u16 index)
__host__ __device__ inline RwgLayout rwg_layout(uint32_t N, uint32_t fcap, uint32_t pmw, uint32_t offw) {
  RwgLayout L;
  uint32_t o = 0;
  L.ctrl = o; o += 32 * 4;
  L.hist = o; o += 256 * 4;
  L.scr = o;  o += RWG_WAVES * RWG_SCR * 4;
  L.cnt = o;  o += 4 * ((N + 1) / 2);           // in-degree u16 (atomics on the containing u32)
  L.qo = o;   o += (offw * N + 3) & ~3u;        // the BFS queue u16[N] (each node enters once, levels
                                                //   are consecutive ranges), then segment ends
  L.pm = o;   o += (pmw * N + 3) & ~3u;         // push masks, then the heavy-node list u16[N]
  L.mk = o;   o += (pmw * N + 3) & ~3u;         // the slot's prune masks: staged for the BFS, prunes
                                                //   applied here, written back after a prune round
  L.eg = o;   o += (N + 3) & ~3u;               // egress per node (popcount of the push mask)
  L.nl = o;   o += (2 * N + 3) & ~3u;           // per node: ring head | len << 5 | entry bucket << 11
  L.hops = o; o += (N + 3) & ~3u;
  L.bm = o;   o += ((N + 31) / 32) * 4;         // stranded bitmap over stake rank
  L.rec = o;  o += (2 * fcap * N + 3) & ~3u;    // inbound sources u16, CSR by destination
  L.total = o;
  return L;
}

__host__ __device__ inline bool rwg_off16(uint32_t N, uint32_t fcap) { return (uint64_t)fcap * N <= 0xFFFFu; }

size_t round_wg_lds_bytes(uint32_t N, uint32_t fcap, uint32_t ASZP) {
  return rwg_layout(N, fcap, ASZP <= 16 ? 2 : 4, rwg_off16(N, fcap) ? 2 : 4).total;
}

// Streaming per-pair state (read or written once per round, ~0.5 GB/round at C2)
// goes through non-temporal loads/stores so that it does not evict the shared
// active-set rows (3.6 MB at C2) from L2.
template <class T>
__device__ inline T ntl(const T* p) { return __builtin_nontemporal_load(p); }
template <class T>
__device__ inline void nts(T* p, T v) {
#if GS_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// ctrl words
enum { C_QN = 0, C_NEXT = 1, C_ERR = 2, C_SEG = 3, C_VIS = 4, C_PUSH = 5, C_STR = 6, C_PRUNES = 7, C_SSUM = 8,
       C_NHC = 10, C_NHP = 11, C_KTH = 12, C_HCNT = 16, C_HSUM = 18, C_HMIN = 20, C_HMAX = 21, C_HMLO = 22,
       C_HMHI = 23, C_LVL = 25 /* 25..27: BFS level sizes, rotating by level mod 3 */, C_MDIRTY = 28 };

// PushActiveSet::prune for one (prunee u, pruner v) pair (push_active_set.rs:56-71,143-151):
// the bit of v's ring slot in u's entry for this slot's origin, if v is still there.
// The row comes in with one set of loads and is matched in registers (a peer occurs
// at most once in an entry, so at most one bit matches). The bit goes into the
// slot's LDS copy of the masks (mkw: u16 per node when the ring has <= 16 slots).
template <int ASZP>
__device__ inline void apply_prune_r(const RoundArgs& a, uint32_t* mkw, const uint16_t* nl_l, uint32_t u, uint32_t v) {
  const uint32_t nl = nl_l[u];
  const uint32_t head = nl & 31u, L = (nl >> 5) & 63u;
  uint32_t row[ASZP];
  load_row<ASZP>(a.peers + (size_t)(u * NB + (nl >> 11)) * ASZP, row);
  uint32_t hit = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    const uint32_t pos = (uint32_t)s >= head ? (uint32_t)s - head : (uint32_t)s + a.ASZ - head;
    hit |= (uint32_t)((uint32_t)s < a.ASZ && pos < L && row[s] == v) << s;
  }
  if (hit) {
    if (ASZP <= 16) atomicOr(&mkw[u >> 1], hit << ((u & 1u) << 4));
    else atomicOr(&mkw[u], hit);
  }
}

// Segment cursor fetch-and-increment (pu) or a dummy LDS atomic (so every slot of
// the row issues one atomic and the wait comes once). u16 cursors share a u32 word;
// their values stay below 2^16, so the add never carries into the neighbour.
template <bool OFF16>
__device__ inline uint32_t off_fetch_inc(uint32_t* offw, uint32_t w, bool pu, uint32_t* dummy) {
  if (OFF16) {
    const uint32_t sh = (w & 1u) << 4;
    return (atomicAdd(pu ? &offw[w >> 1] : dummy, pu ? 1u << sh : 0u) >> sh) & 0xFFFFu;
  }
  return atomicAdd(pu ? &offw[w] : dummy, pu ? 1u : 0u);
}

// Bit j set when record j's id (low 16 bits of rk[j]) equals k, for j < NC (records
// past the in-degree are 0xFFFFFFFF and their bits are never consulted).
typedef unsigned short rwg_u16x2 __attribute__((ext_vector_type(2)));

// Presence of record ids (u16: N < 2^16 here) in the cache entry, two records per
// register: x = pair ^ (key | key << 16) has a zero half where the key matches, and a
// packed u16 min (one v_pk_min_u16) keeps, per half, the smallest x seen -- zero iff
// that record's id is in the entry. One xor and one min per key per TWO records.
template <int NP2>
__device__ inline void match_pairs(const uint32_t (&pk)[8], uint32_t k2, uint32_t (&mn)[8]) {
#pragma unroll
  for (int h = 0; h < NP2; ++h) {
    const uint32_t x = pk[h] ^ k2;
    const rwg_u16x2 m = __builtin_elementwise_min(__builtin_bit_cast(rwg_u16x2, mn[h]), __builtin_bit_cast(rwg_u16x2, x));
    mn[h] = __builtin_bit_cast(uint32_t, m);
  }
}

// ---- C: register path (1 <= c <= 16) ----
__device__ inline void consume_lane(const RoundArgs& a, size_t p, const uint16_t* recs, const uint8_t* hops_l,
                                    uint32_t c, uint32_t& len, uint32_t& up, uint32_t& errf) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t q = (uint32_t)p;
  uint32_t rk[16];
  const uint32_t wc = active_max<5>(c);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    rk[j] = 0xFFFFFFFFu;
    if ((uint32_t)j < wc) {
      const uint32_t s = recs[min((uint32_t)j, c - 1)];
      const uint32_t key = ((uint32_t)hops_l[s] << 16) | s;  // (hop, id): hop = dist[src] + 1 shifts all alike
      rk[j] = (uint32_t)j < c ? key : 0xFFFFFFFFu;
    }
  }
  // records beyond wc are 0xFFFFFFFF already, so sorting the first 4/8/16 suffices
  if (wc <= 4) sort_net<4>(rk);
  else if (wc <= 8) sort_net<8>(rk);
  else if (wc <= 12) sort_net<16, 16, 12>(rk);
  else sort_net<16>(rk);
  // ids of ranks 2h, 2h + 1 in one register (padding ranks carry 0xFFFF, which no key
  // below equals: ids are < N <= 65,535 and an unused row reads as 0xFFFF)
  uint32_t pk[8], mn[8];
#pragma unroll
  for (int h = 0; h < 8; ++h) {
    pk[h] = (rk[2 * h] & 0xFFFFu) | (rk[2 * h + 1] << 16);
    mn[h] = 0xFFFFFFFFu;
  }
  const uint32_t id0 = rk[0] & 0xFFFFu, id1 = rk[1] & 0xFFFFu;
  // look the records up in the entry: rows streamed 8 at a time, loads issued together
  uint32_t w0 = 0, w1 = 0;
  int idx0 = -1, idx1 = -1;
  const uint32_t wl = active_max<7>(len);
  for (uint32_t i0 = 0; i0 < wl; i0 += 8) {
    uint32_t kc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) kc[t] = i0 + t < wl ? ntl(&(a.ckey + (size_t)(i0 + t) * PAIRS)[q]) : 0u;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t i = i0 + t;
      const uint32_t k = i < len ? ck_id(kc[t]) : 0xFFFFu;
      const uint32_t k2 = k | (k << 16);
      if (wc <= 4) match_pairs<2>(pk, k2, mn);
      else if (wc <= 8) match_pairs<4>(pk, k2, mn);
      else match_pairs<8>(pk, k2, mn);
      if (k == id0) { idx0 = (int)i; w0 = kc[t]; }
      if (k == id1) { idx1 = (int)i; w1 = kc[t]; }
    }
  }
  uint32_t present = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) present |= (uint32_t)(((mn[j >> 1] >> (16 * (j & 1))) & 0xFFFFu) == 0u) << j;
  idx0 = c > 0 ? idx0 : -1;
  idx1 = c > 1 ? idx1 : -1;
  up = up < 255 ? up + 1 : 255;  // rank 0 (received_cache.rs:84-86)
#pragma unroll
  for (int j = 0; j < 2; ++j) {  // timely: score += 1, inserted regardless of the 50-key cap
    if ((uint32_t)j >= c) break;
    const int idx = j == 0 ? idx0 : idx1;
    if (idx >= 0) {
      nts(&(a.ckey + (size_t)idx * PAIRS)[q], ck_bump(j == 0 ? w0 : w1));
    } else if (len < CACHE_CAP) {
      nts(&(a.ckey + (size_t)len * PAIRS)[q], ck_make(rk[j] & 0xFFFFu, 1u));
      ++len;
    } else {
      errf |= ERR_CACHE;
    }
  }
#pragma unroll
  for (int j = 2; j < 16; ++j) {  // rank order; inserted only while len < 50 (received_cache.rs:91-97)
    if ((uint32_t)j < c && !((present >> j) & 1u) && len < CACHE_LIMIT) {
      nts(&(a.ckey + (size_t)len * PAIRS)[q], ck_make(rk[j] & 0xFFFFu, 0u));
      ++len;
    }
  }
}

// ---- D: register path (len <= 32). Rows are rewritten in prune order with the
// pruned flag; returns the number of prunees. ----
template <int ASZP>
__device__ inline uint32_t prune_lane(const RoundArgs& a, uint32_t* mkw, const uint16_t* nl_l, uint32_t org, size_t p,
                                      uint32_t v, uint32_t len, uint32_t mi, uint64_t mis) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t q = (uint32_t)p;
  const uint32_t wl = active_max<5>(len);
  uint32_t sk[LANE_L];
  {
#pragma unroll
    for (int i = 0; i < LANE_L; ++i) sk[i] = (uint32_t)i < wl ? ntl(&(a.ckey + (size_t)i * PAIRS)[q]) : 0u;
    asm volatile("" ::: "memory");
    uint32_t pr[LANE_L];
#pragma unroll
    for (int i = 0; i < LANE_L; ++i) pr[i] = (uint32_t)i < wl ? a.prank[(uint32_t)i < len ? ck_id(sk[i]) : 0u] : 0u;
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < LANE_L; ++i)
      sk[i] = (uint32_t)i < len ? (((0x7Fu - ck_score(sk[i])) << 24) | pr[i]) : 0xFFFFFFFFu;
  }
  if (wl <= 8) sort_net<8>(sk);
  else sort_net<LANE_L>(sk);
  // sorted_unstable_by_key(Reverse((score, stake))), ties by id; scan of pre-add
  // cumulative stake; skip(min_ingress_nodes); skip_while(cum < min_ingress_stake).
  // Node ids and stakes of 8 sorted entries at a time are gathered with one wait.
  uint64_t cum = 0;
  uint32_t npr = 0;
  bool tail = false;
#pragma unroll
  for (int c0 = 0; c0 < LANE_L; c0 += 8) {
    if ((uint32_t)c0 >= wl) break;
    uint32_t nd[8];
    uint64_t st[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t i = c0 + t, r = i < len ? sk[c0 + t] & 0xFFFFFFu : 0u;
      const uint4 x = a.rinfo[r];  // node id and stake in one load
      nd[t] = x.x;
      st[t] = ((uint64_t)x.w << 32) | x.z;
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t i = c0 + t;
      if (i < len) {
        tail = tail || (i >= mi && cum >= mis);  // once past both skips, every later entry is pruned
        const bool pruned = tail && nd[t] != org;
        npr += pruned;
        nts(&(a.ckey + (size_t)i * PAIRS)[q], ck_make(nd[t], (0x7Fu - (sk[c0 + t] >> 24)) | (pruned ? PRUNED_FLAG : 0u)));
        if (pruned) apply_prune_r<ASZP>(a, mkw, nl_l, nd[t], v);  // prune_connections
        cum = sat_add(cum, st[t]);
      }
    }
  }
  return npr;
}

// ---- C: wave path (16 < c <= 64), all 64 lanes on one node; len/up uniform ----
__device__ inline void consume_wave(const RoundArgs& a, size_t p, const uint16_t* recs, const uint8_t* hops_l,
                                    uint32_t c, uint32_t& len, uint32_t& up, uint32_t* scr, uint32_t& errf) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t q = (uint32_t)p;
  const uint32_t l = lane_id();
  uint32_t key = 0xFFFFFFFFu;
  if (l < c) {
    const uint32_t s = recs[l];
    key = ((uint32_t)hops_l[s] << 16) | s;
  }
#pragma unroll
  for (uint32_t k = 2; k <= 64; k <<= 1)  // bitonic sort across the wave, ascending by lane
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t other = (uint32_t)__shfl_xor((int)key, (int)j);
      const bool asc = (l & k) == 0;
      const bool lower = (l & j) == 0;
      key = (lower == asc) ? min(key, other) : max(key, other);
    }
  const uint32_t src = key & 0xFFFFu;
  const uint32_t L0 = len;
  for (uint32_t i = l; i < L0; i += 64) scr[i] = (a.ckey + (size_t)i * PAIRS)[q];
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
  if (l < 2) {
    if (found >= 0) {
      (a.ckey + (size_t)found * PAIRS)[q] = ck_bump(scr[found]);
    } else {
      const uint32_t pos = L0 + (l == 1 ? n0 : 0u);
      if (pos < CACHE_CAP) {
        (a.ckey + (size_t)pos * PAIRS)[q] = ck_make(src, 1u);
      } else {
        errf |= ERR_CACHE;
      }
    }
  }
  const uint32_t L1 = min(L0 + n0 + n1, CACHE_CAP);
  const uint64_t rest = nb & ~3ull;
  if (l >= 2 && isnew) {
    const uint32_t pos = L1 + (uint32_t)__popcll(rest & ((1ull << l) - 1));
    if (pos < CACHE_LIMIT) (a.ckey + (size_t)pos * PAIRS)[q] = ck_make(src, 0u);
  }
  const uint32_t nrest = (uint32_t)__popcll(rest);
  len = L1 + (L1 < CACHE_LIMIT ? min(nrest, CACHE_LIMIT - L1) : 0u);
}

// ---- C: any in-degree (c > 64): lane 0 of the wave, records selected in order ----
__device__ inline void consume_serial(const RoundArgs& a, size_t p, const uint16_t* recs, const uint8_t* hops_l,
                                      uint32_t c, uint32_t& len, uint32_t& up, uint32_t& errf) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t l = lane_id();
  uint32_t ln = len, u = up;
  if (l == 0) {
    uint32_t prev = 0;
    u = u < 255 ? u + 1 : 255;
    for (uint32_t k = 0; k < c; ++k) {
      uint32_t best = 0xFFFFFFFFu;
      for (uint32_t j = 0; j < c; ++j) {
        const uint32_t s = recs[j];
        const uint32_t key = ((uint32_t)hops_l[s] << 16) | s;
        if ((k == 0 || key > prev) && key < best) best = key;
      }
      prev = best;
      const uint32_t src = best & 0xFFFFu;
      int found = -1;
      for (uint32_t i = 0; i < ln; ++i)
        if (ck_id(a.ckey[(size_t)i * PAIRS + p]) == src) { found = (int)i; break; }
      if (k < 2) {
        if (found >= 0) {
          uint32_t* sp = a.ckey + (size_t)found * PAIRS + p;
          *sp = ck_bump(*sp);
        } else if (ln < CACHE_CAP) {
          a.ckey[(size_t)ln * PAIRS + p] = ck_make(src, 1u);
          ++ln;
        } else {
          errf |= ERR_CACHE;
        }
      } else if (found < 0 && ln < CACHE_LIMIT) {
        a.ckey[(size_t)ln * PAIRS + p] = ck_make(src, 0u);
        ++ln;
      }
    }
  }
  len = (uint32_t)__shfl((int)ln, 0);
  up = (uint32_t)__shfl((int)u, 0);
}

// ---- D: wave path (any len <= 96), two entries per lane ----
template <int ASZP>
__device__ inline uint32_t prune_wave(const RoundArgs& a, uint32_t* mkw, const uint16_t* nl_l, uint32_t org, size_t p,
                                      uint32_t v, uint32_t len, uint32_t mi, uint64_t mis, uint32_t* scr) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t q = (uint32_t)p;
  const uint32_t l = lane_id();
  __threadfence_block();  // this wave's consume writes to the entry's rows
  uint32_t sk[2], nd[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint32_t i = l + 64 * t;
    sk[t] = 0xFFFFFFFFu;
    nd[t] = 0;
    if (i < len) {
      const uint32_t w = (a.ckey + (size_t)i * PAIRS)[q];
      nd[t] = ck_id(w);
      sk[t] = ((0x7Fu - ck_score(w)) << 24) | a.prank[nd[t]];
    }
  }
  // every lane's two entries and their stakes go round the wave by shuffles (no
  // dependent global load per entry)
  uint64_t stv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) stv[t] = l + 64 * t < len ? a.pstake[sk[t] & 0xFFFFFFu] : 0ull;
  uint32_t rank[2] = {0, 0};
  uint64_t cum[2] = {0, 0};
  for (uint32_t j = 0; j < len; ++j) {
    const bool hi = j >= 64;
    const int src = (int)(j & 63u);
    const uint32_t x = (uint32_t)__shfl((int)(hi ? sk[1] : sk[0]), src);
    const uint64_t sj = hi ? stv[1] : stv[0];
    const uint32_t slo = (uint32_t)__shfl((int)(uint32_t)sj, src), shi = (uint32_t)__shfl((int)(uint32_t)(sj >> 32), src);
    const uint64_t st = ((uint64_t)shi << 32) | slo;
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (x < sk[t]) { ++rank[t]; cum[t] = sat_add(cum[t], st); }  // saturating sums are order-free
  }
  uint32_t npr = 0;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint32_t i = l + 64 * t;
    bool pruned = false;
    if (i < len) {
      pruned = rank[t] >= mi && cum[t] >= mis && nd[t] != org;
      (a.ckey + (size_t)rank[t] * PAIRS)[q] = ck_make(nd[t], (0x7Fu - (sk[t] >> 24)) | (pruned ? PRUNED_FLAG : 0u));
      if (pruned) apply_prune_r<ASZP>(a, mkw, nl_l, nd[t], v);
    }
    npr += (uint32_t)__popcll(__ballot(pruned));
  }
  return npr;
}

// The slot's prune-stake threshold, loaded where a prune needs it (held in a register
// across the whole consume phase it was spilled to scratch).
__device__ inline double rwg_thr(const RoundArgs& a, uint32_t o) { return *(volatile const double*)&a.thr[o]; }

// Finishes a node's cache step: prune when due (lane path), else clear the
// previous round's pruned-len and record no prunes.
__device__ inline void finish_node(const RoundArgs& a, size_t p, uint32_t meta, uint32_t len, uint32_t up,
                                   uint32_t npr_if_pruned, bool pruned_now) {
  uint32_t nm;
  if (pruned_now) nm = len << 16;  // std::mem::take: entry reset, pruned keys kept readable
  else nm = len | (up << 8);
  if (nm != meta) nts(&a.cmeta[p], nm);
  const uint32_t npr = pruned_now ? npr_if_pruned : 0u;
  nts(&a.prune_round[p], (uint8_t)(npr < 255 ? npr : 255));
  if (a.record && npr) a.prune_acc[p] += npr;
}

// Wave 0 finds up to four order statistics (0-based ranks ks[]) of the set bits of
// an LDS bitmap of W words; results in out[].
__device__ inline void wave_kth_bits(const uint32_t* bm, uint32_t W, const uint32_t (&ks)[4], uint32_t* out) {
  const uint32_t l = lane_id();
  const uint32_t chunk = (W + 63) / 64;
  const uint32_t lo = min(W, l * chunk), hi = min(W, lo + chunk);
  uint32_t pc = 0;
  for (uint32_t i = lo; i < hi; ++i) pc += __popc(bm[i]);
  const uint32_t incl = wave_incl_scan(pc);
  const uint32_t before = incl - pc;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t k = ks[t];
    if (k >= before && k < incl) {
      uint32_t need = k - before;
      for (uint32_t i = lo; i < hi; ++i) {
        uint32_t w = bm[i];
        const uint32_t c = __popc(w);
        if (need < c) {
          for (uint32_t j = 0; j < need; ++j) w &= w - 1;
          out[t] = i * 32 + (__ffs(w) - 1);
          break;
        }
        need -= c;
      }
    }
  }
}

// Wave 0: HopsStat inputs from the round's hop histogram (bins 1..254 = reached
// non-origin nodes): count, sum, min, max and the two median bins.
__device__ inline void wave_hop_stats(const uint32_t* hist, uint32_t* ctrl) {
  const uint32_t l = lane_id();
  uint32_t h[4], c = 0;
  uint64_t s = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t i = 4 * l + t;
    h[t] = (i >= 1 && i < 255) ? hist[i] : 0u;
    c += h[t];
    s += (uint64_t)i * h[t];
  }
  const uint32_t incl = wave_incl_scan(c);
  const uint32_t total = (uint32_t)__shfl((int)incl, 63);
  const uint32_t before = incl - c;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)s, off);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(s >> 32), off);
    s += ((uint64_t)hi << 32) | lo;
  }
  const uint64_t nz = __ballot(c > 0);
  if (l == 0) {
    ctrl[C_HCNT] = total;
    *reinterpret_cast<unsigned long long*>(&ctrl[C_HSUM]) = s;
  }
  if (!total) return;
  if (l == (uint32_t)(__ffsll((long long)nz) - 1)) {
    for (int t = 0; t < 4; ++t)
      if (h[t]) { ctrl[C_HMIN] = 4 * l + t; break; }
  }
  if (l == 63u - (uint32_t)__clzll((long long)nz)) {
    for (int t = 3; t >= 0; --t)
      if (h[t]) { ctrl[C_HMAX] = 4 * l + t; break; }
  }
  const uint32_t ks[2] = {total % 2 ? total / 2 : total / 2 - 1, total / 2};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (ks[q] >= before && ks[q] < incl) {
      uint32_t run = before;
      for (int t = 0; t < 4; ++t) {
        if (ks[q] < run + h[t]) { ctrl[C_HMLO + q] = 4 * l + t; break; }
        run += h[t];
      }
    }
  }
}

// The peers of the pushed ring slots, compacted in slot order into dst[0, popc(pushm))
// (the rest 0). The LDS atomics that follow then cover FP lanes' words instead of
// every ring slot: at fanout 6 that halves the atomics of the BFS and the CSR scatter.
template <int ASZP, int FP>
__device__ inline void compact_push(const uint32_t (&row)[ASZP], uint32_t pushm, uint32_t (&dst)[FP]) {
#pragma unroll
  for (int t = 0; t < FP; ++t) dst[t] = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    const uint32_t j = (uint32_t)__popc(pushm & ((1u << s) - 1u));
    const bool b = (pushm >> s) & 1u;
#pragma unroll
    for (int t = 0; t < FP; ++t)
      if (b && j == (uint32_t)t) dst[t] = row[s];
  }
}

// PROF: the phase clocks (GS_PHASE_PROFILE) are compiled in -- only for the C2 shape's
// instantiation; their long-lived 64-bit clock state spilled to scratch in every build.
// Workgroup 0 of a round kernel with rotation ahead: the previous ahead rotation's nodes'
// entries copied from the current row buffer into the other one (which then equals the
// current rows), then this round's rotation (decide, gossip.rs:739-754; rotate_entry,
// push_active_set.rs:73-114,153-187) on the other buffer. The slots' workgroups only read
// the current buffer, so the two never touch the same rows.
// lids: the workgroup's dynamic LDS, N node ids and the count after them (the create-time
// gate checks 4 (N + 1) bytes fit: no static LDS beside the round's layout)
template <int ASZP>
__device__ void rotate_ahead_wg(const RoundArgs& a, uint32_t* lids) {
  const uint32_t tid = threadIdx.x, T = blockDim.x, N = a.N;
  uint32_t& lcount = lids[N];
  if (a.plist) {
    const uint32_t total = *a.pcount * NB;
    for (uint32_t gid = tid; gid < total; gid += T) {
      const uint32_t ent = a.plist[gid / NB] * NB + gid % NB;
#pragma unroll
      for (int w = 0; w < ASZP; ++w) a.rpeers[(size_t)ent * ASZP + w] = a.peers[(size_t)ent * ASZP + w];
      a.rhl[ent] = a.hl[ent];
    }
  }
  if (tid == 0) lcount = 0;
  __syncthreads();
  for (uint32_t u = tid; u < N; u += T) {
    Philox s(a.seed, P_DECIDE, u, a.rround);
    if (unit_f64(s.next()) < a.rp) lids[atomicAdd(&lcount, 1u)] = u;
  }
  __syncthreads();  // (also: the copied rows are visible to the workgroup's rotate_entry loads)
  const uint32_t n = lcount;
  for (uint32_t i = tid; i < n; i += T) a.rlist[i] = lids[i];
  if (tid == 0) *a.rcount = n;
  for (uint32_t gid = tid; gid < n * NB; gid += T)
    rotate_entry<ASZP>(a.bucket, a.P, a.IX, a.rpeers, a.rhl, lids, a.rchanged, N, a.ASZ, a.seed, a.rround, gid);
}

template <int ASZP, bool OFF16, int FP, bool PROF>
__global__ __launch_bounds__(RWG_THREADS, RWG_MIN_WAVES) void k_round_wg(RoundArgs a) {
  using PMT = typename std::conditional<(ASZP <= 16), uint16_t, uint32_t>::type;
  using OFFT = typename std::conditional<OFF16, uint16_t, uint32_t>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t N = a.N;
  const RwgLayout L = rwg_layout(N, a.fcap, (uint32_t)sizeof(PMT), (uint32_t)sizeof(OFFT));
  uint32_t* ctrl = reinterpret_cast<uint32_t*>(smem + L.ctrl);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem + L.hist);
  uint32_t* cntw = reinterpret_cast<uint32_t*>(smem + L.cnt);
  const uint16_t* cnt_l = reinterpret_cast<const uint16_t*>(smem + L.cnt);
  uint16_t* q0 = reinterpret_cast<uint16_t*>(smem + L.qo);
  OFFT* off_l = reinterpret_cast<OFFT*>(smem + L.qo);
  uint32_t* offw = reinterpret_cast<uint32_t*>(smem + L.qo);
  PMT* pm_l = reinterpret_cast<PMT*>(smem + L.pm);
  uint16_t* hv_l = reinterpret_cast<uint16_t*>(smem + L.pm);  // heavy nodes: consume from the front,
                                                              // prune-only from the back
  uint16_t* nl_l = reinterpret_cast<uint16_t*>(smem + L.nl);
  PMT* mk_l = reinterpret_cast<PMT*>(smem + L.mk);
  uint32_t* mkw = reinterpret_cast<uint32_t*>(smem + L.mk);
  uint8_t* hops_l = smem + L.hops;
  uint32_t* bm_l = reinterpret_cast<uint32_t*>(smem + L.bm);
  uint16_t* rec_l = reinterpret_cast<uint16_t*>(smem + L.rec);
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t* scr = reinterpret_cast<uint32_t*>(smem + L.scr) + wid * RWG_SCR;
  const uint32_t W = (N + 31) / 32;

  if (a.rot_on && blockIdx.x == 0) {  // (dispatched first: the rotation overlaps the whole round)
    rotate_ahead_wg<ASZP>(a, reinterpret_cast<uint32_t*>(smem));
    return;
  }
  const uint32_t o = blockIdx.x - a.rot_on;
  const uint32_t org = a.origin[o], ob = a.obkt[o], nf = a.nfail[o];
  const size_t base = (size_t)o * N;
  uint32_t errf = 0;
  unsigned long long t_mark = PROF && a.phase_clk && tid == 0 ? wall_clock64() : 0;

  for (uint32_t i = tid; i < (N + 1) / 2; i += RWG_THREADS) cntw[i] = 0;
  // Each node's mask word, bucket and ring head/len (of the entry the origin uses,
  // push_active_set.rs:38-52), RWG_IN nodes per trip: the trip's bucket loads, then its
  // hl loads, are issued together (one node per trip waited for two dependent round trips
  // per node)
  for (uint32_t v0 = tid; v0 < N; v0 += RWG_IN * RWG_THREADS) {
    uint32_t bk[RWG_IN], mw[RWG_IN], hv[RWG_IN];
#pragma unroll
    for (uint32_t k = 0; k < RWG_IN; ++k) {
      const uint32_t v = v0 + k * RWG_THREADS;
      bk[k] = v < N ? min((uint32_t)a.bucket[v], ob) : 0u;
      mw[k] = v < N ? ntl(&a.mask[base + v]) : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < RWG_IN; ++k) {
      const uint32_t v = v0 + k * RWG_THREADS;
      hv[k] = v < N ? a.hl[v * NB + bk[k]] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < RWG_IN; ++k) {
      const uint32_t v = v0 + k * RWG_THREADS;
      if (v >= N) break;
      hops_l[v] = 0xFF;
      pm_l[v] = 0;
      mk_l[v] = (PMT)mw[k];
      nl_l[v] = (uint16_t)((hv[k] & 0x1Fu) | ((hv[k] >> 8) << 5) | (bk[k] << 11));
    }
  }
  for (uint32_t i = tid; i < 256; i += RWG_THREADS) hist[i] = 0;
  for (uint32_t i = tid; i < W; i += RWG_THREADS) bm_l[i] = 0;
  if (tid < 32) ctrl[tid] = 0;
  __syncthreads();
  if (a.rot_count) {  // Cluster::chance_to_rotate's fresh filters (gossip.rs:739-754): the replaced
                      // ring slots of the last rotation lose this slot's prune bits
    const uint32_t nr = *a.rot_count;
    for (uint32_t i = tid; i < nr; i += RWG_THREADS) {
      const uint32_t u = a.rot_list[i];
      const uint32_t m = a.rot_changed[u * NB + min((uint32_t)a.bucket[u], ob)];
      if (m && (mk_l[u] & m)) {
        mk_l[u] = (PMT)(mk_l[u] & ~m);
        ctrl[C_MDIRTY] = 1;
      }
    }
  }
  if (tid == 0) { ctrl[C_LVL] = 1; hops_l[org] = 0; q0[0] = (uint16_t)org; }
  __syncthreads();  // the rotation clear above changes mk_l
  // Every node's pushes for this origin depend only on its row, the slot's prune
  // mask and the failed set, not on the traversal. They are taken here for all
  // nodes at once (two rows in flight per thread) and kept as u16 lists in the
  // record area (stride fcap; the CSR overwrites it after the BFS), so the BFS levels
  // issue no global loads.
  uint16_t* lst_l = reinterpret_cast<uint16_t*>(smem + L.rec);
  const uint32_t fc = a.fcap;
  for (uint32_t v0 = tid; v0 < N; v0 += 2 * RWG_THREADS) {
    const uint32_t v1 = v0 + RWG_THREADS;
    const bool h1 = v1 < N;
    uint32_t r0[ASZP], r1[ASZP];
    const uint32_t nl0 = nl_l[v0], nl1 = h1 ? nl_l[v1] : 0u;
    load_row<ASZP>(a.peers + (size_t)(v0 * NB + (nl0 >> 11)) * ASZP, r0);
    if (h1) load_row<ASZP>(a.peers + (size_t)(v1 * NB + (nl1 >> 11)) * ASZP, r1);
    uint32_t pm0 = taken_slots<ASZP>(r0, nl0 & 31u, (nl0 >> 5) & 63u, a.ASZ, mk_l[v0], org, a.fanout);
    uint32_t pm1 = 0;
    if (h1) pm1 = taken_slots<ASZP>(r1, nl1 & 31u, (nl1 >> 5) & 63u, a.ASZ, mk_l[v1], org, a.fanout);
    if (nf) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        if (((pm0 >> s) & 1u) && a.frank[r0[s]] < nf) pm0 &= ~(1u << s);
        if (((pm1 >> s) & 1u) && a.frank[r1[s]] < nf) pm1 &= ~(1u << s);
      }
    }
    pm_l[v0] = (PMT)pm0;
    if (h1) pm_l[v1] = (PMT)pm1;
    // pushed slots in FIFO-free slot order, each a predicated u16 store at a running index
    uint32_t j0 = v0 * fc, j1 = v1 * fc;
#pragma unroll
    for (int s = 0; s < ASZP; ++s) {
      if ((pm0 >> s) & 1u) lst_l[j0++] = (uint16_t)r0[s];
      if ((pm1 >> s) & 1u) lst_l[j1++] = (uint16_t)r1[s];
    }
  }
  __syncthreads();
  RWG_MARK(0);

  // ---------------- A: BFS -------------------------------------------------
  unsigned long long prof[5] = {0, 0, 0, 0, 0};  // profiling builds of the run only (thread 0)
  uint16_t* cur = q0;  // this level: cur[0, qn); the next is appended behind it
  // One barrier per level: level d reads its size from ctrl[C_LVL + d % 3], counts
  // the next level into ctrl[C_LVL + (d + 1) % 3], and clears ctrl[C_LVL + (d + 2) % 3]
  // (read at level d - 1, before the last barrier; next counted at level d + 1, after
  // the coming one).
  for (uint32_t d = 0, l3 = 0;; ++d, l3 = l3 == 2 ? 0 : l3 + 1) {
    const uint32_t qn = ctrl[C_LVL + l3];
    if (qn == 0) break;
    if (d + 1 >= 255) { errf |= ERR_DEPTH; break; }
    const uint32_t l3n = l3 == 2 ? 0 : l3 + 1, l3c = l3n == 2 ? 0 : l3n + 1;
    if (tid == 0) ctrl[C_LVL + l3c] = 0;
    uint16_t* nxt = cur + qn;
    unsigned long long tl0 = (PROF && a.phase_clk && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
    for (uint32_t i0 = 0; i0 < qn; i0 += RWG_THREADS) {
      if (i0 + (wid << 6) >= qn) continue;  // wave-uniform: no frontier node for this wave
      const bool valid = i0 + tid < qn;
      uint32_t pushm = 0;
      uint32_t dst[FP];
#pragma unroll
      for (int j = 0; j < FP; ++j) dst[j] = 0;
      if (valid) {
        const uint32_t u = cur[i0 + tid];
        pushm = pm_l[u];
        const uint32_t kk = __popc(pushm);
#pragma unroll
        for (int j = 0; j < FP; ++j)
          if ((uint32_t)j < kk) dst[j] = lst_l[u * fc + j];
        if (PROF && a.phase_clk && tid == 0 && i0 == 0) {
          const unsigned long long t1 = __builtin_amdgcn_s_memtime();
          prof[0] += t1 - tl0;  // level start -> push list read (shader cycles)
          tl0 = t1;
        }
      }
      // The pushed peers (at most FP per lane) issue their LDS atomic back to back,
      // lanes with fewer add 0 to a per-lane dummy word, then one wait: a conditional
      // atomic per push would be followed by its own lgkmcnt(0) wait.
      const uint32_t k = __popc(pushm);
      uint32_t old[FP];
      uint32_t* dummy = scr + lane;
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        const bool pu = (uint32_t)j < k;
        const uint32_t w = dst[j], sh = (w & 1u) << 4;
        old[j] = (atomicAdd(pu ? &cntw[w >> 1] : dummy, pu ? 1u << sh : 0u) >> sh) & 0xFFFFu;
      }
      uint32_t newm = 0;
#pragma unroll
      for (int j = 0; j < FP; ++j)
        if ((uint32_t)j < k && old[j] == 0) {
          newm |= 1u << j;
          hops_l[dst[j]] = (uint8_t)(d + 1);
        }
      // next-level slots: one LDS atomic per wave; the lanes' offsets come from one
      // ballot per push column (mbcnt of the lower lanes), no LDS round trips
      uint32_t nex = 0, ntot = 0;
#pragma unroll
      for (int j = 0; j < FP; ++j) {
        const uint64_t bj = __ballot((newm >> j) & 1u);
        nex += __builtin_amdgcn_mbcnt_hi((uint32_t)(bj >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bj, 0u));
        ntot += (uint32_t)__popcll(bj);
      }
      uint32_t nb = 0;
      if (lane == 0 && ntot) nb = atomicAdd(&ctrl[C_LVL + l3n], ntot);
      uint32_t idx = __builtin_amdgcn_readfirstlane(nb) + nex;
#pragma unroll
      for (int j = 0; j < FP; ++j)
        if ((newm >> j) & 1u) nxt[idx++] = (uint16_t)dst[j];
      if (PROF && a.phase_clk && tid == 0 && i0 == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        prof[1] += t1 - tl0;  // row loaded -> pushes done
        tl0 = t1;
      }
    }
    if (PROF && a.phase_clk && tid == 0) {
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      prof[2] += t1 - tl0;  // remaining iterations of the level
      tl0 = t1;
    }
    __syncthreads();
    cur += qn;
    if (PROF && a.phase_clk && tid == 0) {
      prof[4] += 1;  // levels
      prof[3] += __builtin_amdgcn_s_memtime() - tl0;  // the barrier
    }
  }

  if (PROF && a.phase_clk && tid == 0) {
    atomicAdd(&a.phase_clk[8], prof[0]);
    atomicAdd(&a.phase_clk[9], prof[1]);
    atomicAdd(&a.phase_clk[10], prof[2]);
    atomicAdd(&a.phase_clk[11], prof[3]);
    atomicAdd(&a.phase_clk[7], prof[4]);
  }
  RWG_MARK(1);
  // ---------------- B: inbound CSR, per-pair outputs, round statistics ------
  for (uint32_t v0 = 0; v0 < N; v0 += RWG_THREADS) {  // segment per destination (order free)
    const uint32_t v = v0 + tid;
    const uint32_t c = v < N ? cnt_l[v] : 0;
    const uint32_t incl = wave_incl_scan(c);
    const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
    uint32_t b = 0;
    if (lane == 0 && tot) b = atomicAdd(&ctrl[C_SEG], tot);
    b = (uint32_t)__shfl((int)b, 0);
    if (v < N) off_l[v] = b + incl - c;
  }
  __syncthreads();
  // Every visited node scatters its id into its peers' segments. Only loads and LDS
  // work here: the per-pair global stores and accumulator atomics are issued at the
  // end of the kernel (F), since VMEM operations complete in order and a load issued
  // behind them waits for them. Two nodes per thread per step, both rows in flight.
  uint8_t* eg_l = smem + L.eg;
  if (FP <= 8 && N <= RWG_CSR_REG_NODES) {
    // The push lists (in the record area) are read into registers, two u16 ids per
    // word, then after a barrier the records overwrite them: no row is read again.
    constexpr int FW = (FP + 1) / 2;
    uint32_t pk[CSR_NPT][FW], kk[CSR_NPT];
#pragma unroll
    for (uint32_t i = 0; i < CSR_NPT; ++i) {
      const uint32_t v = tid + i * RWG_THREADS;
      const uint32_t pm = v < N && hops_l[v] != 0xFF ? pm_l[v] : 0u;
      kk[i] = __popc(pm);
      if (v < N) eg_l[v] = (uint8_t)kk[i];
#pragma unroll
      for (int w = 0; w < FW; ++w) {
        const uint32_t lo = (uint32_t)(2 * w) < kk[i] ? lst_l[v * fc + 2 * w] : 0u;
        const uint32_t hi = (uint32_t)(2 * w + 1) < kk[i] ? lst_l[v * fc + 2 * w + 1] : 0u;
        pk[i][w] = lo | hi << 16;
      }
    }
    __syncthreads();
    uint32_t* dummy = scr + lane;
#pragma unroll
    for (uint32_t i = 0; i < CSR_NPT; ++i) {
      if (!kk[i]) continue;
      const uint32_t v = tid + i * RWG_THREADS;
      uint32_t pos[FP];
#pragma unroll
      for (int j = 0; j < FP; ++j)
        pos[j] = off_fetch_inc<OFF16>(offw, (pk[i][j >> 1] >> ((j & 1) * 16)) & 0xFFFFu, (uint32_t)j < kk[i], dummy);
#pragma unroll
      for (int j = 0; j < FP; ++j)
        if ((uint32_t)j < kk[i]) rec_l[pos[j]] = (uint16_t)v;
    }
  } else {
    uint32_t* dummy = scr + lane;
    for (uint32_t v0 = tid; v0 < N; v0 += 2 * RWG_THREADS) {
      const uint32_t v1 = v0 + RWG_THREADS;
      const uint32_t pm0 = hops_l[v0] != 0xFF ? pm_l[v0] : 0u;
      const uint32_t pm1 = v1 < N && hops_l[v1] != 0xFF ? pm_l[v1] : 0u;
      uint32_t r0[ASZP], r1[ASZP];
#pragma unroll
      for (int s = 0; s < ASZP; ++s) r0[s] = r1[s] = 0;
      if (pm0) load_row<ASZP>(a.peers + (size_t)(v0 * NB + (nl_l[v0] >> 11)) * ASZP, r0);
      if (pm1) load_row<ASZP>(a.peers + (size_t)(v1 * NB + (nl_l[v1] >> 11)) * ASZP, r1);
      eg_l[v0] = (uint8_t)__popc(pm0);
      if (v1 < N) eg_l[v1] = (uint8_t)__popc(pm1);
      if (pm0 | pm1) {
        uint32_t d0[FP], d1[FP], p0[FP], p1[FP];
        compact_push<ASZP, FP>(r0, pm0, d0);
        compact_push<ASZP, FP>(r1, pm1, d1);
        const uint32_t k0 = __popc(pm0), k1 = __popc(pm1);
#pragma unroll
        for (int j = 0; j < FP; ++j) p0[j] = off_fetch_inc<OFF16>(offw, d0[j], (uint32_t)j < k0, dummy);
#pragma unroll
        for (int j = 0; j < FP; ++j) p1[j] = off_fetch_inc<OFF16>(offw, d1[j], (uint32_t)j < k1, dummy);
#pragma unroll
        for (int j = 0; j < FP; ++j)
          if ((uint32_t)j < k0) rec_l[p0[j]] = (uint16_t)v0;
#pragma unroll
        for (int j = 0; j < FP; ++j)
          if ((uint32_t)j < k1) rec_l[p1[j]] = (uint16_t)v1;
      }
    }
  }
  __syncthreads();
  RWG_MARK(2);

  // ---------------- C + D: consume, prune (register path) -------------------
  const uint32_t mi = a.min_ingress[o];
  const uint64_t so = a.stake[org];
  uint32_t npr_sum = 0;
  uint32_t meta_next = tid < N ? ntl(&a.cmeta[base + tid]) : 0u;
  for (uint32_t v = tid; v < N; v += RWG_THREADS) {
    const size_t p = base + v;
    const uint32_t meta = meta_next;  // the next node's meta is in flight while this one is consumed
    if (v + RWG_THREADS < N) meta_next = ntl(&a.cmeta[p + RWG_THREADS]);
    const uint32_t c = cnt_l[v];
    if (c > LANE_C) {
      hv_l[atomicAdd(&ctrl[C_NHC], 1u)] = (uint16_t)v;
      continue;
    }
    uint32_t len = meta & 0xFF, up = (meta >> 8) & 0xFF;
    if (c) consume_lane(a, p, rec_l + (off_l[v] - c), hops_l, c, len, up, errf);
    if (up >= MIN_NUM_UPSERTS) {
      if (len > (uint32_t)LANE_L) {
        nts(&a.cmeta[p], len | (up << 8));
        hv_l[N - 1 - atomicAdd(&ctrl[C_NHP], 1u)] = (uint16_t)v;
        continue;
      }
      const uint64_t sv = a.stake[v];
      const uint32_t npr = prune_lane<ASZP>(a, mkw, nl_l, org, p, v, len, mi, min_ingress_stake(sv < so ? sv : so, rwg_thr(a, o)));
      npr_sum += npr;
      finish_node(a, p, meta, len, 0, npr, true);
    } else {
      finish_node(a, p, meta, len, up, 0, false);
    }
  }
  __syncthreads();
  RWG_MARK(3);

  // ---------------- C + D: heavy nodes, one wave each -----------------------
  {
    const uint32_t nhc = ctrl[C_NHC], nhp = ctrl[C_NHP];
    for (uint32_t i = wid; i < nhc + nhp; i += RWG_WAVES) {
      const bool is_c = i < nhc;
      const uint32_t v = is_c ? hv_l[i] : hv_l[N - 1 - (i - nhc)];
      const size_t p = base + v;
      const uint32_t meta = a.cmeta[p];
      uint32_t len = meta & 0xFF, up = (meta >> 8) & 0xFF;
      if (is_c) {
        const uint32_t c = cnt_l[v];
        const uint16_t* recs = rec_l + (off_l[v] - c);
        if (c <= a.wave_c_max) consume_wave(a, p, recs, hops_l, c, len, up, scr, errf);
        else consume_serial(a, p, recs, hops_l, c, len, up, errf);
      }
      const bool due = up >= MIN_NUM_UPSERTS;
      uint32_t npr = 0;
      if (due) {
        const uint64_t sv = a.stake[v];
        npr = prune_wave<ASZP>(a, mkw, nl_l, org, p, v, len, mi, min_ingress_stake(sv < so ? sv : so, rwg_thr(a, o)), scr);
        if (lane == 0) npr_sum += npr;
      }
      if (lane == 0) finish_node(a, p, meta, len, due ? 0u : up, npr, due);
    }
  }
  if (npr_sum) atomicAdd(&ctrl[C_PRUNES], npr_sum);
  if (errf) atomicOr(&ctrl[C_ERR], errf);
  RWG_MARK(4);

  // ---------------- F: per-pair outputs and measured-round statistics --------
  // (gossip_main.rs:480-514) Stranded nodes' stake/rank loads go first, then only
  // stores and fire-and-forget atomics.
  if (a.record) {
    uint32_t sc = 0;
    uint64_t ss = 0;
    for (uint32_t v = tid; v < N; v += RWG_THREADS) {
      if (hops_l[v] != 0xFF || (nf && a.frank[v] < nf)) continue;
      ++sc;
      ss += a.stake[v];
      const uint32_t r = a.srank[v];
      atomicOr(&bm_l[r >> 5], 1u << (r & 31));
    }
    if (sc) atomicAdd(&ctrl[C_STR], sc);
    if (ss) atomicAdd(reinterpret_cast<unsigned long long*>(&ctrl[C_SSUM]), (unsigned long long)ss);
  }
  {
    uint32_t vis = 0, pushes = 0;
    for (uint32_t v = tid; v < N; v += RWG_THREADS) {
      const size_t p = base + v;
      const uint32_t h = hops_l[v], c = cnt_l[v], eg = eg_l[v];
      nts(&a.hops[p], (uint8_t)h);
      nts(&a.cnt[p], c);
      nts(&a.egress[p], (uint8_t)eg);
      if (a.record) {
        pushes += c;
        if (c) atomicAdd(&a.ingress_acc[p], c);
        if (eg) atomicAdd(&a.egress_acc[p], eg);
        if (h != 0xFF) {
          ++vis;
          atomicAdd(&hist[h], 1u);
        } else if (!(nf && a.frank[v] < nf)) {
          atomicAdd(&a.strand[p], 1u);
        }
      }
    }
    if (a.record) {
      if (vis) atomicAdd(&ctrl[C_VIS], vis);
      if (pushes) atomicAdd(&ctrl[C_PUSH], pushes);
    }
  }
  __syncthreads();
  RWG_MARK(5);

  // ---------------- E: slot summary -----------------------------------------
  if (tid == 0) {
    a.slot_prunes[o] = ctrl[C_PRUNES];
    if (ctrl[C_ERR]) atomicOr(a.err, ctrl[C_ERR]);
  }
  if (ctrl[C_PRUNES] || ctrl[C_MDIRTY])  // prunes / a rotation's clear changed the LDS masks: write back
    for (uint32_t v = tid; v < N; v += RWG_THREADS) nts(&a.mask[base + v], (uint32_t)mk_l[v]);
  if (!a.record) return;
  for (uint32_t i = tid; i < 256; i += RWG_THREADS)
    if (hist[i]) a.hist_acc[(size_t)o * 256 + i] += hist[i];
  const uint32_t sc = ctrl[C_STR];
  if (wid == 0) wave_hop_stats(hist, ctrl);
  if (wid == 1 && sc) {
    const uint32_t ks[4] = {0u, sc - 1, sc % 2 ? sc / 2 : sc / 2 - 1, sc / 2};
    wave_kth_bits(bm_l, W, ks, &ctrl[C_KTH]);
  }
  __syncthreads();
  if (tid == 0) {
    gs_round_summary s = {};
    s.visited = ctrl[C_VIS];
    s.pushes = ctrl[C_PUSH];
    s.stranded = sc;
    s.prunes = ctrl[C_PRUNES];
    s.stranded_stake_sum = *reinterpret_cast<unsigned long long*>(&ctrl[C_SSUM]);
    s.hop_count = ctrl[C_HCNT];  // HopsStat over reached non-origin nodes (gossip_stats.rs:47-98)
    s.hop_sum = *reinterpret_cast<unsigned long long*>(&ctrl[C_HSUM]);
    if (s.hop_count) {
      s.hop_min = ctrl[C_HMIN];
      s.hop_max = ctrl[C_HMAX];
      s.hop_med_lo = ctrl[C_HMLO];
      s.hop_med_hi = ctrl[C_HMHI];
    }
    if (sc) {  // StrandedNodeStats order statistics by stake (gossip_stats.rs:767-819)
      s.stranded_stake_min = a.stake[a.by_srank[ctrl[C_KTH + 0]]];
      s.stranded_stake_max = a.stake[a.by_srank[ctrl[C_KTH + 1]]];
      s.stranded_med_lo = a.stake[a.by_srank[ctrl[C_KTH + 2]]];
      s.stranded_med_hi = a.stake[a.by_srank[ctrl[C_KTH + 3]]];
    }
    a.sum[o] = s;
  }
  RWG_MARK(6);
}

template <int ASZP, bool OFF16, int FP, bool PROF>
static hipError_t launch_rwg_p(Engine& e, const RoundArgs& a, size_t lds) {
  if (e.rwg_attr_lds != lds || e.rwg_attr_prof != PROF) {
    hipError_t r = hipFuncSetAttribute((const void*)k_round_wg<ASZP, OFF16, FP, PROF>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (r != hipSuccess) return r;
    e.rwg_attr_lds = lds;
    e.rwg_attr_prof = PROF;
  }
  hipLaunchKernelGGL((k_round_wg<ASZP, OFF16, FP, PROF>), dim3(e.S + a.rot_on), dim3(RWG_THREADS), lds, e.st, a);
  return hipSuccess;
}

template <int ASZP, bool OFF16, int FP>
static hipError_t launch_rwg_fp(Engine& e, const RoundArgs& a, size_t lds) {
  if constexpr (ASZP == 12 && OFF16 && FP == 6) {  // C2's shape: phase clocks available
    if (a.phase_clk) return launch_rwg_p<ASZP, OFF16, FP, true>(e, a, lds);
  }
  return launch_rwg_p<ASZP, OFF16, FP, false>(e, a, lds);
}

template <int ASZP, bool OFF16>
static hipError_t launch_rwg(Engine& e, const RoundArgs& a, size_t lds) {
  // FP: compacted pushes per lane (fanout <= 6, the reference's default, or the ring)
  constexpr int FP6 = ASZP < 6 ? ASZP : 6;
  if (a.fcap <= (uint32_t)FP6) return launch_rwg_fp<ASZP, OFF16, FP6>(e, a, lds);
  return launch_rwg_fp<ASZP, OFF16, ASZP>(e, a, lds);
}

hipError_t launch_round_wg(Engine& e, bool record, uint32_t rec_slot, bool rot_clear, const RotAhead* ra) {
  RoundArgs a;
  a.rot_on = ra ? 1u : 0u;
  a.P = e.P; a.IX = e.IX; a.seed = e.prm.seed; a.rp = e.prm.rotation_probability;
  a.rpeers = ra ? ra->peers2 : nullptr; a.rhl = ra ? ra->hl2 : nullptr;
  a.rlist = ra ? ra->list : nullptr; a.rcount = ra ? ra->count : nullptr; a.rchanged = ra ? ra->changed : nullptr;
  a.plist = ra ? ra->plist : nullptr; a.pcount = ra ? ra->pcount : nullptr;
  a.rround = ra ? ra->round : 0u;
  a.stake = e.stake; a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.frank = e.frank; a.srank = e.srank;
  a.by_srank = e.by_srank; a.prank = e.prank; a.by_prank = e.by_prank; a.pstake = e.pstake; a.rinfo = e.rinfo; a.origin = e.origin;
  a.obkt = e.obkt; a.nfail = e.nfail; a.min_ingress = e.min_ingress; a.thr = e.thr; a.slot_prunes = e.slot_prunes;
  a.hops = e.hops; a.cnt = e.cnt; a.mask = e.mask; a.cmeta = e.cmeta; a.ckey = e.ckey;
  a.egress = e.egress; a.prune_round = e.prune_round; a.egress_acc = e.egress_acc; a.ingress_acc = e.ingress_acc;
  a.prune_acc = e.prune_acc; a.strand = e.strand; a.hist_acc = e.hist_acc;
  a.sum = record ? e.sum + (size_t)rec_slot * e.S : nullptr;
  a.rot_list = e.rot_list;
  a.rot_count = rot_clear ? e.rot_count + e.rot_parity : nullptr;
  a.rot_changed = e.rot_changed;
  a.err = e.err; a.phase_clk = e.phase_clk;
  a.wave_c_max = (e.prm.flags & GS_FLAG_NARROW_WAVE_PATH) ? 24u : 64u; a.N = e.N; a.S = e.S; a.ASZ = e.ASZ; a.fanout = e.fanout; a.fcap = e.fcap; a.PAIRS = e.PAIRS;
  a.record = record ? 1 : 0;
  const size_t lds = round_wg_lds_bytes(e.N, e.fcap, e.ASZP);
  hipError_t r;
  const bool off16 = rwg_off16(e.N, e.fcap);
  GS_ASZP_DISPATCH(e.ASZP, r = (off16 ? launch_rwg<A, true>(e, a, lds) : launch_rwg<A, false>(e, a, lds)));
  if (r != hipSuccess) return r;
  return hipGetLastError();
}

}  // namespace gs
