// gs_consume_g.hip -- consume + prune for the level-synchronous rounds (large N).
//
// gs_round's step-kernel path (BFS modes LEVEL / BINNED) leaves each pair's inbound
// records in HBM as rows inb[j][pair] = hop << 24 | src (j < in-degree). Per pair:
//   consume_messages + ReceivedCache::record (gossip.rs:618-653, received_cache.rs:27-36,
//   83-98): the records sorted by (hop, id) -- their u32 order -- in registers by a
//   sorting network, looked up in the cache entry whose rows are streamed 8 at a time,
//   coalesced across lanes;
//   send_prunes + ReceivedCache::prune + prune_connections (gossip.rs:657-737,
//   received_cache.rs:38-63,100-131) for the entries that reached 20 upserts, found
//   by a scan of the meta words: the (score, stake) order as one 31-bit key per entry sorted in registers,
//   pre-add cumulative stake, prune bits set in the prunees' masks.
// In-degree > 16 (consume) or entries > 32 keys (prune) are taken by the whole wave,
// one pair at a time, after the wave's lanes finish their own pairs; in-degree > 64 by
// an ordered single-lane selection. Results are identical to the generic per-pair code
// in gs_kernels.hip (cp_generic), which remains the step-wise gs_consume_messages /
// gs_send_prunes / gs_prune_connections.
#include <algorithm>

#include "gs_consume_dev.h"
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

namespace {

constexpr uint32_t CG_THREADS = 256;
constexpr uint32_t CG_WAVES = CG_THREADS / 64;
constexpr uint32_t CG_SCR = 128;  // per-wave LDS scratch (u32)
constexpr uint32_t LANE_L = 16;  // register prune path capacity

struct CgArgs {
  const uint64_t* stake;
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
  const uint32_t* own;  // own-bucket rows (BINNED / MULTI; else null), ORW words each
  const uint32_t* origin;
  const uint8_t* obkt;
  const uint32_t* min_ingress;
  const double* thr;
  const uint32_t* prank;
  const uint32_t* by_prank;
  const uint64_t* pstake;
  const uint4* pinfo;  // by id: {prune rank, 0, stake lo, stake hi}
  const uint32_t* cnt;
  const uint32_t* inb;
  uint32_t* cmeta;
  uint32_t* ckey;
  uint8_t* prune_round;
  uint32_t* slot_prunes;
  uint32_t* mask;  // prune bits land here
  uint32_t* ingress_acc;
  uint32_t* prune_acc;
  uint32_t* err;
  uint32_t N, S, ASZ, capin, ORW;
  uint32_t NP, vlo;  // pair q = slot * NP + (node - vlo)
  size_t mso, msu;  // prune-mask strides of (slot, node)
  uint32_t lane_c, lane_l, wave_c;  // register-path bounds (16, 16) and wave-consume bound (64);
                                    // GS_FLAG_NARROW_WAVE_PATH: (4, 4, 8), so small tests reach every path
  size_t PAIRS;
  int record;
  int zero_sp;  // k_cg_consume zeroes slot_prunes (block 0) for the k_cg_prune that follows
};

// ---- consume, register path (1 <= c <= 16) ----
__device__ inline void consume_lane(const CgArgs& a, uint32_t q, uint32_t c, uint32_t& len, uint32_t& up,
                                    uint32_t& errf) {
  const size_t PAIRS = a.PAIRS;
  uint32_t rk[16];
  const uint32_t wc = active_max<5>(c);
#pragma unroll
  for (int j = 0; j < 16; ++j)  // only the lane's own rows: rows past its in-degree are not read (a wave-wide
                                // bound read ~3x the inbound bytes at C4's mean in-degree of 4)
    rk[j] = (uint32_t)j < c ? ntl(&(a.inb + (size_t)j * PAIRS)[q]) : 0xFFFFFFFFu;
  asm volatile("" ::: "memory");
  uint32_t kc0[8];
  cache_prefetch(a.ckey, PAIRS, q, len, kc0);
  sort_ranked(rk, wc);
  cache_update_lane(a.ckey, PAIRS, q, rk, c, wc, kc0, len, up, errf);
}

// ---- consume, wave path (16 < c <= 64): all lanes on pair q; len/up wave-uniform ----
__device__ inline void consume_wave(const CgArgs& a, uint32_t q, uint32_t c, uint32_t& len, uint32_t& up,
                                    uint32_t* scr, uint32_t& errf) {
  const uint32_t l = lane_id();
  const uint32_t key = wave_sort(l < c ? (a.inb + (size_t)l * a.PAIRS)[q] : 0xFFFFFFFFu);
  cache_update_wave(a.ckey, a.PAIRS, q, key, c, len, up, scr, errf);
}

// ---- consume, any in-degree (c > 64): lane 0, records selected in order ----
__device__ inline void consume_serial(const CgArgs& a, uint32_t q, uint32_t c, uint32_t& len, uint32_t& up,
                                      uint32_t& errf) {
  const size_t PAIRS = a.PAIRS;
  cache_update_serial(a.ckey, PAIRS, q, c, len, up, errf, [&](uint32_t k, uint32_t prev) {
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t j = 0; j < c; ++j) {
      const uint32_t r = a.inb[(size_t)j * PAIRS + q];
      if ((k == 0 || r > prev) && r < best) best = r;
    }
    return best;
  });
}

// After a pair's consume: record its in-degree, queue a due prune, else clear the
// previous round's pruned-len and prune count.
__device__ inline void after_consume(const CgArgs& a, uint32_t q, uint32_t meta, uint32_t c, uint32_t len,
                                     uint32_t up, bool& due) {
  due = up >= MIN_NUM_UPSERTS;
  const uint32_t nm = due ? (len | (up << 8) | (meta & 0xFF0000u)) : (len | (up << 8));
  if (nm != meta) a.cmeta[q] = nm;
  if (!due) a.prune_round[q] = 0;
  if (a.record && c) a.ingress_acc[q] += c;
}

// PushActiveSet::prune (push_active_set.rs:56-71,143-151) for (prunee u, pruner v) of slot o.
template <int ASZP>
__device__ inline void apply_prune(const CgArgs& a, uint32_t o, uint32_t ob, uint32_t u, uint32_t v) {
  const uint32_t bu = a.bucket[u], k = min(bu, ob);
  uint32_t row[ASZP], hv;
  if (a.own && k == bu) {  // the own-bucket row (64 B, cache-resident) instead of the full table's
    const uint32_t* orow = a.own + (size_t)u * a.ORW;
    load_row<ASZP>(orow, row);
    hv = orow[ASZP] & 0xFFFFu;
  } else {
    const uint32_t ent = u * NB + k;
    hv = a.hl[ent];
    load_row<ASZP>(a.peers + (size_t)ent * ASZP, row);
  }
  const uint32_t head = hv & 0xFF, L = hv >> 8;
  uint32_t hit = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    const uint32_t pos = (uint32_t)s >= head ? (uint32_t)s - head : (uint32_t)s + a.ASZ - head;
    hit |= (uint32_t)((uint32_t)s < a.ASZ && pos < L && row[s] == v) << s;
  }
  if (hit) atomicOr(&a.mask[o * a.mso + u * a.msu], hit);
}

// ---- prune, register path (len <= 32) ----
// Prunes found by a lane are appended (by ballot, in step order) to its wave's LDS list
// (prunee id, pruner lane) and applied afterwards by all 64 lanes, one list entry each:
// applied in place, a lane's prunes were one dependent row load after another, and
// the wave waited for its longest entry's chain (a prune wave's 42 M prunes at C4).
constexpr uint32_t CG_PL = 1024;  // per-wave deferred prunes (beyond: applied in place)
struct PruneList {
  uint32_t* u;
  uint8_t* lane;
  uint32_t n;  // wave-uniform among the lanes in the prune path
};

// Entries [0, W) of a lane's cache entry (keys ~0 beyond its length): each entry's position
// in prune order = the number of smaller keys (keys are distinct), its pre-add cumulative
// stake = the saturating sum of their stakes (order-free); the rows are rewritten in prune
// order with the pruned flag, prunes are appended to the wave's list.
template <int ASZP, int W>
__device__ inline void prune_ranks(const CgArgs& a, uint32_t q, uint32_t o, uint32_t ob, uint32_t org, uint32_t v,
                                   uint32_t len, uint32_t mi, uint64_t mis, const uint32_t (&kk)[LANE_L],
                                   const uint32_t (&nd)[LANE_L], const uint64_t (&st)[LANE_L], PruneList& pl,
                                   uint32_t& npr) {
  uint32_t rk[W], ow[W];
#pragma unroll
  for (int i = 0; i < W; ++i) {
    uint32_t rank = 0;
    uint64_t cum = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const bool lt = kk[j] < kk[i];
      rank += lt ? 1u : 0u;
      cum = sat_add(cum, lt ? st[j] : 0ull);
    }
    const bool live = (uint32_t)i < len;
    const bool pruned = live && rank >= mi && cum >= mis && nd[i] != org;
    rk[i] = rank;
    ow[i] = ck_make(nd[i], (0x7Fu - (kk[i] >> 24)) | (pruned ? PRUNED_FLAG : 0u));
    npr += pruned ? 1u : 0u;
    const uint64_t pb = __ballot(pruned);
    if (pruned) {
      const uint32_t k = pl.n + __builtin_amdgcn_mbcnt_hi((uint32_t)(pb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pb, 0u));
      if (k < CG_PL) {
        pl.u[k] = nd[i];
        pl.lane[k] = (uint8_t)lane_id();
      } else {
        apply_prune<ASZP>(a, o, ob, nd[i], v);
      }
    }
    pl.n += (uint32_t)__popcll(pb);
  }
  // the rows rewritten position by position: every lane stores to row p together (one
  // coalesced store per position instead of a lane-scattered store per entry)
#pragma unroll
  for (int p = 0; p < W; ++p) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) w = rk[i] == (uint32_t)p ? ow[i] : w;
    if ((uint32_t)p < len) (a.ckey + (size_t)p * a.PAIRS)[q] = w;
  }
}

template <int ASZP>
__device__ inline uint32_t prune_lane(const CgArgs& a, uint32_t q, uint32_t o, uint32_t v, uint32_t len, PruneList& pl) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t org = a.origin[o], ob = a.obkt[o], mi = a.min_ingress[o];
  const uint64_t sv = a.stake[v], so = a.stake[org];
  const uint64_t mis = min_ingress_stake(sv < so ? sv : so, a.thr[o]);
  const uint32_t wl = active_max<5>(len);
  // every entry's cache word, then its node's prune rank and stake (one 16-B load each,
  // all in flight together)
  uint32_t kk[LANE_L], nd[LANE_L];
  uint64_t st[LANE_L];
#pragma unroll
  for (int i = 0; i < (int)LANE_L; ++i) nd[i] = (uint32_t)i < wl ? ntl(&(a.ckey + (size_t)i * PAIRS)[q]) : 0u;
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < (int)LANE_L; ++i) {
    kk[i] = 0xFFFFFFFFu;
    st[i] = 0;
    if ((uint32_t)i < wl) {
      const uint32_t id = (uint32_t)i < len ? ck_id(nd[i]) : 0u;
      const uint4 x = a.pinfo[id];
      kk[i] = (uint32_t)i < len ? (((0x7Fu - ck_score(nd[i])) << 24) | x.x) : 0xFFFFFFFFu;
      st[i] = ((uint64_t)x.w << 32) | x.z;
      nd[i] = id;
    }
  }
  // sorted_unstable_by_key(Reverse((score, stake))), ties by id: entry i's position is the
  // number of smaller keys (keys are distinct), its pre-add cumulative stake the saturating
  // sum of their stakes (order-free); skip(min_ingress_nodes), then skip_while(cum <
  // min_ingress_stake): pruned iff position >= mi and cum >= mis (cum never decreases).
  // The rows are rewritten in prune order with the pruned flag.
  uint32_t npr = 0;
  if (wl <= 8) prune_ranks<ASZP, 8>(a, q, o, ob, org, v, len, mi, mis, kk, nd, st, pl, npr);
  else prune_ranks<ASZP, LANE_L>(a, q, o, ob, org, v, len, mi, mis, kk, nd, st, pl, npr);
  return npr;
}

// A wave's deferred prunes, four lanes per prune: lane j of a quad loads 16 B of the prunee's
// own-bucket row (words 4j..4j+3; its one 64-B line holds the ring, hl | bucket << 16 in
// word ASZP, and the failure classes), the quad ORs its ring-slot hits, and one lane sets
// the mask bits. One coalesced line per prune instead of five scattered loads per lane
// (bucket, three row quads, hl): a prune wave is bound by the texture address unit's
// per-lane work (profiles/r03/pmc_prune_c4.txt: TA busy 84 % of the kernel). A prunee
// whose entry for this origin is not its own bucket (origin bucket below it) takes
// apply_prune.
template <int ASZP>
__device__ inline void apply_prunes_quad(const CgArgs& a, const PruneList& pl, uint32_t pn, uint32_t qb) {
  static_assert(ASZP % 4 == 0 && ASZP <= 12, "one quad of lanes covers the ring and word ASZP");
  constexpr uint32_t NQ = ASZP / 4 + 1;
  const uint32_t l = lane_id(), sub = l & 3u, lead = l & ~3u;
  for (uint32_t k0 = 0; k0 < pn; k0 += 16) {
    const uint32_t k = k0 + (l >> 2);
    const bool ok = k < pn;
    uint32_t u = 0, v = 0, po = 0;
    if (ok) {
      u = pl.u[k];
      const uint32_t pq = qb + pl.lane[k];
      po = pq / a.NP;
      v = a.vlo + (pq - po * a.NP);
    }
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (ok && sub < NQ) w = reinterpret_cast<const uint4*>(a.own + (size_t)u * a.ORW)[sub];
    const uint32_t wm = (uint32_t)__shfl((int)w.x, (int)(lead | (ASZP / 4)));  // word ASZP
    const uint32_t head = wm & 0xFFu, L = (wm >> 8) & 0xFFu, bu = wm >> 16;
    const uint32_t rw[4] = {w.x, w.y, w.z, w.w};
    uint32_t hit = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t s = sub * 4 + (uint32_t)j;
      const uint32_t pos = s >= head ? s - head : s + a.ASZ - head;
      hit |= (uint32_t)(sub < ASZP / 4 && s < a.ASZ && pos < L && rw[j] == v) << s;
    }
    hit |= (uint32_t)__shfl_xor((int)hit, 1);
    hit |= (uint32_t)__shfl_xor((int)hit, 2);
    if (ok && sub == 0) {
      const uint32_t ob = a.obkt[po];
      if (ob >= bu) {
        if (hit) atomicOr(&a.mask[po * a.mso + u * a.msu], hit);
      } else {
        apply_prune<ASZP>(a, po, ob, u, v);
      }
    }
  }
}

// ---- prune, wave path (32 < len <= 96): two entries per lane ----
template <int ASZP>
__device__ inline uint32_t prune_wave(const CgArgs& a, uint32_t q, uint32_t o, uint32_t v, uint32_t len) {
  const size_t PAIRS = a.PAIRS;
  const uint32_t l = lane_id();
  const uint32_t org = a.origin[o], ob = a.obkt[o], mi = a.min_ingress[o];
  const uint64_t sv = a.stake[v], so = a.stake[org];
  const uint64_t mis = min_ingress_stake(sv < so ? sv : so, a.thr[o]);
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
      if (pruned) apply_prune<ASZP>(a, o, ob, nd[t], v);
    }
    npr += (uint32_t)__popcll(__ballot(pruned));
  }
  return npr;
}

__device__ inline void finish_prune(const CgArgs& a, uint32_t q, uint32_t len, uint32_t npr) {
  a.cmeta[q] = len << 16;  // std::mem::take: entry reset, the pruned keys stay readable
  a.prune_round[q] = (uint8_t)(npr < 255 ? npr : 255);
  if (npr && a.record) a.prune_acc[q] += npr;
}

// Adds each lane's prunee count to its slot's total. A block takes a contiguous range of
// pairs, which spans few slots: the counts go to LDS counters (one per slot of the
// range, sc[o - o_lo]) and each block adds them to the S global counters once at its
// end. (S counters share a line or two: a global atomic per wave and slot made a prune
// wave's 200 K atomics at C4 queue on one line, 2.4 of its 4.2 ms.) Slots beyond the
// LDS counters (ranges of tiny slots) add per wave.
constexpr uint32_t CG_SC = 64;
__device__ inline void add_slot_prunes(const CgArgs& a, uint32_t o, uint32_t npr, uint32_t o_lo, uint32_t* sc) {
  const uint32_t o0 = __builtin_amdgcn_readfirstlane(o);
  if (__ballot(o != o0) == 0) {
    uint32_t s = npr;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off);
    if (lane_id() == 0 && s) {
      if (o0 - o_lo < CG_SC) atomicAdd(&sc[o0 - o_lo], s);
      else atomicAdd(&a.slot_prunes[o0], s);
    }
  } else if (npr) {
    if (o - o_lo < CG_SC) atomicAdd(&sc[o - o_lo], npr);
    else atomicAdd(&a.slot_prunes[o], npr);
  }
}

// Kernel 1: consume every pair, queue due prunes. Pairs with in-degree > 16 are taken
// by the whole wave after its lanes finish their own pairs.
__global__ __launch_bounds__(CG_THREADS) void k_cg_consume(CgArgs a) {
  __shared__ uint32_t scr_all[CG_WAVES * CG_SCR];
  uint32_t* scr = scr_all + (threadIdx.x >> 6) * CG_SCR;
  uint32_t errf = 0;
  if (a.zero_sp && blockIdx.x == 0)  // (instead of a memset launch before this kernel)
    for (uint32_t i = threadIdx.x; i < a.S; i += CG_THREADS) a.slot_prunes[i] = 0;
  const uint32_t P = (uint32_t)a.PAIRS;
  for (uint32_t p0 = blockIdx.x * CG_THREADS; p0 < P; p0 += gridDim.x * CG_THREADS) {
    const uint32_t q = p0 + threadIdx.x;
    const bool in = q < P;
    const uint32_t meta = in ? ntl(&a.cmeta[q]) : 0u;
    uint32_t c = in ? a.cnt[q] : 0u;
    if (c > a.capin) c = a.capin;
    uint32_t len = meta & 0xFF, up = (meta >> 8) & 0xFF;
    const bool heavy = in && c > a.lane_c;
    bool due = false;
    if (in && !heavy) {
      if (c) consume_lane(a, q, c, len, up, errf);
      after_consume(a, q, meta, c, len, up, due);
    }
    uint64_t hv = __ballot(heavy);
    while (hv) {  // the wave's heavy pairs, one at a time
      const int l = __ffsll((long long)hv) - 1;
      hv &= hv - 1;
      const uint32_t hq = (uint32_t)__shfl((int)q, l);
      const uint32_t hmeta = (uint32_t)__shfl((int)meta, l);
      const uint32_t hc = (uint32_t)__shfl((int)c, l);
      uint32_t hlen = hmeta & 0xFF, hup = (hmeta >> 8) & 0xFF;
      if (hc <= a.wave_c) consume_wave(a, hq, hc, hlen, hup, scr, errf);
      else consume_serial(a, hq, hc, hlen, hup, errf);
      bool hdue = false;
      if (lane_id() == 0) after_consume(a, hq, hmeta, hc, hlen, hup, hdue);
    }
  }
  if (errf) atomicOr(a.err, errf);
}

// Kernel 2: send_prunes + prune_connections of the pairs whose entry reached 20
// upserts (a scan of the meta words: no contended worklist counter).
template <int ASZP>
__global__ __launch_bounds__(CG_THREADS) void k_cg_prune(CgArgs a) {
  __shared__ uint32_t pl_u_all[CG_WAVES * CG_PL];
  __shared__ uint8_t pl_l_all[CG_WAVES * CG_PL];
  __shared__ uint32_t sc[CG_SC];  // prunes per slot of this block's range
  const uint32_t wid = threadIdx.x >> 6;
  const uint32_t P = (uint32_t)a.PAIRS;
  // this block's contiguous range of pairs (whole blocks of CG_THREADS)
  const uint32_t nblk = (P + CG_THREADS - 1) / CG_THREADS, per = (nblk + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = min(P, blockIdx.x * per * CG_THREADS), hi = min(P, lo + per * CG_THREADS);
  const uint32_t o_lo = lo / a.NP;
  if (threadIdx.x < CG_SC) sc[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t p0 = lo; p0 < hi; p0 += CG_THREADS) {
    const uint32_t q = p0 + threadIdx.x;
    const uint32_t meta = q < hi ? ntl(&a.cmeta[q]) : 0u;
    const bool due = q < hi && ((meta >> 8) & 0xFF) >= MIN_NUM_UPSERTS;
    if (!__ballot(due)) continue;
    const uint32_t o = q / a.NP, v = a.vlo + (q - o * a.NP);
    const uint32_t len = meta & 0xFF;
    const bool heavy = due && len > a.lane_l;
    uint32_t npr = 0;
    PruneList pl{pl_u_all + wid * CG_PL, pl_l_all + wid * CG_PL, 0u};
    if (due && !heavy) {
      npr = prune_lane<ASZP>(a, q, o, v, len, pl);
      finish_prune(a, q, len, npr);
    }
    uint32_t pn = pl.n;  // (0 in lanes outside the lane path)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) pn = max(pn, (uint32_t)__shfl_xor((int)pn, off));
    pn = min(pn, CG_PL);
    if (pn) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint32_t qb = p0 + (wid << 6);
      bool quad = false;
      if constexpr (ASZP <= 12) {
        quad = a.own != nullptr;
        if (quad) apply_prunes_quad<ASZP>(a, pl, pn, qb);
      }
      if (!quad)
        for (uint32_t k = lane_id(); k < pn; k += 64) {
          const uint32_t pq = qb + pl.lane[k];
          const uint32_t po = pq / a.NP;
          apply_prune<ASZP>(a, po, a.obkt[po], pl.u[k], a.vlo + (pq - po * a.NP));
        }
      __builtin_amdgcn_wave_barrier();  // the list is reused by the wave's next pairs
    }
    uint64_t hv = __ballot(heavy);
    while (hv) {  // the wave's long entries, one at a time
      const int l = __ffsll((long long)hv) - 1;
      hv &= hv - 1;
      const uint32_t hq = (uint32_t)__shfl((int)q, l);
      const uint32_t ho = hq / a.NP, hvn = a.vlo + (hq - ho * a.NP);
      const uint32_t hlen = (uint32_t)__shfl((int)len, l);
      const uint32_t hn = prune_wave<ASZP>(a, hq, ho, hvn, hlen);
      if (lane_id() == 0) finish_prune(a, hq, hlen, hn);
      if ((int)lane_id() == l) npr = hn;
    }
    add_slot_prunes(a, o, npr, o_lo, sc);
  }
  __syncthreads();
  if (threadIdx.x < CG_SC && sc[threadIdx.x]) atomicAdd(&a.slot_prunes[o_lo + threadIdx.x], sc[threadIdx.x]);
}

}  // namespace

// consume_messages + send_prunes + prune_connections of every slot (gs_round's step path).
hipError_t launch_consume_prune_g(Engine& e, bool record, bool consume, bool zero_slot_prunes) {
  CgArgs a;
  a.stake = e.stake; a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.origin = e.origin; a.obkt = e.obkt;
  a.own = e.own; a.ORW = e.ORW;
  a.min_ingress = e.min_ingress; a.thr = e.thr; a.prank = e.prank; a.by_prank = e.by_prank; a.pstake = e.pstake; a.pinfo = e.pinfo;
  a.cnt = e.cnt; a.inb = e.inb; a.cmeta = e.cmeta; a.ckey = e.ckey; a.prune_round = e.prune_round;
  a.slot_prunes = e.slot_prunes; a.mask = e.mask; a.ingress_acc = e.ingress_acc; a.prune_acc = e.prune_acc;
  a.NP = e.NP; a.vlo = e.vlo;
  a.err = e.err;
  a.N = e.N; a.S = e.S; a.ASZ = e.ASZ; a.capin = e.capin; a.PAIRS = e.PAIRS; a.record = record ? 1 : 0;
  a.mso = e.mso;
  a.msu = e.msu;
  const bool narrow = (e.prm.flags & GS_FLAG_NARROW_WAVE_PATH) != 0;
  a.zero_sp = consume && zero_slot_prunes ? 1 : 0;
  a.lane_c = narrow ? 4u : 16u;
  a.lane_l = narrow ? 4u : LANE_L;
  a.wave_c = narrow ? 8u : 64u;
  // (slot_prunes was zeroed by the caller, or is by k_cg_consume when zero_slot_prunes)
  const uint32_t grid = (uint32_t)std::min<size_t>((e.PAIRS + CG_THREADS - 1) / CG_THREADS, 8192);
  if (consume) hipLaunchKernelGGL(k_cg_consume, dim3(grid), dim3(CG_THREADS), 0, e.st, a);
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_cg_prune<A>, dim3(grid), dim3(CG_THREADS), 0, e.st, a));
  return hipGetLastError();
}

}  // namespace gs
