// gs_bfs_binned.hip -- Cluster::run_gossip (gossip.rs:494-615) for large clusters:
// level-synchronous BFS over every slot at once, propagation-blocked, with the
// inbound records grouped by destination only once per round.
//
// A push is a scatter: (destination pair, source) lands at a random pair. Scattered
// global atomics and 4-byte stores cost a 64-128 B memory transaction each on
// gfx950, so here no push is ever written to its destination directly. Pairs are
// cut into bins of 2^BS consecutive pair indices; per BFS level:
//
//   expand (workgroup w owns frontier positions [w*PW, (w+1)*PW)): loads each
//     frontier pair's active-set row -- from the compact own-entry table when the
//     origin's bucket allows (push_active_set.rs:38-52: entry min(bucket[u],
//     bucket[origin])) -- takes the first `fanout` unpruned, non-origin peers
//     (failed peers burn a slot), counts pushes per bin in LDS (the atomic's return
//     is the push's rank in its bin), stages the records sorted by bin in LDS and
//     writes them out as one contiguous run; T[w][b] = the run's bin starts.
//   apply (one workgroup per bin, bins dealt to XCDs in contiguous ranges so that
//     the T rows and area lines a bin reads are shared in its XCD's L2): walks the
//     bin's segment of every expand workgroup, marks first arrivals in an LDS
//     bitmap seeded from the bin's hops (first arrival = hop d+1, gossip.rs:594-600),
//     appends the level's records (local pair, hop<<24 | src) to a pool run of its
//     own, writes the bin's hops back and appends the new frontier in pair order.
//   gather (after the last level, one workgroup per bin): counts the bin's records
//     per pair over all levels, builds the inbound lists as a CSR in LDS and writes
//     the rows inb[k][pair] (k < in-degree) and the in-degrees cnt[pair] coalesced.
//
// Results equal k_bfs_level's: hops, in-degrees, the inbound record SET of each pair
// (consume sorts them by (hop, src), gossip.rs:639-645), egress, frontier sizes.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>
#include <vector>
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

constexpr uint32_t X_PPT = 4;          // frontier pairs per expand thread
constexpr uint32_t APPLY_THREADS = 256;
constexpr uint32_t GATHER_THREADS_S = 512, GATHER_THREADS_L = 1024;
constexpr uint32_t SEG_CHUNK = 1024;   // expand workgroups' segments scanned per apply chunk

struct BinArgs {
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
  const uint32_t* own;   // [N][ORW] own-bucket entry rows; word ASZP = hl | bucket << 16
  const uint32_t* frank;
  const uint32_t* origin;
  const uint8_t* obkt;
  const uint32_t* nfail;
  const uint32_t* mask;
  uint8_t* hops;
  uint32_t* cnt;
  uint32_t* inb;
  uint8_t* egress;
  uint32_t* egress_acc;
  uint32_t* lvl;
  uint32_t* err;
  void* area;      // expand -> apply: workgroup w's records sorted by bin at w*PW*fc (RecW / RecN)
  uint32_t* T;     // [Gmax][nbins + 1] bin starts of each expand workgroup's run (+ its total)
  void* pool;      // apply -> gather: per (level, bin) runs (RecW / RecN)
  uint2* Lt;       // [256][nbins] (pool start, count) of bin b's run at level d
  uint32_t* binoff;  // [nbins] records in bin b's pool region so far this round (only bin b's apply touches it)
  uint32_t* visbm;  // [PAIRS / 32] visited pairs (hop != unreached) of this round
  uint32_t* hlvl;   // host-mapped [256]: expand(d) writes level d's frontier size (the polled loop)
  uint32_t* dpair;  // [258] level of expand/apply pair i (predicted loop): head writes [0], pair i [i + 1]
  uint32_t* hprof;  // host-mapped: the tail kernel's level profile (seq, levels, sizes)
  uint32_t N, ASZ, fanout, fc, capin, Gmax, PW, BS, nbins, ORW, csr_cap, qmin;
  size_t PAIRS, pool_bin_cap;  // pool region of a bin: 2^BS * capin records (in-degrees are <= capin)
  int record;
};

// bins dealt to XCDs in contiguous ranges (workgroup i runs on XCD i % 8)
__device__ inline uint32_t xcd_bin(uint32_t i, uint32_t nbins) {
  const uint32_t per = (nbins + 7) / 8;
  return (i & 7u) * per + (i >> 3);
}

// Record formats. Wide (uint2): area (pair, src), pool (local pair, hop << 24 | src).
// Narrow (u32, bins of 2^11 pairs and N <= 2^21): area and pool (local pair << 21 | src);
// the bin is known from the segment/run and the hop from the level.
constexpr uint32_t NARROW_SRC_BITS = 21, NARROW_BS = 11;
struct RecW {
  using T = uint2;
  __device__ static T area(uint32_t q, uint32_t u, uint32_t) { return make_uint2(q, u); }
  __device__ static uint32_t area_ql(T r, uint32_t q0) { return r.x - q0; }
  __device__ static uint32_t area_src(T r) { return r.y; }
  __device__ static T pool(uint32_t ql, uint32_t hopv, uint32_t src) { return make_uint2(ql, hopv | src); }
  __device__ static uint32_t pool_ql(T r) { return r.x; }
  __device__ static uint32_t pool_val(T r, uint32_t) { return r.y; }
};
struct RecN {
  using T = uint32_t;
  __device__ static T area(uint32_t q, uint32_t u, uint32_t BPm) { return ((q & BPm) << NARROW_SRC_BITS) | u; }
  __device__ static uint32_t area_ql(T r, uint32_t) { return r >> NARROW_SRC_BITS; }
  __device__ static uint32_t area_src(T r) { return r & ((1u << NARROW_SRC_BITS) - 1); }
  __device__ static T pool(uint32_t ql, uint32_t, uint32_t src) { return (ql << NARROW_SRC_BITS) | src; }
  __device__ static uint32_t pool_ql(T r) { return r >> NARROW_SRC_BITS; }
  __device__ static uint32_t pool_val(T r, uint32_t hopv) { return hopv | (r & ((1u << NARROW_SRC_BITS) - 1)); }
};

// The pushes of frontier pair p (gossip.rs:511-541): ring slots taken this round.
template <int ASZP>
__device__ inline uint32_t pair_pushes(const BinArgs& a, uint32_t p, uint32_t (&row)[ASZP], uint32_t& o,
                                       uint32_t& u) {
  o = p / a.N;
  u = p - o * a.N;
  const uint32_t org = a.origin[o], nf = a.nfail[o], ob = a.obkt[o];
  const uint32_t* orow = a.own + (size_t)u * a.ORW;
  load_row<ASZP>(orow, row);
  const uint32_t meta = orow[ASZP];
  uint32_t hv = meta & 0xFFFFu;
  if ((meta >> 16) > ob) {  // the origin's bucket is lower: entry min(bucket[u], bucket[origin])
    const uint32_t ent = u * NB + ob;
    hv = a.hl[ent];
    load_row<ASZP>(a.peers + (size_t)ent * ASZP, row);
  }
  uint32_t pushm = taken_slots<ASZP>(row, hv & 0xFF, hv >> 8, a.ASZ, a.mask[p], org, a.fanout);
  if (nf) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
    for (int s = 0; s < ASZP; ++s)
      if (((pushm >> s) & 1u) && a.frank[row[s]] < nf) pushm &= ~(1u << s);
  }
  return pushm;
}

// Exclusive scan of LDS h[0..n) in place by the whole workgroup; wsum holds 16 words.
__device__ inline uint32_t block_excl_scan(uint32_t* h, uint32_t n, uint32_t* wsum) {
  const uint32_t TH = blockDim.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = TH >> 6;
  const uint32_t per = (n + TH - 1) / TH;
  const uint32_t lo = min(n, tid * per), hi = min(n, lo + per);
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += h[i];
  const uint32_t incl = wave_incl_scan(s);
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (uint32_t k = 0; k < nw; ++k) {
    if (k < wid) wb += wsum[k];
    tot += wsum[k];
  }
  uint32_t run = wb + incl - s;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = h[i];
    h[i] = run;
    run += c;
  }
  __syncthreads();
  return tot;
}

__host__ __device__ inline size_t bin_expand_lds_bytes(uint32_t nbins, uint32_t PW, uint32_t fc, uint32_t rec_bytes) {
  return 4 * (size_t)((nbins + 16 + 1) & ~1u) + rec_bytes * (size_t)PW * fc;
}

// Levels with fewer than qmin (BIN_MIN_FRONTIER) frontier pairs: one thread per frontier pair,
// a global in-degree atomic per push (cheap when there are few) that also gives the
// record's inbound slot; first visits from the round's visited bitmap, shared with the
// binned levels. The gather places the binned levels' records after these slots.
constexpr uint32_t BIN_MIN_FRONTIER = 1u << 17;

// WG: run by the single-workgroup kernel (k_bin_small): its atomics are workgroup scope
// (executed in the XCD's L2, atomic_or_wg); the grid-wide expand's are device scope.
template <int ASZP, bool WG = false>
__device__ inline void bin_direct(const BinArgs& a, uint32_t d, uint32_t qn, const uint32_t* __restrict__ qcur,
                                  uint32_t* __restrict__ qnxt) {
  const uint32_t rec_hop = (d + 1) << 24;
  bool overflow = false;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < qn; i0 += gridDim.x * blockDim.x) {  // uniform trips
    const uint32_t i = i0 + threadIdx.x;
    uint32_t row[ASZP], pm = 0, o = 0, u = 0;
#pragma unroll
    for (int s = 0; s < ASZP; ++s) row[s] = 0;
    if (i < qn) {
      uint32_t p = qcur[i];
      if (GS_OOB(p, a.PAIRS, a.err, "direct frontier pair")) p = 0;
      pm = pair_pushes<ASZP>(a, p, row, o, u);
      const uint32_t eg = __popc(pm);
      a.egress[p] = (uint8_t)eg;
      if (a.record && eg) a.egress_acc[p] += eg;
    }
    const uint32_t qb = o * a.N;
    uint32_t slot[ASZP], vold[ASZP];
#pragma unroll
    for (int s = 0; s < ASZP; ++s) {  // all atomics back to back, then their results
      const uint32_t q = qb + row[s];
      const bool on = (pm >> s) & 1u;
      slot[s] = on ? (WG ? atomic_add_wg(&a.cnt[q], 1u) : atomicAdd(&a.cnt[q], 1u)) : 0u;
      vold[s] = on ? (WG ? atomic_or_wg(&a.visbm[q >> 5], 1u << (q & 31)) : atomicOr(&a.visbm[q >> 5], 1u << (q & 31)))
                   : ~0u;
    }
    uint32_t newm = 0;
#pragma unroll
    for (int s = 0; s < ASZP; ++s) {
      if (!((pm >> s) & 1u)) continue;
      const uint32_t q = qb + row[s];
      if (slot[s] < a.capin) a.inb[(size_t)slot[s] * a.PAIRS + q] = rec_hop | u;
      else overflow = true;
      if (!((vold[s] >> (q & 31)) & 1u)) {  // first visit: hop = dist[src] + 1 (gossip.rs:594-600)
        newm |= 1u << s;
        a.hops[q] = (uint8_t)(d + 1);
      }
    }
    const uint32_t k = __popc(newm);
    const uint32_t incl = wave_incl_scan(k);
    const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
    uint32_t qbase = 0;
    if (lane_id() == 63 && tot) qbase = WG ? atomic_add_wg(&a.lvl[d + 1], tot) : atomicAdd(&a.lvl[d + 1], tot);
    uint32_t pos = (uint32_t)__shfl((int)qbase, 63) + incl - k;
#pragma unroll
    for (int s = 0; s < ASZP; ++s)
      if ((newm >> s) & 1u) qnxt[pos++] = qb + row[s];
  }
  if (overflow) atomicOr(a.err, ERR_INBOUND);
}

// A level with fewer than qmin frontier pairs runs bin_direct in this same launch
// (no dispatch of its own); a larger one is expanded into bin runs for k_bin_apply.
// Direct levels of at most BIN_SMALL frontier pairs run inside ONE workgroup, level after
// level, with no launch between them (bin_direct's device-scope atomics order the
// level's first arrivals; the next level's size is read after a barrier). Starts at
// level d0; stops at the first level with no pairs, more than BIN_SMALL, or at qmin;
// writes (level, pairs) to the host-mapped hstate.
constexpr uint32_t BIN_SMALL = 1024, BIN_ST = 1024;
constexpr uint32_t BIN_NOPAIR = 0xFFFFFFFFu;
enum : uint32_t { BIN_POLL = 0, BIN_HEAD = 1, BIN_TAIL = 2 };
// Modes: BIN_POLL from level d0 while levels have at most lim pairs (the polled loop);
// BIN_HEAD the same from level 0, leaving the level where it stopped in dpair[0] for the
// expand/apply pairs of the predicted loop; BIN_TAIL from level dpair[pi] to the end of
// the BFS whatever the sizes (correct for any level, fast for the small tail), publishing
// the round's level profile (hprof) for the host's next prediction.
template <int ASZP>
__global__ __launch_bounds__(BIN_ST) void k_bin_small(BinArgs a, uint32_t mode, uint32_t d0, uint32_t pi, uint32_t lim,
                                                     uint32_t* __restrict__ q0, uint32_t* __restrict__ q1,
                                                     uint32_t* __restrict__ hstate, uint32_t seq) {
  __shared__ uint32_t s_qn;
  uint32_t d = mode == BIN_TAIL ? a.dpair[pi] : d0;
  if (mode == BIN_TAIL) lim = 0xFFFFFFFFu;
  if (threadIdx.x == 0) s_qn = d < 256 ? a.lvl[d] : 0u;
  __syncthreads();
  uint32_t qn = s_qn;
  while (qn > 0 && qn <= lim && d < 254) {
    if (threadIdx.x == 0 && mode == BIN_POLL) __hip_atomic_store(&a.hlvl[d], qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    bin_direct<ASZP, true>(a, d, qn, (d & 1) ? q1 : q0, (d & 1) ? q0 : q1);
    __syncthreads();
    if (threadIdx.x == 0) s_qn = __hip_atomic_load(&a.lvl[d + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    qn = s_qn;
    ++d;
  }
  if (threadIdx.x == 0) {
    if (mode == BIN_HEAD) a.dpair[0] = d;
    if (mode == BIN_TAIL) {
      if (qn > 0) atomicOr(a.err, ERR_DEPTH);  // level 254 not empty
      const uint32_t nl = min(d, 255u);
      // seqlock: 0 (in progress, the host skips it) before the sizes, the new seq after
      __hip_atomic_store(&a.hprof[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __atomic_thread_fence(__ATOMIC_RELEASE);
      for (uint32_t k = 0; k < nl; ++k)
        __hip_atomic_store(&a.hprof[2 + k], __hip_atomic_load(&a.lvl[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&a.hprof[1], nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&a.hprof[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&hstate[1], qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hstate[0], d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // the host polls this word
  }
}

// Level d (pi == BIN_NOPAIR), or pair pi's level dpair[pi] (the predicted loop; no
// entries there when the BFS already ended). A level below qmin, or any level when no
// apply follows (binned == 0), runs the direct path here; pair pi then records its next
// level in dpair[pi + 1] (the apply does when it runs).
template <int ASZP, class R>
__global__ __launch_bounds__(512) void k_bin_expand(BinArgs a, uint32_t d, uint32_t pi, uint32_t binned,
                                                    uint32_t* __restrict__ q0, uint32_t* __restrict__ q1) {
  using RT = typename R::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (pi != BIN_NOPAIR) d = a.dpair[pi];
  const uint32_t qn = d < 254 ? a.lvl[d] : 0u;
  const uint32_t* __restrict__ qcur = (d & 1) ? q1 : q0;
  uint32_t* __restrict__ qnxt = (d & 1) ? q0 : q1;
  if (pi == BIN_NOPAIR && blockIdx.x == 0 && threadIdx.x == 0)  // the host's level poll (host-mapped)
    __hip_atomic_store(&a.hlvl[d], qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (qn < a.qmin || !binned) {
    if (pi != BIN_NOPAIR && blockIdx.x == 0 && threadIdx.x == 0) a.dpair[pi + 1] = qn ? d + 1 : d;
    bin_direct<ASZP>(a, d, qn, qcur, qnxt);
    return;
  }
  const uint32_t G = (qn + a.PW - 1) / a.PW;
  const uint32_t nb = a.nbins, BS = a.BS, tid = threadIdx.x, TH = blockDim.x;
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);                               // [nb] + 16
  RT* stage = reinterpret_cast<RT*>(smem + 4 * (size_t)((nb + 16 + 1) & ~1u));  // [PW * fc]
  const uint32_t BPm = (1u << BS) - 1;
  for (uint32_t w = blockIdx.x; w < G; w += gridDim.x) {  // workgroup slices, grid <= 2 per CU
    const uint32_t lo = w * a.PW, hi = min(qn, lo + a.PW);
    for (uint32_t i = tid; i < nb; i += TH) hist[i] = 0;
    __syncthreads();
    uint32_t row[X_PPT][ASZP], rk[X_PPT][ASZP], pm[X_PPT], qb[X_PPT], uu[X_PPT];
#pragma unroll
    for (uint32_t j = 0; j < X_PPT; ++j) {
      const uint32_t i = lo + j * TH + tid;
      pm[j] = 0; qb[j] = 0; uu[j] = 0;
      if (i < hi) {
        uint32_t p = qcur[i];
        if (GS_OOB(p, a.PAIRS, a.err, "binned frontier pair")) p = 0;
        uint32_t o, u;
        pm[j] = pair_pushes<ASZP>(a, p, row[j], o, u);
        const uint32_t eg = __popc(pm[j]);
        a.egress[p] = (uint8_t)eg;
        if (a.record && eg) a.egress_acc[p] += eg;
        qb[j] = o * a.N;
        uu[j] = u;
      } else {
#pragma unroll
        for (int s = 0; s < ASZP; ++s) row[j][s] = 0;
      }
    }
    // every LDS atomic after every load: the rank of each push within its bin
#pragma unroll
    for (uint32_t j = 0; j < X_PPT; ++j)
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        rk[j][s] = ((pm[j] >> s) & 1u) ? atomicAdd(&hist[(qb[j] + row[j][s]) >> BS], 1u) : 0u;
    __syncthreads();
    const uint32_t total = block_excl_scan(hist, nb, hist + nb);
    uint32_t* Tw = a.T + (size_t)w * (nb + 1);
    for (uint32_t b = tid; b < nb; b += TH) Tw[b] = hist[b];
    if (tid == 0) Tw[nb] = total;
#pragma unroll
    for (uint32_t j = 0; j < X_PPT; ++j)
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if ((pm[j] >> s) & 1u) {
          const uint32_t q = qb[j] + row[j][s];
          stage[hist[q >> BS] + rk[j][s]] = R::area(q, uu[j], BPm);
        }
    __syncthreads();
    RT* area = reinterpret_cast<RT*>(a.area) + (size_t)w * a.PW * a.fc;
    for (uint32_t i = tid; i < total; i += TH) area[i] = stage[i];
    __syncthreads();
  }
}

// apply LDS: pre [SEG_CHUNK + 1], sb [SEG_CHUNK], vis / vis0 bitmaps [BP / 32], control
__host__ __device__ inline size_t bin_apply_lds_bytes(uint32_t BS) {
  return 4 * (2 * (size_t)SEG_CHUNK + 1 + 2 * (((size_t)1 << BS) / 32) + 32);
}

template <class R>
__global__ __launch_bounds__(APPLY_THREADS) void k_bin_apply(BinArgs a, uint32_t d, uint32_t pi, uint32_t* __restrict__ qa,
                                                            uint32_t* __restrict__ qb) {
  using RT = typename R::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (pi != BIN_NOPAIR) d = a.dpair[pi];
  const uint32_t qn = d < 254 ? a.lvl[d] : 0u;
  uint32_t* __restrict__ qnxt = (d & 1) ? qa : qb;
  if (qn == 0 || qn < a.qmin) return;  // (a direct level: no Lt entry, the gather skips it)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (pi != BIN_NOPAIR) a.dpair[pi + 1] = d + 1;
    a.lvl[256 + d] = 1;  // level d's records are in Lt[d] (the gather reads them only then)
  }
  const uint32_t b = xcd_bin(blockIdx.x, a.nbins);
  if (b >= a.nbins) return;
  const uint32_t tid = threadIdx.x, nb = a.nbins, BP = 1u << a.BS, NW = BP / 32;
  const uint32_t G = (qn + a.PW - 1) / a.PW;
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem);  // [SEG_CHUNK + 1]
  uint32_t* sb = pre + SEG_CHUNK + 1;                 // [SEG_CHUNK]
  uint32_t* vis = sb + SEG_CHUNK;                     // [NW]
  uint32_t* vis0 = vis + NW;                          // [NW]
  uint32_t* ctl = vis0 + NW;                          // [0] pool base, [1] frontier base, [2] err, [8..23] scan
  const uint32_t q0 = b << a.BS;
  // 1. the bin's record count this level (T rows of every expand workgroup)
  uint32_t cntp = 0;
  for (uint32_t w = tid; w < G; w += APPLY_THREADS) {
    const uint32_t* Tw = a.T + (size_t)w * (nb + 1);
    cntp += Tw[b + 1] - Tw[b];  // starts are exclusive and Tw[nb] is the run's total
  }
  {
    const uint32_t s = wave_incl_scan(cntp);
    if ((tid & 63) == 63) ctl[8 + (tid >> 6)] = s;
  }
  if (tid < NW) {  // the bin's visited bits (hop != unreached)
    const uint32_t m = a.visbm[(q0 >> 5) + tid];
    vis[tid] = m;
    vis0[tid] = m;
  }
  __syncthreads();
  uint32_t total = 0;
  for (uint32_t k = 0; k < APPLY_THREADS / 64; ++k) total += ctl[8 + k];
  uint2* Ltd = a.Lt + (size_t)d * nb;
  if (total == 0) {
    if (tid == 0) Ltd[b] = make_uint2(0, 0);
    return;
  }
  // 2. the level's pool run for this bin
  if (tid == 0) {  // the bin's own pool region: no device-wide counter; Lt holds the bin-relative start
    const uint32_t used = a.binoff[b];
    ctl[0] = used;
    ctl[2] = 0;
    if ((size_t)used + total > a.pool_bin_cap) { atomicOr(a.err, ERR_INBOUND); ctl[2] = 1; }
    else a.binoff[b] = used + total;
    Ltd[b] = make_uint2(used, ctl[2] ? 0u : total);
  }
  __syncthreads();
  RT* const bpool = reinterpret_cast<RT*>(a.pool) + (size_t)b * a.pool_bin_cap;  // (64-bit: the pool passes 2^32 records)
  const uint32_t pbase = ctl[0];
  const bool pool_ok = ctl[2] == 0;
  // 3. the records, one thread each, in chunks of SEG_CHUNK expand workgroups
  const uint32_t rec_hop = (d + 1) << 24;
  uint32_t done = 0;
  for (uint32_t c0 = 0; c0 < G; c0 += SEG_CHUNK) {
    const uint32_t gc = min(SEG_CHUNK, G - c0);
    for (uint32_t i = tid; i < gc; i += APPLY_THREADS) {
      const uint32_t* Tw = a.T + (size_t)(c0 + i) * (nb + 1);
      const uint32_t st = Tw[b];
      pre[i] = Tw[b + 1] - st;
      sb[i] = st;
    }
    __syncthreads();
    const uint32_t ct = block_excl_scan(pre, gc, ctl + 8);
    if (tid == 0) pre[gc] = ct;
    __syncthreads();
    for (uint32_t r = tid; r < ct; r += APPLY_THREADS) {
      uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= r) lo = mid; else hi = mid;
      }
      const RT rec = reinterpret_cast<const RT*>(a.area)[(size_t)(c0 + lo) * a.PW * a.fc + sb[lo] + (r - pre[lo])];
      uint32_t ql = R::area_ql(rec, q0);
      if (GS_OOB(ql, BP, a.err, "binned record pair")) ql = 0;
      if (pool_ok) bpool[pbase + done + r] = R::pool(ql, rec_hop, R::area_src(rec));
      atomicOr(&vis[ql >> 5], 1u << (ql & 31));
    }
    done += ct;
    __syncthreads();
  }
  // 4. first arrivals (hop d + 1) and the next frontier in pair order; one bitmap
  //    word per thread (NW <= APPLY_THREADS)
  const uint32_t m = tid < NW ? (vis[tid] & ~vis0[tid]) : 0u;
  const uint32_t c = __popc(m);
  const uint32_t incl = wave_incl_scan(c);
  if ((tid & 63) == 63) ctl[8 + (tid >> 6)] = incl;
  __syncthreads();
  uint32_t off = 0, tnew = 0;
  for (uint32_t k = 0; k < APPLY_THREADS / 64; ++k) {
    if (k < (tid >> 6)) off += ctl[8 + k];
    tnew += ctl[8 + k];
  }
  if (tnew == 0) return;
  if (tid == 0) ctl[1] = atomicAdd(&a.lvl[d + 1], tnew);
  if (m) a.visbm[(q0 >> 5) + tid] = vis[tid];
  __syncthreads();
  uint32_t pos = ctl[1] + off + incl - c;
  for (uint32_t mm = m; mm; mm &= mm - 1) {
    const uint32_t q = q0 + tid * 32 + __ffs(mm) - 1;
    qnxt[pos++] = q;
    a.hops[q] = (uint8_t)(d + 1);
  }
}

// Wide records carry their global pair index, so one apply workgroup can take a SUPER-BIN
// of 2^SB_LOG consecutive bins: the rows of T are read once per super-bin (one range
// [T[w][b0], T[w][b0 + 16]) per expand workgroup) instead of once per bin -- with
// thousands of bins (10M-node clusters) every bin's workgroup read a scattered word of
// every T row, twice. Each record goes to its own bin's pool region (per-bin cursors in
// LDS); first arrivals and the next frontier as in k_bin_apply.
constexpr uint32_t SB_LOG = 2, SB_N = 1u << SB_LOG;  // C5: 4,017 us of BFS per round at 4 bins, 4,067 at 2, 4,548 at 8, 5,755 at 16; 4,811 per bin
__host__ __device__ inline size_t bin_apply_sb_lds_bytes(uint32_t BS) {
  return 4 * (2 * (size_t)SEG_CHUNK + 1 + 2 * SB_N * (((size_t)1 << BS) / 32) + 2 * SB_N + 64);
}

__global__ __launch_bounds__(APPLY_THREADS) void k_bin_apply_sb(BinArgs a, uint32_t d, uint32_t pi,
                                                               uint32_t* __restrict__ qa, uint32_t* __restrict__ qb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (pi != BIN_NOPAIR) d = a.dpair[pi];
  const uint32_t qn = d < 254 ? a.lvl[d] : 0u;
  uint32_t* __restrict__ qnxt = (d & 1) ? qa : qb;
  if (qn == 0 || qn < a.qmin) return;  // (a direct level: no Lt entry, the gather skips it)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (pi != BIN_NOPAIR) a.dpair[pi + 1] = d + 1;
    a.lvl[256 + d] = 1;  // level d's records are in Lt[d] (the gather reads them only then)
  }
  const uint32_t nb = a.nbins, nsb = (nb + SB_N - 1) >> SB_LOG;
  const uint32_t B = xcd_bin(blockIdx.x, nsb);
  if (B >= nsb) return;
  const uint32_t tid = threadIdx.x, BS = a.BS, BP = 1u << BS, NW = BP / 32;
  const uint32_t b0 = B << SB_LOG, nbb = min(SB_N, nb - b0), NWS = nbb * NW;
  const uint32_t G = (qn + a.PW - 1) / a.PW;
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem);  // [SEG_CHUNK + 1]
  uint32_t* sb = pre + SEG_CHUNK + 1;                 // [SEG_CHUNK]
  uint32_t* vis = sb + SEG_CHUNK;                     // [SB_N * NW]
  uint32_t* vis0 = vis + SB_N * NW;                   // [SB_N * NW]
  uint32_t* cur = vis0 + SB_N * NW;                   // [SB_N] records appended per bin this level
  uint32_t* bo = cur + SB_N;                          // [SB_N] the bins' pool fills before this level
  uint32_t* ctl = bo + SB_N;                          // [64]: [1] frontier base, [8..] scan words
  const size_t q0 = (size_t)b0 << BS;                 // the super-bin's first pair
  for (uint32_t i = tid; i < NWS; i += APPLY_THREADS) {
    const uint32_t m = a.visbm[(q0 >> 5) + i];
    vis[i] = m;
    vis0[i] = m;
  }
  if (tid < SB_N) {
    cur[tid] = 0;
    bo[tid] = tid < nbb ? a.binoff[b0 + tid] : 0u;
  }
  __syncthreads();
  const uint32_t rec_hop = (d + 1) << 24;
  const uint2* area = reinterpret_cast<const uint2*>(a.area);
  uint2* pool = reinterpret_cast<uint2*>(a.pool);
  for (uint32_t c0 = 0; c0 < G; c0 += SEG_CHUNK) {
    const uint32_t gc = min(SEG_CHUNK, G - c0);
    for (uint32_t i = tid; i < gc; i += APPLY_THREADS) {
      const uint32_t* Tw = a.T + (size_t)(c0 + i) * (nb + 1);
      const uint32_t st = Tw[b0];
      pre[i] = Tw[b0 + nbb] - st;  // (Tw[nb] is the run's total: b0 + nbb <= nb)
      sb[i] = st;
    }
    __syncthreads();
    const uint32_t ct = block_excl_scan(pre, gc, ctl + 8);
    if (tid == 0) pre[gc] = ct;
    __syncthreads();
    for (uint32_t r = tid; r < ct; r += APPLY_THREADS) {
      uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= r) lo = mid; else hi = mid;
      }
      const uint2 rec = area[(size_t)(c0 + lo) * a.PW * a.fc + sb[lo] + (r - pre[lo])];
      uint32_t ql = (uint32_t)(rec.x - q0);  // pair within the super-bin
      if (GS_OOB(ql, nbb * BP, a.err, "binned record pair")) ql = 0;
      const uint32_t j = ql >> BS;
      const uint32_t pos = atomicAdd(&cur[j], 1u);
      if ((size_t)bo[j] + pos < a.pool_bin_cap)
        pool[(size_t)(b0 + j) * a.pool_bin_cap + bo[j] + pos] = RecW::pool(ql & (BP - 1), rec_hop, rec.y);
      atomicOr(&vis[ql >> 5], 1u << (ql & 31));
    }
    __syncthreads();
  }
  uint2* Ltd = a.Lt + (size_t)d * nb;
  if (tid < nbb) {  // each bin's run of this level
    const uint32_t used = bo[tid], n = cur[tid];
    const bool over = (size_t)used + n > a.pool_bin_cap;
    if (over) atomicOr(a.err, ERR_INBOUND);
    Ltd[b0 + tid] = make_uint2(used, over ? 0u : n);  // bin-relative start (the gather adds the bin's base)
    if (!over) a.binoff[b0 + tid] = used + n;
  }
  // first arrivals (hop d + 1) and the next frontier in pair order: a contiguous run of
  // bitmap words per thread
  const uint32_t per = (NWS + APPLY_THREADS - 1) / APPLY_THREADS;
  const uint32_t wlo = min(NWS, tid * per), whi = min(NWS, wlo + per);
  uint32_t c = 0;
  for (uint32_t w = wlo; w < whi; ++w) c += __popc(vis[w] & ~vis0[w]);
  const uint32_t incl = wave_incl_scan(c);
  if ((tid & 63) == 63) ctl[8 + (tid >> 6)] = incl;
  __syncthreads();
  uint32_t off = 0, tnew = 0;
  for (uint32_t k = 0; k < APPLY_THREADS / 64; ++k) {
    if (k < (tid >> 6)) off += ctl[8 + k];
    tnew += ctl[8 + k];
  }
  if (tnew == 0) return;
  if (tid == 0) ctl[1] = atomicAdd(&a.lvl[d + 1], tnew);
  __syncthreads();
  uint32_t pos = ctl[1] + off + incl - c;
  for (uint32_t w = wlo; w < whi; ++w) {
    const uint32_t m = vis[w] & ~vis0[w];
    if (!m) continue;
    a.visbm[(q0 >> 5) + w] = vis[w];
    for (uint32_t mm = m; mm; mm &= mm - 1) {
      const uint32_t q = (uint32_t)(q0 + w * 32 + __ffs(mm) - 1);
      qnxt[pos++] = q;
      a.hops[q] = (uint8_t)(d + 1);
    }
  }
}

// gather LDS: direct-level in-degrees [BP], binned counts [BP], CSR cursors [BP], CSR [csr_cap],
// per-level run table [3][256] + prefix [257], scan words
constexpr uint32_t G_CACHE = 24;  // pool records per thread kept in registers between the passes
__host__ __device__ inline size_t bin_gather_lds_bytes(uint32_t BS, uint32_t csr_cap) {
  return 4 * (3 * ((size_t)1 << BS) + (size_t)csr_cap + 3 * 256 + 257 + 32);
}

// After the last level: the binned levels' records of the bin go to inbound slots after
// the direct levels' (cnt[pair] so far), rows written coalesced from an LDS CSR; cnt[pair]
// becomes the round's in-degree. Records are numbered f over the bin's level runs in
// level order; a thread takes f = tid + j * GATHER_THREADS and keeps its first G_CACHE
// records in registers for the placement pass.
// GATHER_THREADS: 512 (two workgroups per CU, bins of 2^11 pairs) or 1,024 (one per CU
// with 160 KB of LDS for bins of 2^12+: twice the waves to hide the pool loads' latency).
template <class R, uint32_t GATHER_THREADS>
__global__ __launch_bounds__(GATHER_THREADS) void k_bin_gather(BinArgs a) {
  using RT = typename R::T;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t b = xcd_bin(blockIdx.x, a.nbins);
  if (b >= a.nbins) return;
  const RT* pool = reinterpret_cast<const RT*>(a.pool) + (size_t)b * a.pool_bin_cap;  // this bin's region; Lt is relative
  const uint32_t tid = threadIdx.x, nb = a.nbins, BP = 1u << a.BS;
  uint32_t* cd = reinterpret_cast<uint32_t*>(smem);  // [BP] direct-level in-degree
  uint32_t* cb = cd + BP;                            // [BP] binned-level records
  uint32_t* of = cb + BP;                            // [BP] CSR cursor
  uint32_t* csr = of + BP;                           // [csr_cap]
  uint32_t* rs = csr + a.csr_cap;                    // [256] pool start of level d's run
  uint32_t* rp = rs + 256;                           // [257] records before level d's run
  uint32_t* ctl = rp + 257;                          // scan words
  const uint32_t q0 = b << a.BS;
  const uint32_t nq = (uint32_t)min((size_t)BP, a.PAIRS - q0);
  for (uint32_t i = tid; i < BP; i += GATHER_THREADS) {
    cd[i] = i < nq ? a.cnt[q0 + i] : 0u;
    cb[i] = 0;
  }
  uint32_t rn = 0;  // 1. run table: thread d < 255 reads level d's run
  if (tid < 255) {
    // Only levels an apply really ran: in the predicted loop a level the profile put below
    // qmin runs direct whatever its real size, and its Lt row is stale.
    if (a.lvl[256 + tid]) {
      const uint2 L = a.Lt[(size_t)tid * nb + b];
      rs[tid] = L.x;
      rn = L.y;
    }
  }
  {
    const uint32_t incl = wave_incl_scan(rn);
    if ((tid & 63) == 63) ctl[tid >> 6] = incl;
    __syncthreads();
    uint32_t off = incl - rn;
    for (uint32_t w = 0; w < (tid >> 6); ++w) off += ctl[w];
    if (tid < 256) rp[tid] = off;
    if (tid == 255) rp[256] = off + rn;
  }
  __syncthreads();
  const uint32_t Etot = rp[256];
  if (Etot == 0) return;  // no binned-level records: cnt[] already holds the in-degrees
  // 2. count per pair; cache records
  RT cache[G_CACHE];
  uint32_t lv = 0;
#pragma unroll
  for (uint32_t j = 0; j < G_CACHE; ++j) {
    const uint32_t f = tid + j * GATHER_THREADS;
    if (f < Etot) {
      while (f >= rp[lv + 1]) ++lv;
      cache[j] = pool[rs[lv] + (f - rp[lv])];
      atomicAdd(&cb[R::pool_ql(cache[j])], 1u);
    }
  }
  for (uint32_t f = tid + G_CACHE * GATHER_THREADS; f < Etot; f += GATHER_THREADS) {
    while (f >= rp[lv + 1]) ++lv;
    atomicAdd(&cb[R::pool_ql(pool[rs[lv] + (f - rp[lv])])], 1u);
  }
  __syncthreads();
  uint32_t kmax = 0;
  bool over = false;
  for (uint32_t i = tid; i < BP; i += GATHER_THREADS) {
    const uint32_t c = cb[i];
    of[i] = c;
    kmax = max(kmax, c);
    if (i < nq && c) {
      a.cnt[q0 + i] = cd[i] + c;
      over |= cd[i] + c > a.capin;
    }
  }
  if (over) atomicOr(a.err, ERR_INBOUND);
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
  if ((tid & 63) == 0) ctl[16 + (tid >> 6)] = kmax;
  __syncthreads();
  kmax = 0;
  for (uint32_t k = 0; k < GATHER_THREADS / 64; ++k) kmax = max(kmax, ctl[16 + k]);
  const uint32_t E = block_excl_scan(of, BP, ctl);  // of[i] = CSR start of pair i
  const bool in_lds = E <= a.csr_cap;
  if (!in_lds) {  // more records than the LDS CSR holds: cursors at the direct count, placed directly
    for (uint32_t i = tid; i < BP; i += GATHER_THREADS) of[i] = cd[i];
    __syncthreads();
  }
  // 3. placement (cached records first, then re-read ones)
  lv = 0;
#pragma unroll
  for (uint32_t j = 0; j < G_CACHE; ++j) {
    const uint32_t f = tid + j * GATHER_THREADS;
    if (f < Etot) {
      while (f >= rp[lv + 1]) ++lv;
      const uint32_t ql = R::pool_ql(cache[j]), v = R::pool_val(cache[j], (lv + 1) << 24);
      const uint32_t pos = atomicAdd(&of[ql], 1u);
      if (in_lds) csr[pos] = v;
      else if (pos < a.capin) a.inb[(size_t)pos * a.PAIRS + q0 + ql] = v;
    }
  }
  for (uint32_t f = tid + G_CACHE * GATHER_THREADS; f < Etot; f += GATHER_THREADS) {
    while (f >= rp[lv + 1]) ++lv;
    const RT rec = pool[rs[lv] + (f - rp[lv])];
    const uint32_t ql = R::pool_ql(rec), v = R::pool_val(rec, (lv + 1) << 24);
    const uint32_t pos = atomicAdd(&of[ql], 1u);
    if (in_lds) csr[pos] = v;
    else if (pos < a.capin) a.inb[(size_t)pos * a.PAIRS + q0 + ql] = v;
  }
  if (!in_lds) return;
  __syncthreads();  // of[i] is now the END of pair i's list
  // 4. rows k of the bin, coalesced over pairs; per-pair state hoisted out of the k loop.
  // A wave loops to ITS largest count; pairs with more than G_HEAVY records are written
  // afterwards by a whole wave each (lanes over k): power-law in-degrees (thousands at a
  // 10M-node top-stake node) made every wave loop to the bin's largest count (kmax).
  constexpr uint32_t PPT = 4;  // BP / GATHER_THREADS pairs per thread (BP <= 2048 here; more loop below)
  constexpr uint32_t G_HEAVY = 64;
  (void)kmax;
  uint32_t* hv = cb;  // the binned counts are dead once a step's c[] is loaded: the heavy list (i, n)
  if (tid == 0) ctl[40] = 0;
  for (uint32_t i0 = 0; i0 < nq; i0 += PPT * GATHER_THREADS) {
    uint32_t c[PPT], st[PPT], sl[PPT];
#pragma unroll
    for (uint32_t t = 0; t < PPT; ++t) {
      const uint32_t i = i0 + t * GATHER_THREADS + tid;
      c[t] = i < nq ? cb[i] : 0u;
      st[t] = i < nq ? of[i] - c[t] : 0u;
      sl[t] = i < nq ? cd[i] : 0u;
    }
    __syncthreads();  // every c[] of this step is loaded before the list overwrites cb
    const uint32_t hcap = min(BP, i0 + PPT * GATHER_THREADS);  // counts of later steps stay intact
    uint32_t cm = 0;
#pragma unroll
    for (uint32_t t = 0; t < PPT; ++t) {
      if (c[t] > G_HEAVY) {
        const uint32_t h = atomicAdd(&ctl[40], 1u);
        if (2 * h + 1 < hcap) {  // (a full list leaves the pair to the lane loop)
          hv[2 * h] = i0 + t * GATHER_THREADS + tid;
          hv[2 * h + 1] = c[t];
          c[t] = 0;
        }
      }
      cm = max(cm, c[t]);
    }
    for (int o = 32; o > 0; o >>= 1) cm = max(cm, (uint32_t)__shfl_xor((int)cm, o));
    for (uint32_t k = 0; k < cm; ++k)
#pragma unroll
      for (uint32_t t = 0; t < PPT; ++t) {
        const uint32_t i = i0 + t * GATHER_THREADS + tid;
        if (k < c[t] && sl[t] + k < a.capin) a.inb[(size_t)(sl[t] + k) * a.PAIRS + q0 + i] = csr[st[t] + k];
      }
    __syncthreads();
    const uint32_t nh = min(ctl[40], hcap / 2);
    for (uint32_t h = tid >> 6; h < nh; h += GATHER_THREADS / 64) {
      const uint32_t i = hv[2 * h], n = hv[2 * h + 1];
      const uint32_t s0 = of[i] - n, d0 = cd[i];
      for (uint32_t k = tid & 63; k < n; k += 64)
        if (d0 + k < a.capin) a.inb[(size_t)(d0 + k) * a.PAIRS + q0 + i] = csr[s0 + k];
    }
    __syncthreads();
    if (tid == 0) ctl[40] = 0;
    __syncthreads();
  }
}

__global__ void k_bin_seed(BinArgs a, const uint32_t* __restrict__ origin, uint32_t S, uint32_t* q0) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= S) return;
  const size_t p = (size_t)o * a.N + origin[o];
  a.hops[p] = 0;
  atomicOr(&a.visbm[p >> 5], 1u << (p & 31));
  q0[o] = (uint32_t)p;
  if (o == 0) a.lvl[0] = S;
}

}  // namespace gs

namespace gs {

// Own-bucket entry rows (the entry a node uses for every origin whose bucket is at
// least its own, push_active_set.rs:38-52): own[u] = peers[u][bucket[u]] and, in word
// ASZP, hl | bucket << 16; with fcls (the multi-source BFS) words ASZP + 1 .. hold the
// peers' failure classes, one byte each, so a row and its failure test are one line.
// Refreshed after init, rotation, entry uploads and failures.
template <int ASZP>
__global__ void k_own_rows(const uint8_t* __restrict__ bucket, const uint32_t* __restrict__ peers,
                           const uint16_t* __restrict__ hl, const uint32_t* __restrict__ list,
                           const uint32_t* __restrict__ count, uint32_t n_all, uint32_t ORW,
                           const uint8_t* __restrict__ fcls, uint32_t* __restrict__ own) {
  const uint32_t n = count ? *count : n_all;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    own_row<ASZP>(bucket, peers, hl, ORW, fcls, own, list ? list[i] : i);
}

hipError_t launch_own_rows(Engine& e, const uint32_t* list, const uint32_t* count) {
  if (!e.own) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<size_t>((e.N + 255) / 256, 2048);
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_own_rows<A>, dim3(grid), dim3(256), 0, e.st, e.bucket, e.peers,
                                              e.hl, list, count, e.N, e.ORW, e.mv_fcls, e.own));
  return hipGetLastError();
}

void bin_geometry(uint32_t N, size_t PAIRS, uint32_t fcap, BinGeom& g, bool allow_narrow) {
  uint32_t lg = 0;
  while ((1ull << lg) < PAIRS) ++lg;
  g.BS = std::min(13u, std::max(11u, lg > 13 ? lg - 13 : 0u));  // <= 8192 bins up to 2^26 pairs
  g.nbins = (uint32_t)((PAIRS + (1ull << g.BS) - 1) >> g.BS);
  g.narrow = allow_narrow && g.BS == NARROW_BS && N <= (1u << NARROW_SRC_BITS);
  const uint32_t rb = g.narrow ? 4 : 8;
  uint32_t pw = 2048;
  while (pw > 256 && (size_t)pw * fcap * rb > 48 * 1024) pw >>= 1;  // LDS-staged records <= 48 KiB
  g.PW = pw;
  g.Gmax = (uint32_t)((PAIRS + pw - 1) / pw);
  g.T_words = (size_t)g.Gmax * (g.nbins + 1);
  // two gather workgroups per CU (LDS <= 80 KiB) for bins of 2^11 pairs, one beyond
  const size_t budget = g.BS <= 11 ? 80 * 1024 : 160 * 1024;
  g.csr_cap = (uint32_t)((budget - 4 * (3 * ((size_t)1 << g.BS) + 3 * 256 + 257 + 32)) / 4);
}

bool bin_supported(const BinGeom& g, uint32_t fcap) {
  return g.T_words * 4 <= (1ull << 30) && bin_expand_lds_bytes(g.nbins, g.PW, fcap, g.narrow ? 4 : 8) <= 160 * 1024;
}

template <class R>
static hipError_t run_binned(Engine& e, BinArgs& a) {
  hipError_t r;
  const size_t lds_x = bin_expand_lds_bytes(a.nbins, a.PW, a.fc, sizeof(typename R::T));
  const size_t lds_a = bin_apply_lds_bytes(a.BS);
  const size_t lds_g = bin_gather_lds_bytes(a.BS, a.csr_cap);
  const uint32_t xth = a.PW / X_PPT;
  const uint32_t xgrid = std::min<uint32_t>(a.Gmax, 256 * (xth <= 256 ? 2 : 1));  // slices looped
  const uint32_t bgrid = ((a.nbins + 7) / 8) * 8;
  if ((r = hipFuncSetAttribute((const void*)k_bin_apply<R>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a)))
    return r;
  // wide records: super-bin apply (one workgroup per 16 bins)
  constexpr bool SBA = std::is_same<R, RecW>::value;
  const size_t lds_sb = bin_apply_sb_lds_bytes(a.BS);
  const uint32_t sbgrid = ((((a.nbins + SB_N - 1) >> SB_LOG) + 7) / 8) * 8;
  if (SBA && (r = hipFuncSetAttribute((const void*)k_bin_apply_sb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_sb)))
    return r;
  if ((r = hipFuncSetAttribute((const void*)k_bin_gather<R, GATHER_THREADS_S>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g)))
    return r;
  if ((r = hipFuncSetAttribute((const void*)k_bin_gather<R, GATHER_THREADS_L>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g)))
    return r;
  GS_ASZP_DISPATCH(e.ASZP, {
    r = hipFuncSetAttribute((const void*)k_bin_expand<A, R>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_x);
  });
  if (r != hipSuccess) return r;
  // Levels of at most `lim` frontier pairs run in one workgroup (k_bin_small); larger ones
  // as expand (+ apply when binned). Two forms, as in the multi-source BFS: predicted
  // (a level profile from an earlier round: the head kernel, one expand (+ apply) per
  // level the profile had above the tail threshold, the tail kernel -- all enqueued at
  // once, the host never waits) or polled (the host enqueues level d after seeing level
  // d - lag's size, host-mapped, written by expand).
  volatile uint32_t* hl = e.mv_hlvl;
  volatile uint32_t* hs = e.mv_hlvl + 256;
  uint32_t small = BIN_SMALL;
  if (const char* x = std::getenv("GS_BIN_SMALL")) small = (uint32_t)std::strtoul(x, nullptr, 10);
  if (e.prm.flags & GS_FLAG_NO_SMALL_LEVELS) small = 0;
  const uint32_t lim = std::min(small, a.qmin - 1), lag = 2;
  static const bool polled_only = std::getenv("GS_MV_POLLED") && std::getenv("GS_MV_POLLED")[0] == '1';
  static const uint32_t tail_thr = [] {
    const char* x = std::getenv("GS_BIN_TAIL");
    return x ? (uint32_t)std::strtoul(x, nullptr, 10) : 2048u;
  }();
  {  // the newest published profile (a tail kernel of an earlier round)
    volatile uint32_t* vp = e.mv_prof;
    const uint32_t sq = vp[0];
    if (sq != 0 && sq != e.mv_prof_seen[0]) {
      std::atomic_thread_fence(std::memory_order_acquire);
      const uint32_t nl = std::min<uint32_t>((uint32_t)vp[1], 255u);
      std::vector<uint32_t> pv(nl);
      for (uint32_t k = 0; k < nl; ++k) pv[k] = vp[2 + k];
      std::atomic_thread_fence(std::memory_order_acquire);
      if (vp[0] == sq) {  // (a rewrite sets 0 first, then a new seq)
        e.mv_pred[0] = std::move(pv);
        e.mv_prof_seen[0] = sq;
      }
    }
  }
  const std::vector<uint32_t>& pv = e.mv_pred[0];
  const bool predicted = !pv.empty() && !polled_only && lim > 0;
  if (predicted) {
    uint32_t k0 = 0;
    while (k0 < pv.size() && pv[k0] <= lim) ++k0;
    uint32_t k1 = (uint32_t)pv.size();  // one past the last level above the tail threshold
    while (k1 > k0 && pv[k1 - 1] <= std::min(tail_thr, lim)) --k1;
    const uint32_t npairs = std::min<uint32_t>(k1 - k0 + mv_margin(), 250);
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_bin_small<A>), dim3(1), dim3(BIN_ST), 0, e.st, a, BIN_HEAD, 0u, 0u,
                                                lim, e.q[0], e.q[1], e.mv_hstate_dev, 0u));
    // GS_FLAG_MISPREDICT_LEVELS (tests): every other round inverts the predicted binned /
    // direct choice of each pair, so real levels of >= qmin pairs run direct while the
    // Lt rows of the round before are still there
    const uint32_t flip = (e.prm.flags & GS_FLAG_MISPREDICT_LEVELS) ? (e.mv_seq & 1u) : 0u;
    for (uint32_t i = 0; i < npairs; ++i) {
      const uint32_t binned = (k0 + i < pv.size() && pv[k0 + i] >= a.qmin ? 1u : 0u) ^ flip;  // predicted binned level
      GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_bin_expand<A, R>), dim3(xgrid), dim3(xth), lds_x, e.st, a, 0u, i,
                                                  binned, e.q[0], e.q[1]));
      if (binned) {
        if (SBA) hipLaunchKernelGGL(k_bin_apply_sb, dim3(sbgrid), dim3(APPLY_THREADS), lds_sb, e.st, a, 0u, i, e.q[0], e.q[1]);
        else hipLaunchKernelGGL(k_bin_apply<R>, dim3(bgrid), dim3(APPLY_THREADS), lds_a, e.st, a, 0u, i, e.q[0], e.q[1]);
      }
    }
    const uint32_t seq = ++e.mv_seq ? e.mv_seq : ++e.mv_seq;
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_bin_small<A>), dim3(1), dim3(BIN_ST), 0, e.st, a, BIN_TAIL, 0u, npairs,
                                                lim, e.q[0], e.q[1], e.mv_hstate_dev, seq));
  } else {
    uint32_t d = 0, nlev = 0;
    for (;;) {
      hs[0] = MV_PENDING;
      GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_bin_small<A>), dim3(1), dim3(BIN_ST), 0, e.st, a, BIN_POLL, d, 0u,
                                                  lim, e.q[0], e.q[1], e.mv_hstate_dev, 0u));
      e.bfs_level = d;
      if ((r = mv_wait(hs, e.st, d))) return r;
      if (hs[1] == 0) { nlev = d; break; }
      const uint32_t dl = d;
      bool done = false;
      for (;; ++d) {
        if (d >= 254) {  // levels through 253 enqueued: the hops fit u8 iff level 254 is empty
          bool empty = false;
          if ((r = level_empty(e, 254, empty))) return r;
          if (!empty) return hipErrorNotSupported;
          nlev = d;
          done = true;
          break;
        }
        hl[d] = MV_PENDING;
        GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_bin_expand<A, R>), dim3(xgrid), dim3(xth), lds_x, e.st, a, d,
                                                    BIN_NOPAIR, 1u, e.q[0], e.q[1]));
        if (SBA) hipLaunchKernelGGL(k_bin_apply_sb, dim3(sbgrid), dim3(APPLY_THREADS), lds_sb, e.st, a, d, BIN_NOPAIR, e.q[0], e.q[1]);
        else hipLaunchKernelGGL(k_bin_apply<R>, dim3(bgrid), dim3(APPLY_THREADS), lds_a, e.st, a, d, BIN_NOPAIR, e.q[0], e.q[1]);
        if (d >= dl + lag) {
          uint32_t x = 0;
          e.bfs_level = d - lag;
          if ((r = mv_wait(hl + (d - lag), e.st, x))) return r;
          if (x == 0) { nlev = d + 1; done = true; break; }
          if (x <= lim) { ++d; break; }  // levels through d are enqueued; small levels from d + 1
        }
      }
      if (done) break;
    }
    if (!polled_only && lim > 0) {  // this round's sizes seed the prediction
      std::vector<uint32_t> p2(nlev);  // (levels past the BFS's end may still read PENDING: 0)
      for (uint32_t k = 0; k < nlev; ++k) p2[k] = hl[k] == MV_PENDING ? 0u : hl[k];
      while (!p2.empty() && p2.back() == 0) p2.pop_back();
      e.mv_pred[0] = std::move(p2);
    }
  }
  if (a.BS <= 11) hipLaunchKernelGGL((k_bin_gather<R, GATHER_THREADS_S>), dim3(bgrid), dim3(GATHER_THREADS_S), lds_g, e.st, a);
  else hipLaunchKernelGGL((k_bin_gather<R, GATHER_THREADS_L>), dim3(bgrid), dim3(GATHER_THREADS_L), lds_g, e.st, a);
  return hipGetLastError();
}

hipError_t launch_bfs_binned(Engine& e, bool record) {
  BinArgs a;
  a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.own = e.own; a.frank = e.frank; a.origin = e.origin;
  a.obkt = e.obkt; a.nfail = e.nfail; a.mask = e.mask; a.hops = e.hops; a.cnt = e.cnt; a.inb = e.inb;
  a.egress = e.egress; a.egress_acc = e.egress_acc; a.lvl = e.lvl; a.err = e.err; a.area = e.bin_area;
  a.T = e.bin_T; a.pool = e.bin_pool; a.Lt = e.bin_Lt; a.binoff = e.bin_binoff;
  a.visbm = e.bin_vis; a.hlvl = e.mv_hlvl_dev; a.dpair = e.mv_dpair; a.hprof = e.mv_prof_dev;
  a.N = e.N; a.ASZ = e.ASZ; a.fanout = e.fanout; a.fc = e.fcap; a.capin = e.capin; a.Gmax = e.bin.Gmax;
  a.PW = e.bin.PW; a.BS = e.bin.BS; a.nbins = e.bin.nbins; a.ORW = e.ORW; a.csr_cap = e.bin.csr_cap;
  a.qmin = (e.prm.flags & GS_FLAG_BINNED_ALL_LEVELS) ? 1u : BIN_MIN_FRONTIER;
  if (e.prm.flags & GS_FLAG_NARROW_WAVE_PATH) a.csr_cap = 256;  // small tests reach the gather's direct placement
  a.PAIRS = e.PAIRS; a.pool_bin_cap = ((size_t)1 << e.bin.BS) * e.capin; a.record = record ? 1 : 0;
  hipError_t r;
  if ((r = hipMemsetAsync(e.hops, 0xFF, e.PAIRS, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.lvl, 0, 512 * 4, e.st)) != hipSuccess) return r;  // sizes and binned flags
  if ((r = hipMemsetAsync(e.cnt, 0, e.PAIRS * 4, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.bin_binoff, 0, (size_t)e.bin.nbins * 4, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.bin_vis, 0, (e.PAIRS + 31) / 32 * 4, e.st)) != hipSuccess) return r;
  hipLaunchKernelGGL(k_bin_seed, dim3((e.S + 255) / 256), dim3(256), 0, e.st, a, e.origin, e.S, e.q[0]);
  return e.bin.narrow ? run_binned<RecN>(e, a) : run_binned<RecW>(e, a);
}

}  // namespace gs
