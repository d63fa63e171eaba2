// gs_bfs_hybrid.hip -- Cluster::run_gossip (gossip.rs:494-615) for large clusters as a
// direction-optimizing multi-source BFS over the round's push graph (GS_BFS_HYBRID).
//
// A node's pushes in a round depend only on its active-set row, its prune masks and the
// failed set (PushActiveSet::get_nodes(..).take(fanout), failed peers burning their slot:
// gossip.rs:527-541), never on when the BFS reaches it; an inbound record's hop is the
// pusher's distance + 1 (gossip.rs:594-607). So one slot group's round is:
//
//   1. the push graph, built once per round: k_hb_graph expands EVERY node for every slot
//      of the group (mv_expand_entry; the egress bytes of every (node, slot) are written
//      here, read only where the node was reached) and bins the pushes by coarse
//      destination bin in LDS (one contiguous run and one T row per slice of XT nodes);
//      k_hb_csr turns each coarse bin's runs into in-records (src | slot mask << 32)
//      grouped by destination node, pgo[v] = {first, count}. k_hb_graph also initialises
//      the round's visited masks (the slots in which the node failed count as visited) and
//      distances (0xFF);
//   2. the levels, carrying slot masks and distances only -- no push record is written:
//      - top-down (small frontiers: k_hb_small in one workgroup, k_hb_td over the chip): a
//        frontier entry (node, entry k, slot mask) re-expands its row; an atomicOr on the
//        pushed-to node's visited mask returns the slots it reaches first (hop d + 1,
//        gossip.rs:594-600), which become its distance bytes and next-level entries;
//      - bottom-up (large frontiers: k_hb_bu): every node still missing slots scans its
//        in-records for pushers that first reached those slots at level d (F_d, one u32
//        slot mask per node: 4 MB at 1M nodes, L2-resident where the 16-byte distance rows
//        are not) -- such a pusher pushed to it at level d; the pushers are the same in
//        either direction, so the distances are the BFS's in both.
//      Every level kernel records its first arrivals in F_{d+1} (buffer (d + 1) % 3) and
//      clears F_{d-1}, so buffer (d + 2) % 3 is zero when level d + 1 starts;
//   3. the gather (k_hb_gather): per (slot, node) the in-records whose pusher was reached in
//      that slot, keyed hop << 24 | src with hop = the pusher's distance + 1, as the inbound
//      rows k_cg_consume consumes; the in-degree; the hop = the node's distance.
//
// Results equal k_bfs_level's: hops, in-degrees, inbound record sets, egress.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>

#include "gs_device.h"
#include "gs_internal.h"
#include "gs_mv_dev.h"

namespace gs {

namespace {

constexpr uint32_t HB_CT = 1024;   // k_hb_csr threads (one workgroup per coarse bin)
constexpr uint32_t HB_LT = 256;    // level kernels (k_hb_td, k_hb_bu) and gather threads
constexpr uint32_t HB_ST = 1024;   // k_hb_small threads
constexpr uint32_t HB_SQ = 2048;   // frontier entries of a level kept in k_hb_small's LDS queue
constexpr uint32_t HB_SMALL = 1024;  // a head level has at most this many entries (GS_HB_SMALL)
constexpr uint32_t HB_GH = 64;     // gather / bottom-up: nodes with more in-records take the wave path
enum : uint32_t { HB_HEAD = 0, HB_TAIL = 1, HB_POLL = 2 };

__device__ inline uint32_t* hb_F(const MvArgs& a, uint32_t d) { return a.F + (size_t)(d % 3) * a.N; }

// Distance bytes j in `bits` of node v := d + 1 (one byte store per slot: other slots' bytes
// of the same row may be written by other threads at this level).
__device__ inline void hb_set_dist(uint8_t* dist, uint32_t DSP, uint32_t v, uint32_t bits, uint32_t d1) {
  uint8_t* row = dist + (size_t)v * DSP;
  while (bits) {
    const uint32_t j = (uint32_t)__builtin_ctz(bits);
    bits &= bits - 1u;
    row[j] = (uint8_t)d1;
  }
}

// The slots of the group in which node u failed (fcls[u] <= the slot's failure class): they
// count as visited, so no level looks for a pusher of u in them.
__device__ inline uint32_t hb_failed_slots(const MvArgs& a, const MvSlots& S, uint32_t u) {
  if (!a.any_fail) return 0u;
  const uint32_t fc = a.fcls[u];
  uint32_t m = 0;
  for (uint32_t j = 0; j < a.Sg; ++j) m |= (uint32_t)(S.sfk[j] != 0 && fc <= S.sfk[j]) << j;
  return m;
}

// Part `it` of node u's entries for the slot mask M (mv_parts_to's order): false if none.
__device__ inline bool hb_part(const uint32_t* gt, uint32_t u, uint32_t M, uint32_t bu, uint32_t it, uint2& ent) {
  bool found = false;
  mv_parts_to(gt, u, M, bu, [&](uint32_t k, uint2 x) {
    if (k == it) {
      ent = x;
      found = true;
    }
  });
  return found;
}

// ------------------------------------------------------------ push graph ----
// Slice w = nodes [w * XT, (w + 1) * XT), part it (T row w * pg_parts + it): every node's
// part-it entry (node, k, all the group's slots that push from entry k) expanded as a
// frontier entry would be at any level; the pushes become area records src | node-in-bin
// << UB | slot mask << (UB + BSC), binned by coarse destination bin (a run per row at the
// fixed place row * XT * ASZ: an entry pushes to at most ASZ distinct peers).
template <int ASZP, uint32_t XT>
__global__ __launch_bounds__(XT) void k_hb_graph(MvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ MvSlots S;
  __shared__ uint32_t gt[GT_WORDS];
  const uint32_t tid = threadIdx.x, nb = a.nbc, BSC = a.BSC, UB = a.UB, BPm = (1u << BSC) - 1;
  const uint32_t gm = a.Sg >= 32 ? 0xFFFFFFFFu : (1u << a.Sg) - 1u;
  mv_slots_load(a, S, tid, XT);
  for (uint32_t i = tid; i < GT_WORDS; i += XT) gt[i] = a.gt[i];
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);  // [nb] + scan words
  unsigned long long* stage = reinterpret_cast<unsigned long long*>(smem + mv_hist_bytes(nb));  // [XT * ASZP]
  __syncthreads();
  for (uint32_t w = blockIdx.x; w < a.pg_slices; w += gridDim.x) {
    const uint32_t u0 = w * XT + tid;
    const bool valid = u0 < a.N;
    uint32_t bu = 0;
    if (valid) {  // the round's visited masks (failed slots preset) and distances
      bu = a.bucket[u0];
      a.vis[u0] = hb_failed_slots(a, S, u0);
      a.F[u0] = 0;
      a.F[(size_t)a.N + u0] = 0;
      a.F[2 * (size_t)a.N + u0] = 0;
      uint4* dr = reinterpret_cast<uint4*>(a.dist + (size_t)u0 * a.DSP);
      dr[0] = make_uint4(~0u, ~0u, ~0u, ~0u);
      if (a.DSP > 16) dr[1] = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    for (uint32_t it = 0; it < a.pg_parts; ++it) {
      for (uint32_t i = tid; i < nb; i += XT) hist[i] = 0;
      __syncthreads();
      uint32_t row[ASZP], acc[ASZP], u = 0;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) { row[s] = 0; acc[s] = 0; }
      uint2 ent;
      if (valid && hb_part(gt, u0, gm, bu, it, ent)) mv_expand_entry<ASZP, true>(a, ent, S, row, acc, u);
      uint32_t rk[ASZP];
#pragma unroll
      for (int s = 0; s < ASZP; ++s) rk[s] = acc[s] ? atomicAdd(&hist[row[s] >> BSC], 1u) : 0u;
      __syncthreads();
      const uint32_t total = mv_block_scan(hist, nb, hist + nb);
      const size_t rw = (size_t)w * a.pg_parts + it;
      const size_t b64 = rw * XT * a.ASZ;
      const bool ok = b64 + total <= a.area_cap;
      if (!ok && tid == 0) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_AREA);
      for (uint32_t b = tid; b < nb; b += XT) mv_t(a, (uint32_t)rw, 1 + b) = ok ? hist[b] : 0u;
      if (tid == 0) {
        mv_t(a, (uint32_t)rw, 0) = ok ? (uint32_t)b64 : 0u;
        mv_t(a, (uint32_t)rw, 1 + nb) = ok ? total : 0u;
      }
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if (acc[s]) {
          const uint32_t wp = row[s];
          stage[hist[wp >> BSC] + rk[s]] = (unsigned long long)u | ((unsigned long long)(wp & BPm) << UB) |
                                           ((unsigned long long)acc[s] << (UB + BSC));
        }
      __syncthreads();
      if (ok)
        for (uint32_t r = tid; r < total; r += XT) a.area[b64 + r] = stage[r];
      __syncthreads();
    }
  }
}

__host__ __device__ inline size_t hb_csr_lds_bytes(uint32_t BSC) {
  return 4 * (2 * (size_t)MV_SEG + 1 + 2 * (((size_t)1 << BSC) + 1) + 64);
}

constexpr uint32_t HB_RC = 4;  // k_hb_csr: trips of 4 records per thread kept in registers between the passes

// One coarse bin c (2^BSC destination nodes): its segment of every push-graph row (the T
// column), counted per destination, then placed as in-records src | slot mask << 32 at
// pgr[c * pg_bin_cap + ...], grouped by destination (pgo[v] = {first, count}). The first
// HB_RC trips' records stay in registers between the count and the placement.
__global__ __launch_bounds__(HB_CT) void k_hb_csr(MvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t c = mv_xcd_bin(blockIdx.x, a.nbc);
  if (c >= a.nbc) return;
  const uint32_t tid = threadIdx.x, BSC = a.BSC, UB = a.UB, BP = 1u << BSC, BPm = BP - 1;
  const uint32_t v0 = c << BSC, nv = min(BP, a.N - v0);
  const uint32_t R = a.pg_slices * a.pg_parts;
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem);  // [MV_SEG + 1]
  uint32_t* sb = pre + MV_SEG + 1;                    // [MV_SEG]
  uint32_t* cn = sb + MV_SEG;                         // [BP + 1] records per node -> firsts
  uint32_t* cur = cn + BP + 1;                        // [BP + 1] placement cursors
  uint32_t* ctl = cur + BP + 1;                       // [64]
  for (uint32_t i = tid; i <= BP; i += HB_CT) cn[i] = 0;
  const unsigned long long um = (1ull << UB) - 1;
  const size_t base = (size_t)c * a.pg_bin_cap;
  unsigned long long rc[HB_RC][4];  // (the first segment chunk's first trips)
  // pass 0 counts, pass 1 places
  for (uint32_t pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      __syncthreads();
      const uint32_t tot = mv_block_scan(cn, nv, ctl);
      if (tid == 0) {
        cn[nv] = tot;
        ctl[32] = tot <= a.pg_bin_cap ? 1u : 0u;
        if (tot > a.pg_bin_cap) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_AREA);
      }
      __syncthreads();
      if (!ctl[32]) {
        for (uint32_t i = tid; i < nv; i += HB_CT) a.pgo[v0 + i] = make_uint2((uint32_t)base, 0u);
        return;
      }
      for (uint32_t i = tid; i < nv; i += HB_CT) {
        cur[i] = cn[i];
        a.pgo[v0 + i] = make_uint2((uint32_t)(base + cn[i]), cn[i + 1] - cn[i]);
      }
      __syncthreads();
    }
    for (uint32_t c0 = 0; c0 < R; c0 += MV_SEG) {
      const uint32_t gc = min(MV_SEG, R - c0);
      for (uint32_t i = tid; i < gc; i += HB_CT) {
        const uint32_t st = mv_t(a, c0 + i, 1 + c);
        pre[i] = mv_t(a, c0 + i, 2 + c) - st;
        sb[i] = mv_t(a, c0 + i, 0) + st;
      }
      __syncthreads();
      const uint32_t ct = mv_block_scan(pre, gc, ctl);
      if (tid == 0) pre[gc] = ct;
      __syncthreads();
      uint32_t trip = 0;
      for (uint32_t r0 = 0; r0 < ct; r0 += HB_CT * 4, ++trip) {
        const bool cached = c0 == 0 && trip < HB_RC;
        unsigned long long rec[4];
        if (pass == 1 && cached) {
#pragma unroll
          for (uint32_t t = 0; t < HB_RC; ++t)
            if (t == trip) {
#pragma unroll
              for (uint32_t k = 0; k < 4; ++k) rec[k] = rc[t][k];
            }
        } else {
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) {  // four records' searches and loads in flight
            const uint32_t r = r0 + k * HB_CT + tid;
            uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
            while (hi - lo > 1) {
              const uint32_t mid = (lo + hi) >> 1;
              if (pre[mid] <= r) lo = mid; else hi = mid;
            }
            rec[k] = r < ct ? a.area[sb[lo] + (r - pre[lo])] : ~0ull;
          }
          if (pass == 0 && cached) {
#pragma unroll
            for (uint32_t t = 0; t < HB_RC; ++t)
              if (t == trip) {
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) rc[t][k] = rec[k];
              }
          }
        }
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
          if (r0 + k * HB_CT + tid >= ct) continue;
          uint32_t vl = (uint32_t)(rec[k] >> UB) & BPm;
          if (GS_OOB(vl, nv, a.err, "push-graph record node")) vl = 0;
          if (pass == 0) {
            atomicAdd(&cn[vl], 1u);
          } else {
            const uint32_t p = atomicAdd(&cur[vl], 1u);
            a.pgr[base + p] = (rec[k] & um) | ((rec[k] >> (UB + BSC)) << 32);
          }
        }
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------------------- top-down ----
// One frontier entry at level d: its pushes (mv_expand_entry, egress already written by the
// push graph); per pushed-to peer the atomicOr on its visited mask returns the slots it
// reaches first, whose distance bytes become d + 1 and whose bits go to F_{d+1}. Returns
// the next-level entries.
template <int ASZP, bool WG>
__device__ inline uint32_t hb_td_entry(const MvArgs& a, uint2 ent, const MvSlots& S, const uint32_t* gt, uint32_t d,
                                       uint32_t (&row)[ASZP], uint32_t (&nwm)[ASZP], uint32_t (&bw)[ASZP]) {
  uint32_t acc[ASZP], u = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) { row[s] = 0; acc[s] = 0; }
  mv_expand_entry<ASZP, false>(a, ent, S, row, acc, u);
  uint32_t old[ASZP];
#pragma unroll
  for (int s = 0; s < ASZP; ++s)
    old[s] = acc[s] ? (WG ? atomic_or_wg(&a.vis[row[s]], acc[s]) : atomicOr(&a.vis[row[s]], acc[s])) : 0xFFFFFFFFu;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) bw[s] = acc[s] ? (uint32_t)a.bucket[row[s]] : 0u;
  uint32_t* Fn = hb_F(a, d + 1);
  uint32_t n = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    nwm[s] = acc[s] & ~old[s];
    if (nwm[s]) {
      hb_set_dist(a.dist, a.DSP, row[s], nwm[s], d + 1);
      if (WG) atomic_or_wg(&Fn[row[s]], nwm[s]);
      else atomicOr(&Fn[row[s]], nwm[s]);
      n += mv_parts(gt, row[s], nwm[s], bw[s], nullptr, 0);
    }
  }
  return n;
}

// Levels inside ONE workgroup while they are small (LDS queue, LDS-only barriers), as
// k_mv_small: HB_HEAD seeds the group (level sizes, the origins' visited bits, distances
// and F_0) and runs while a level has at most a.small entries (where it stopped:
// dpair[0]); HB_TAIL runs from dpair[pi] to the end whatever the sizes and publishes the
// round's level profile (seqlock) for the host's next prediction; HB_POLL runs from d0
// while small. Every mode reports (level, entries) where it stopped in hstate. Entries are
// written to the global queue too (the level kernels and F's clearing read them there), and
// each level first clears F_{d-1} at its entries (level d - 1's first arrivals).
template <int ASZP>
__global__ __launch_bounds__(HB_ST) void k_hb_small(MvArgs a, uint32_t mode, uint32_t d0, uint32_t pi,
                                                    uint2* __restrict__ q0, uint2* __restrict__ q1,
                                                    uint32_t* __restrict__ hstate, const uint2* __restrict__ seeds,
                                                    uint32_t nseed, uint32_t seq) {
  __shared__ uint2 qL[2][HB_SQ];
  __shared__ MvSlots S;
  __shared__ uint32_t gt[GT_WORDS], cnt_s;
  const uint32_t tid = threadIdx.x;
  mv_slots_load(a, S, tid, HB_ST);
  for (uint32_t i = tid; i < GT_WORDS; i += HB_ST) gt[i] = a.gt[i];
  uint32_t d = mode == HB_TAIL ? a.dpair[pi] : d0;
  bool inL = false;     // level d's entries [0, HB_SQ) are in qL[d & 1]
  bool prevL = false;   // level d - 1's entries [0, HB_SQ) are in qL[(d - 1) & 1]
  if (mode == HB_HEAD) {
    for (uint32_t i = tid; i < 256; i += HB_ST) a.lvl[i] = i == 0 ? nseed : 0u;
    if (tid < nseed) {
      const uint2 sd = seeds[tid];  // distinct origins
      const uint32_t o = sd.x & 0xFFFFFFu;
      qL[0][tid] = sd;
      q0[tid] = sd;
      a.vis[o] |= sd.y;  // (k_hb_graph preset the failed slots)
      a.F[o] = sd.y;     // F_0
      uint32_t b = sd.y;
      while (b) {
        const uint32_t j = (uint32_t)__builtin_ctz(b);
        b &= b - 1u;
        a.dist[(size_t)o * a.DSP + j] = 0;
      }
    }
    inL = true;
  }
  __syncthreads();  // (full: the seeds' stores land before any atomic)
  uint32_t qn = mode == HB_HEAD ? nseed : (d < 256 ? a.lvl[d] : 0u);
  const uint32_t lim = mode == HB_TAIL ? 0xFFFFFFFFu : a.small;
  while (qn > 0 && qn <= lim && d < 254) {
    const uint2* qg = (d & 1) ? q1 : q0;
    uint2* qgn = (d & 1) ? q0 : q1;
    const uint2* ql = qL[d & 1];
    uint2* qln = qL[(d + 1) & 1];
    if (d >= 1) {  // F_{d-1} := 0 at level d - 1's entries (qgn / qln still hold them)
      uint32_t* Fp = hb_F(a, d + 2);
      const uint32_t pn = min(a.lvl[d - 1], (uint32_t)a.q_cap);
      for (uint32_t i = tid; i < pn; i += HB_ST) Fp[(prevL && i < HB_SQ ? qln[i].x : qgn[i].x) & 0xFFFFFFu] = 0;
    }
    if (tid == 0) cnt_s = 0;
    __syncthreads();  // (full: the clears and the previous level's global stores before this level's)
    for (uint32_t i0 = 0; i0 < qn; i0 += HB_ST) {
      const uint32_t i = i0 + tid;
      uint32_t row[ASZP], nwm[ASZP], bw[ASZP];
#pragma unroll
      for (int s = 0; s < ASZP; ++s) { row[s] = 0; nwm[s] = 0; bw[s] = 0; }
      uint32_t n = 0;
      if (i < qn) n = hb_td_entry<ASZP, true>(a, inL && i < HB_SQ ? ql[i] : qg[i], S, gt, d, row, nwm, bw);
      if (n) {
        const uint32_t base = atomicAdd(&cnt_s, n);
        if ((size_t)base + n <= a.q_cap) {
          uint32_t k0 = 0;
#pragma unroll
          for (int s = 0; s < ASZP; ++s)
            if (nwm[s])
              k0 += mv_parts_to(gt, row[s], nwm[s], bw[s], [&](uint32_t k, uint2 x) {
                const uint32_t p = base + k0 + k;
                if (p < HB_SQ) qln[p] = x;
                qgn[p] = x;
              });
        } else {
          atomicOr(a.err, ERR_MV_CAP | ERR_MVD_Q);
        }
      }
    }
    lds_barrier();
    qn = min(cnt_s, (uint32_t)a.q_cap);
    ++d;
    if (tid == 0) a.lvl[d] = qn;
    prevL = inL;
    inL = true;
    lds_barrier();
  }
  if (mode == HB_TAIL && qn > 0 && tid == 0) atomicOr(a.err, ERR_DEPTH);  // level 254 not empty
  if (tid == 0) {
    if (mode == HB_HEAD) a.dpair[0] = d;
    if (mode == HB_TAIL) {  // the round's level profile for the host's next prediction (seqlock)
      uint32_t* hp = a.hprof;
      const uint32_t nl = min(d, 255u);
      __hip_atomic_store(&hp[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __atomic_thread_fence(__ATOMIC_RELEASE);
      for (uint32_t k = 0; k < nl; ++k) __hip_atomic_store(&hp[2 + k], a.lvl[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&hp[1], nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&hp[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&hstate[1], qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hstate[0], d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // the host polls this word
  }
}

// The level of launch pi (the predicted loop: dpair[pi], a no-op once the BFS ended), or d.
// A live level clears F_{d-1} over the whole grid (nothing reads it at level d).
__device__ inline uint32_t hb_level(const MvArgs& a, uint32_t d, uint32_t pi, uint32_t& qn) {
  if (pi != MV_NOPAIR) d = a.dpair[pi];
  qn = d < 254 ? a.lvl[d] : 0u;
  if (pi != MV_NOPAIR && blockIdx.x == 0 && threadIdx.x == 0) a.dpair[pi + 1] = qn ? d + 1 : d;
  if (qn) {
    uint4* Fp = reinterpret_cast<uint4*>(hb_F(a, d + 2));  // (N is a multiple of 4 or the tail is cleared below)
    const uint32_t n4 = a.N / 4;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
      Fp[i] = make_uint4(0, 0, 0, 0);
    if (blockIdx.x == 0 && threadIdx.x < (a.N & 3)) hb_F(a, d + 2)[4 * n4 + threadIdx.x] = 0;
  }
  return d;
}

// Next-level entries of a wave: lane counts n, one reservation per wave on lvl[d + 1].
__device__ inline uint32_t hb_wave_reserve(const MvArgs& a, uint32_t d, uint32_t n, bool& ok) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t incl = wave_incl_scan(n);
  const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
  uint32_t wb = 0;
  if (lane == 63 && tot) wb = atomicAdd(&a.lvl[d + 1], tot);
  const uint32_t pos = (uint32_t)__shfl((int)wb, 63) + incl - n;
  ok = (size_t)pos + n <= a.q_cap;
  if (!ok && n) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_Q);
  return pos;
}

// A top-down level over the chip: 64-entry chunks dealt over every wave.
template <int ASZP>
__global__ __launch_bounds__(HB_LT) void k_hb_td(MvArgs a, uint32_t d, uint32_t pi, uint2* __restrict__ q0,
                                                 uint2* __restrict__ q1) {
  __shared__ MvSlots S;
  __shared__ uint32_t gt[GT_WORDS];
  uint32_t qn;
  d = hb_level(a, d, pi, qn);
  if (qn == 0) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t nwv = gridDim.x * (HB_LT / 64), gw = blockIdx.x * (HB_LT / 64) + (tid >> 6);
  if ((size_t)blockIdx.x * HB_LT >= qn) return;  // (workgroups beyond the level leave before any setup)
  mv_slots_load(a, S, tid, HB_LT);
  for (uint32_t i = tid; i < GT_WORDS; i += HB_LT) gt[i] = a.gt[i];
  __syncthreads();
  const uint2* qc = (d & 1) ? q1 : q0;
  uint2* qx = (d & 1) ? q0 : q1;
  for (uint32_t i0 = gw * 64; i0 < qn; i0 += nwv * 64) {  // (uniform per wave)
    const uint32_t i = i0 + lane;
    uint32_t row[ASZP], nwm[ASZP], bw[ASZP];
#pragma unroll
    for (int s = 0; s < ASZP; ++s) { row[s] = 0; nwm[s] = 0; bw[s] = 0; }
    uint32_t n = 0;
    if (i < qn) n = hb_td_entry<ASZP, false>(a, qc[i], S, gt, d, row, nwm, bw);
    bool ok;
    uint32_t pos = hb_wave_reserve(a, d, n, ok);
    if (ok && n) {
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if (nwm[s]) pos += mv_parts_to(gt, row[s], nwm[s], bw[s], [&](uint32_t k, uint2 x) { qx[pos + k] = x; });
    }
  }
}

// ------------------------------------------------------------ bottom-up ----
constexpr uint32_t HB_BR = 8;  // in-records per batch of the bottom-up scan (loads in flight per lane)

// A bottom-up level: every node v still missing slots (need = the group's slots not yet
// visited at v) scans its in-records, HB_BR at a time, for pushers whose F_d holds those
// slots; the slots found are v's first arrivals at hop d + 1. v's words are written by its
// thread only. Nodes with more than a.gh in-records are scanned by their whole wave, 64
// records per step.
__global__ __launch_bounds__(HB_LT) void k_hb_bu(MvArgs a, uint32_t d, uint32_t pi, uint2* __restrict__ q0,
                                                 uint2* __restrict__ q1) {
  __shared__ uint32_t gt[GT_WORDS];
  uint32_t qn;
  d = hb_level(a, d, pi, qn);
  if (qn == 0) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  for (uint32_t i = tid; i < GT_WORDS; i += HB_LT) gt[i] = a.gt[i];
  __syncthreads();
  uint2* qx = (d & 1) ? q0 : q1;
  const uint32_t* Fd = hb_F(a, d);
  uint32_t* Fn = hb_F(a, d + 1);
  const uint32_t gm = a.Sg >= 32 ? 0xFFFFFFFFu : (1u << a.Sg) - 1u;
  const uint32_t stride = gridDim.x * HB_LT;
  for (uint32_t v0 = blockIdx.x * HB_LT + (tid & ~63u); v0 < a.N; v0 += stride) {  // (uniform per wave)
    const uint32_t v = v0 + lane;
    uint32_t vw = 0, need = 0, nb = 0;
    uint2 pg = make_uint2(0, 0);
    if (v < a.N) {
      vw = a.vis[v];
      need = gm & ~vw;
      if (need) {
        const unsigned long long x = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(a.pgo) + v);
        pg = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
      }
    }
    const bool heavy = need && pg.y > a.gh;
    if (need && !heavy) {
      const unsigned long long* rp = a.pgr + pg.x;
      for (uint32_t r0 = 0; r0 < pg.y; r0 += HB_BR) {
        unsigned long long rec[HB_BR];
#pragma unroll
        for (uint32_t k = 0; k < HB_BR; ++k) rec[k] = r0 + k < pg.y ? __builtin_nontemporal_load(&rp[r0 + k]) : 0ull;
        uint32_t f[HB_BR];
#pragma unroll
        for (uint32_t k = 0; k < HB_BR; ++k) {
          const uint32_t m = (uint32_t)(rec[k] >> 32) & need & ~nb;
          f[k] = m ? m & Fd[(uint32_t)rec[k] & 0xFFFFFFu] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < HB_BR; ++k) nb |= f[k];
        if (nb == need) break;
      }
    }
    uint64_t hv = __ballot(heavy);
    while (hv) {  // the wave's heavy nodes, one at a time
      const int hl = __ffsll((long long)hv) - 1;
      hv &= hv - 1;
      const uint32_t hneed = (uint32_t)__shfl((int)need, hl);
      const uint32_t h0 = (uint32_t)__shfl((int)pg.x, hl), hc = (uint32_t)__shfl((int)pg.y, hl);
      uint32_t found = 0;
      for (uint32_t rb = 0; rb < hc; rb += 64) {
        uint32_t f = 0;
        if (rb + lane < hc) {
          const unsigned long long rec = a.pgr[h0 + rb + lane];
          const uint32_t m = (uint32_t)(rec >> 32) & hneed & ~found;
          if (m) f = m & Fd[(uint32_t)rec & 0xFFFFFFu];
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) f |= (uint32_t)__shfl_xor((int)f, off);
        found |= f;
        if (found == hneed) break;
      }
      if (lane == (uint32_t)hl) nb = found;
    }
    uint32_t n = 0, bv = 0;
    if (nb) {
      a.vis[v] = vw | nb;
      Fn[v] = nb;
      hb_set_dist(a.dist, a.DSP, v, nb, d + 1);
      bv = a.bucket[v];
      n = mv_parts(gt, v, nb, bv, nullptr, 0);
    }
    bool ok;
    const uint32_t pos = hb_wave_reserve(a, d, n, ok);
    if (ok && n) mv_parts_to(gt, v, nb, bv, [&](uint32_t k, uint2 x) { qx[pos + k] = x; });
  }
}

// --------------------------------------------------------------- gather ----
constexpr uint32_t HB_GR = 8;  // in-records per batch of the gather

// Per (slot, node) of nodes [vlo, vhi): the in-records whose pusher was reached in the slot,
// keyed hop << 24 | src (hop = the pusher's distance + 1, gossip.rs:601-607), as the
// inbound rows inb[c][pair] (lanes hold consecutive nodes: row c of a slot is one store
// instruction), the in-degree and the hop (the node's distance; 0 at the origin, 0xFF
// unreached). A batch of HB_GR in-records and their pushers' 16-byte distance rows are
// loaded together and feed all (up to 16) slots of the half; nodes with more than a.gh
// in-records take the wave path.
__global__ __launch_bounds__(HB_LT) void k_hb_gather(MvArgs a) {
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t v = a.vlo + blockIdx.x * HB_LT + tid;
  const bool in = v < a.vhi;
  const uint32_t Sg = a.Sg, DW = a.DSP / 4;
  const uint4* dist4 = reinterpret_cast<const uint4*>(a.dist);
  const uint2 pg = in ? a.pgo[v] : make_uint2(0, 0);
  const bool heavy = in && pg.y > a.gh;
  bool over = false;
  if (in && !heavy) {
    const unsigned long long* rp = a.pgr + pg.x;
    for (uint32_t h = 0; h * 16 < Sg; ++h) {  // slots [16h, 16h + 16)
      const uint4 dv = dist4[(size_t)v * (DW / 4) + h];
      uint32_t c[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) c[t] = 0;
      for (uint32_t r0 = 0; r0 < pg.y; r0 += HB_GR) {
        uint32_t su[HB_GR], sm[HB_GR];
        uint4 sd[HB_GR];
#pragma unroll
        for (uint32_t k = 0; k < HB_GR; ++k) {
          const bool ok = r0 + k < pg.y;
          const unsigned long long rec = ok ? rp[r0 + k] : 0ull;
          su[k] = (uint32_t)rec & 0xFFFFFFu;
          sm[k] = ok ? (uint32_t)(rec >> (32 + 16 * h)) & 0xFFFFu : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < HB_GR; ++k)
          sd[k] = sm[k] ? dist4[(size_t)su[k] * (DW / 4) + h] : make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
        for (uint32_t t = 0; t < 16; ++t) {
          const uint32_t j = 16 * h + t;
          uint32_t* __restrict__ row = a.inb + (size_t)(a.s0 + j) * a.NP + (v - a.vlo);
#pragma unroll
          for (uint32_t k = 0; k < HB_GR; ++k) {
            const uint32_t w = t < 4 ? sd[k].x : t < 8 ? sd[k].y : t < 12 ? sd[k].z : sd[k].w;
            const uint32_t hp = (w >> (8 * (t & 3))) & 0xFFu;
            if (j < Sg && ((sm[k] >> t) & 1u) && hp != 0xFFu) {  // (sm has no bits at j >= Sg)
              if (c[t] < a.capin) row[(size_t)c[t] * a.PAIRS] = ((hp + 1) << 24) | su[k];
              ++c[t];
            }
          }
        }
      }
#pragma unroll
      for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t j = 16 * h + t;
        if (j >= Sg) continue;
        const size_t p = (size_t)(a.s0 + j) * a.NP + (v - a.vlo);
        const uint32_t w = t < 4 ? dv.x : t < 8 ? dv.y : t < 12 ? dv.z : dv.w;
        over |= c[t] > a.capin;
        a.cnt[p] = c[t];
        a.hops[p] = (uint8_t)((w >> (8 * (t & 3))) & 0xFFu);
      }
    }
  }
  uint64_t hv = __ballot(heavy);
  while (hv) {  // the wave's heavy nodes, one at a time: 64 records per step, ranks by ballot
    const int hl = __ffsll((long long)hv) - 1;
    hv &= hv - 1;
    const uint32_t hvn = (uint32_t)__shfl((int)v, hl);
    const uint32_t h0 = (uint32_t)__shfl((int)pg.x, hl), hc = (uint32_t)__shfl((int)pg.y, hl);
    for (uint32_t j = 0; j < Sg; ++j) {
      const size_t p = (size_t)(a.s0 + j) * a.NP + (hvn - a.vlo);
      uint32_t cc = 0;
      for (uint32_t rb = 0; rb < hc; rb += 64) {
        const uint32_t r = rb + lane;
        bool b = false;
        uint32_t key = 0;
        if (r < hc) {
          const unsigned long long rec = a.pgr[h0 + r];
          if ((uint32_t)(rec >> (32 + j)) & 1u) {
            const uint32_t u = (uint32_t)rec & 0xFFFFFFu;
            const uint32_t hp = a.dist[(size_t)u * a.DSP + j];
            b = hp != 0xFFu;
            key = ((hp + 1) << 24) | u;
          }
        }
        const uint64_t bal = __ballot(b);
        const uint32_t pos =
            cc + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (b && pos < a.capin) a.inb[(size_t)pos * a.PAIRS + p] = key;
        cc += (uint32_t)__popcll(bal);
      }
      if (lane == 0) {
        over |= cc > a.capin;
        a.cnt[p] = cc;
        a.hops[p] = a.dist[(size_t)hvn * a.DSP + j];
      }
    }
  }
  if (over) atomicOr(a.err, ERR_INBOUND);
}

}  // namespace

// ------------------------------------------------------------------ host ----
// Push-graph geometry: slices of the multi BFS's expand width, T rows of its coarse bins,
// and per coarse bin a region of pgr holding every push into it (an entry pushes to at
// most ASZ peers; `parts` entries per node at most).
void hb_geometry(Engine& e, uint32_t parts) {
  MvGeom& g = e.mv;
  // 1,024-node slices where the stage fits LDS: a quarter of the T rows every coarse bin's
  // CSR walks (C4: 977 rows instead of 3,907)
  static const bool narrow = std::getenv("GS_HB_XT256") && std::getenv("GS_HB_XT256")[0] == '1';  // (tuning)
  if (!narrow && mv_hist_bytes(g.nbc) + (size_t)MV_XT_L * e.ASZP * 8 <= 160 * 1024) g.XT = MV_XT_L;
  e.hb_parts = parts;
  e.hb_slices = (e.N + g.XT - 1) / g.XT;
  g.rows_cap = (size_t)e.hb_slices * parts;
  g.area_cap = g.rows_cap * g.XT * e.ASZ;
  e.hb_bin_cap = ((size_t)1 << g.BSC) * e.ASZ * parts;
}

static MvArgs hb_args(Engine& e, const MvGroup& gr, uint32_t g) {
  MvArgs a = mv_args(e, gr, g);
  a.dist = e.hb_dist;
  a.DSP = e.hb_dsp;
  a.pgo = e.hb_pgo;
  a.F = e.hb_F;
  a.pgr = e.hb_pgr;
  a.pg_bin_cap = e.hb_bin_cap;
  a.pg_parts = e.hb_parts;
  a.pg_slices = e.hb_slices;
  a.gh = (e.prm.flags & GS_FLAG_NARROW_WAVE_PATH) ? 4u : HB_GH;  // (small tests reach the wave paths)
  a.small = HB_SMALL;
  if (const char* x = std::getenv("GS_HB_SMALL")) a.small = (uint32_t)std::strtoul(x, nullptr, 10);
  if (e.prm.flags & GS_FLAG_NO_SMALL_LEVELS) a.small = 0;
  a.bu_min = std::max<uint32_t>(1, e.N / 32);  // (tuning: GS_HB_BU_MIN)
  if (const char* x = std::getenv("GS_HB_BU_MIN")) a.bu_min = (uint32_t)std::strtoul(x, nullptr, 10);
  return a;
}

static void hb_launch_level(Engine& e, const MvArgs& a, bool bu, uint32_t d, uint32_t pi, uint32_t pred) {
  if (bu) {
    const uint32_t grid = std::min<uint32_t>((e.N + HB_LT - 1) / HB_LT, 4096);
    hipLaunchKernelGGL(k_hb_bu, dim3(grid), dim3(HB_LT), 0, e.st, a, d, pi, e.mv_q[0], e.mv_q[1]);
  } else {
    // (at least enough workgroups to clear F_{d-1} with <= 16 stores of 16 B per thread)
    const uint32_t gclr = std::min<uint32_t>(2048, (e.N / 4 + HB_LT * 16 - 1) / (HB_LT * 16));
    const uint32_t grid = std::max<uint32_t>(
        std::max<uint32_t>(1, gclr), std::min<uint32_t>((std::max<uint32_t>(pred, 1) * 2 + HB_LT - 1) / HB_LT, 8192));
    GS_ASZP_DISPATCH_V(e.ASZP, hipLaunchKernelGGL(k_hb_td<A>, dim3(grid), dim3(HB_LT), 0, e.st, a, d, pi, e.mv_q[0],
                                                  e.mv_q[1]));
  }
}

static void hb_launch_small(Engine& e, const MvArgs& a, uint32_t mode, uint32_t d0, uint32_t pi, const uint2* seeds,
                            uint32_t nseed, uint32_t seq) {
  GS_ASZP_DISPATCH_V(e.ASZP, hipLaunchKernelGGL(k_hb_small<A>, dim3(1), dim3(HB_ST), 0, e.st, a, mode, d0, pi,
                                                e.mv_q[0], e.mv_q[1], e.mv_hstate_dev, seeds, nseed, seq));
}

hipError_t launch_bfs_hybrid(Engine& e, bool record) {
  hipError_t r = hipSuccess;
  const MvGeom& g = e.mv;
  const size_t lds_x = mv_hist_bytes(g.nbc) + (size_t)g.XT * e.ASZP * 8;
  const size_t lds_c = hb_csr_lds_bytes(g.BSC);
  if (!e.mv_attr_set) {
    GS_ASZP_DISPATCH(e.ASZP, {
      r = g.XT == MV_XT_L ? hipFuncSetAttribute((const void*)k_hb_graph<A, MV_XT_L>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_x)
                          : hipFuncSetAttribute((const void*)k_hb_graph<A, MV_XT>,
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_x);
    });
    if (r != hipSuccess) return r;
    if ((r = hipFuncSetAttribute((const void*)k_hb_csr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c)))
      return r;
    e.mv_attr_set = true;
  }
  static const bool polled_only = std::getenv("GS_MV_POLLED") && std::getenv("GS_MV_POLLED")[0] == '1';
  const uint32_t cgrid = ((g.nbc + 7) / 8) * 8;
  const uint32_t ggrid = (e.NP + HB_LT - 1) / HB_LT;
  for (uint32_t gi = 0; gi < (uint32_t)e.mv_groups.size(); ++gi) {
    const MvGroup& gr = e.mv_groups[gi];
    MvArgs a = hb_args(e, gr, gi);
    a.record = record ? 1u : 0u;
    uint32_t* hp = e.mv_prof + (size_t)gi * MV_PROF_WORDS;
    a.hprof = e.mv_prof_dev + (size_t)gi * MV_PROF_WORDS;
    {  // the newest published level profile of this group (a tail kernel of an earlier round)
      volatile uint32_t* vp = hp;
      const uint32_t sq = vp[0];
      if (sq != e.mv_prof_seen[gi] && sq != 0) {
        std::atomic_thread_fence(std::memory_order_acquire);
        const uint32_t nl = std::min<uint32_t>((uint32_t)vp[1], 255u);
        std::vector<uint32_t> pv(nl);
        for (uint32_t k = 0; k < nl; ++k) pv[k] = vp[2 + k];
        std::atomic_thread_fence(std::memory_order_acquire);
        if (vp[0] == sq) {
          e.mv_pred[gi] = std::move(pv);
          e.mv_prof_seen[gi] = sq;
        }
      }
    }
    hipEvent_t t0;
    e.tbegin("bfs", &t0);
    // 1. the push graph (also the round's visited masks and distances)
    const uint32_t xgrid = std::min<uint32_t>(e.hb_slices, 4096);
    if (g.XT == MV_XT_L) {
      GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_hb_graph<A, MV_XT_L>), dim3(xgrid), dim3(MV_XT_L), lds_x, e.st, a));
    } else {
      GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_hb_graph<A, MV_XT>), dim3(xgrid), dim3(MV_XT), lds_x, e.st, a));
    }
    hipLaunchKernelGGL(k_hb_csr, dim3(cgrid), dim3(HB_CT), lds_c, e.st, a);
    // 2. the levels
    const std::vector<uint32_t>& pv = e.mv_pred[gi];
    volatile uint32_t* hs = e.mv_hlvl + 256;  // host-mapped: the small kernel's (level, entries)
    if (pv.empty() || polled_only) {  // no profile yet: the host follows the levels
      std::vector<uint32_t> prof;
      hs[0] = MV_PENDING;
      hb_launch_small(e, a, HB_HEAD, 0u, 0u, e.mv_seed + gr.seed0, gr.nseed, 0u);
      uint32_t d = 0;
      if ((r = mv_wait(hs, e.st, d))) return r;
      uint32_t qn = hs[1];
      std::vector<uint32_t> sizes(256, 0);
      if ((r = hipMemcpyAsync(sizes.data(), e.lvl, 256 * 4, hipMemcpyDeviceToHost, e.st))) return r;
      if ((r = hipStreamSynchronize(e.st))) return r;
      prof.assign(sizes.begin(), sizes.begin() + std::min<uint32_t>(d + 1, 256));
      while (qn > 0) {
        if (d >= 254) return hipErrorNotSupported;  // frontier still non-empty after 254 levels
        e.bfs_level = d;
        if (qn <= a.small) {
          hs[0] = MV_PENDING;
          hb_launch_small(e, a, HB_POLL, d, 0u, nullptr, 0u, 0u);
          if ((r = mv_wait(hs, e.st, d))) return r;
          qn = hs[1];
        } else {
          hb_launch_level(e, a, qn >= a.bu_min, d, MV_NOPAIR, qn);
          ++d;
          if ((r = hipMemcpyAsync(e.h_err + 1, e.lvl + d, 4, hipMemcpyDeviceToHost, e.st))) return r;
          if ((r = hipStreamSynchronize(e.st))) return r;
          qn = e.h_err[1];
        }
        if ((r = hipMemcpyAsync(sizes.data(), e.lvl, 256 * 4, hipMemcpyDeviceToHost, e.st))) return r;
        if ((r = hipStreamSynchronize(e.st))) return r;
        prof.assign(sizes.begin(), sizes.begin() + std::min<uint32_t>(d + 1, 256));
      }
      while (!prof.empty() && prof.back() == 0) prof.pop_back();
      if (!polled_only) e.mv_pred[gi] = std::move(prof);
    } else {
      // predicted: head kernel, one level kernel per profiled level above the small bound
      // (bottom-up for the large ones), a margin, and the tail kernel
      uint32_t k0 = 0;
      while (k0 < pv.size() && pv[k0] <= a.small) ++k0;
      uint32_t k1 = (uint32_t)pv.size();
      while (k1 > k0 && pv[k1 - 1] <= a.small) --k1;
      const uint32_t nlev = std::min<uint32_t>(k1 - k0 + mv_margin(), 250);
      if (e.mv_diag) {
        std::fprintf(stderr, "GS_HB_DIAG group %u: head levels %u, then", gi, k0);
        for (uint32_t i = 0; i < nlev; ++i) {
          const uint32_t pred = k0 + i < pv.size() ? pv[k0 + i] : 0u;
          std::fprintf(stderr, " %u%s", pred, pred >= a.bu_min ? "(bu)" : "(td)");
        }
        std::fprintf(stderr, ", tail from %u\n", k0 + nlev);
      }
      hb_launch_small(e, a, HB_HEAD, 0u, 0u, e.mv_seed + gr.seed0, gr.nseed, 0u);
      for (uint32_t i = 0; i < nlev; ++i) {
        const uint32_t pred = k0 + i < pv.size() ? pv[k0 + i] : 0u;
        hb_launch_level(e, a, pred >= a.bu_min, 0u, i, pred);
      }
      const uint32_t seq = ++e.mv_seq ? e.mv_seq : ++e.mv_seq;  // (never 0)
      hb_launch_small(e, a, HB_TAIL, 0u, nlev, nullptr, 0u, seq);
    }
    e.tend("bfs", t0);
    // 3. the gather
    e.tbegin("gather", &t0);
    hipLaunchKernelGGL(k_hb_gather, dim3(ggrid), dim3(HB_LT), 0, e.st, a);
    e.tend("gather", t0);
  }
  return hipGetLastError();
}

}  // namespace gs
