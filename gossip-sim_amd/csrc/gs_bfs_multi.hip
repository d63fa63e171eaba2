// gs_bfs_multi.hip -- Cluster::run_gossip (gossip.rs:494-615) for large clusters as a
// batched multi-source frontier BFS: every slot of a slot group advances at once,
// and a node's active-set row is expanded ONCE per level for all the group's slots
// that reach it at that level.
//
// A slot group is a contiguous range of at most GW slots (bit j = slot s0 + j). The
// visited state is a slot mask per node (vis[N]); a frontier entry is (node u, entry
// k, slot mask M): the slots in M first reached u at this level and all of them push
// from u's entry k = min(bucket[u], bucket[origin]) (push_active_set.rs:38-52). Slots
// that reach u at the same level through different entries become separate entries.
// Prune masks and egress bytes are node-major ([node][slot]) in this mode: an entry
// reads all its slots' masks in one line. Per BFS level:
//
//   expand (workgroup w owns frontier entries [w*256, (w+1)*256)): loads the entry's
//     row (the compact own-bucket table when k = bucket[u]) and its slots' masks, takes
//     per slot the first `fanout` unpruned non-origin ring slots (failed peers burn a
//     slot, gossip.rs:527-541) and ORs the slot's bit into a per-ring-slot mask; every
//     pushed-to peer w becomes ONE record (src u, w, slots) however many slots pushed
//     there. Records are ranked per coarse destination bin (2^BSC nodes) with LDS
//     atomics, staged sorted by bin and written as one contiguous run; T row [base, bin
//     starts..., total].
//   apply (one workgroup per coarse bin, bins dealt to XCDs in contiguous ranges): ORs
//     the level's records into an LDS copy of the bin's vis masks -- new bits are first
//     arrivals at hop d+1 (gossip.rs:594-600) -- appends new nodes to the next frontier
//     (one entry per distinct entry k) and the level's records, stamped with their hop,
//     to the fine bins' pools.
//   gather (after the last level, one workgroup per fine bin of 2^BSF nodes): the
//     fine bin's pool (records of every level) as an LDS CSR by destination; per (slot, node): in-degree, the inbound records
//     hop << 24 | src (gossip.rs:601-607) as rows inb[c][pair] coalesced over nodes, and
//     the hop (1 + the smallest pusher level; 0 at the origin; unreached = 0xFF).
//
// The level loop never stalls the GPU on the host: expand(d) writes its frontier size
// to host-mapped memory and the host polls it two levels late (after an event).
// Results equal k_bfs_level's: hops, in-degrees, inbound record sets, egress.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "gs_consume_dev.h"
#include "gs_device.h"
#include "gs_internal.h"
#include "gs_mv_dev.h"

namespace gs {

namespace {



// Level d (pi == MV_NOPAIR), or pair pi's level dpair[pi] (the predicted loop; 0 entries
// there when the BFS already ended: a no-op).
// XT entries per slice (= threads): a slice writes one T row of nbc + 2 words and every
// apply workgroup reads one word of every row, so with thousands of coarse bins (C5: 1,220)
// the rows cost more than the records; 1,024-entry slices make 4x fewer rows (C5 BFS
// 9.36 -> 6.95 ms per round) while at C4's 245 bins 256-entry slices stay faster (730 vs
// 768 us).
template <int ASZP, uint32_t XT>
__global__ __launch_bounds__(XT) void k_mv_expand(MvArgs a, uint32_t d, uint32_t pi, const uint2* __restrict__ q0,
                                                  const uint2* __restrict__ q1) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ MvSlots S;
  __shared__ uint32_t sbase;
  if (pi != MV_NOPAIR) d = a.dpair[pi];
  const uint32_t qn = d < 254 ? a.lvl[d] : 0u;
  const uint2* __restrict__ qcur = (d & 1) ? q1 : q0;
  if (pi == MV_NOPAIR && blockIdx.x == 0 && threadIdx.x == 0)  // the host's termination poll (host-mapped)
    __hip_atomic_store(&a.hlvl[d], qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint32_t G = (qn + XT - 1) / XT;
  if (blockIdx.x >= G) return;  // idle workgroups leave before any setup
  if (G > a.rows_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_ROWS);
    return;
  }
  const uint32_t tid = threadIdx.x, nb = a.nbc, BSC = a.BSC, UB = a.UB, BPm = (1u << BSC) - 1;
  mv_slots_load(a, S, tid, XT);
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);  // [nb] + scan words
  unsigned long long* stage = reinterpret_cast<unsigned long long*>(smem + mv_hist_bytes(nb));  // [XT * ASZP]
  for (uint32_t w = blockIdx.x; w < G; w += gridDim.x) {
    for (uint32_t i = tid; i < nb; i += XT) hist[i] = 0;
    __syncthreads();
    uint32_t row[ASZP], acc[ASZP], u = 0;
#pragma unroll
    for (int s = 0; s < ASZP; ++s) { row[s] = 0; acc[s] = 0; }
    const uint32_t i = w * XT + tid;
    if (i < qn) mv_expand_entry<ASZP>(a, qcur[i], S, row, acc, u);
    // every LDS atomic after every load: each record's rank within its coarse bin
    uint32_t rk[ASZP];
#pragma unroll
    for (int s = 0; s < ASZP; ++s) rk[s] = acc[s] ? atomicAdd(&hist[row[s] >> BSC], 1u) : 0u;
    __syncthreads();
    const uint32_t total = mv_block_scan(hist, nb, hist + nb);
    // the slice's run at a fixed place (an entry pushes to at most ASZ distinct peers): no
    // device-wide counter, which ~2,700 slices of a peak level would queue on (one word
    // takes ~88 returning atomics per us)
    if (tid == 0) {
      const size_t b64 = (size_t)w * XT * a.ASZ;
      uint32_t base = (uint32_t)b64;
      if (b64 + total > a.area_cap) {
        atomicOr(a.err, ERR_MV_CAP | ERR_MVD_AREA);
        base = 0xFFFFFFFFu;
      }
      sbase = base;
    }
    __syncthreads();
    const uint32_t base = sbase;
    const bool ok = base != 0xFFFFFFFFu;
    for (uint32_t b = tid; b < nb; b += XT) mv_t(a, w, 1 + b) = ok ? hist[b] : 0u;
    if (tid == 0) {
      mv_t(a, w, 0) = ok ? base : 0u;
      mv_t(a, w, 1 + nb) = ok ? total : 0u;
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
      for (uint32_t r = tid; r < total; r += XT) a.area[base + r] = stage[r];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- apply ----
__host__ __device__ inline size_t mv_apply_lds_bytes(uint32_t BSC) {
  return 4 * (2 * (size_t)MV_SEG + 1 + 2 * ((size_t)1 << BSC) + 64 + GT_WORDS);
}


__global__ __launch_bounds__(MV_AT) void k_mv_apply(MvArgs a, uint32_t d, uint32_t pi, uint2* __restrict__ q0,
                                                   uint2* __restrict__ q1) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (pi != MV_NOPAIR) d = a.dpair[pi];
  const uint32_t qn = d < 254 ? a.lvl[d] : 0u;
  uint2* __restrict__ qnxt = (d & 1) ? q0 : q1;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.ctr[0] = 0;  // expand(d) is done with it; expand(d + 1) starts at 0
    if (pi != MV_NOPAIR) a.dpair[pi + 1] = qn ? d + 1 : d;
  }
  if (qn == 0 && !a.xrows) return;  // (an exchange partition applies what other ranks pushed to it)
  const uint32_t c = mv_xcd_bin(blockIdx.x, a.nbc);
  if (c >= a.nbc) return;
  const uint32_t tid = threadIdx.x, BSC = a.BSC, UB = a.UB, BP = 1u << BSC, BPm = BP - 1;
  const uint32_t G = a.xrows ? a.xrows : (qn + a.XT - 1) / a.XT;
  const uint32_t v0 = c << BSC, nv = min(BP, a.N - v0);
  // GS_PHASE_PROFILE: thread 0's clocks at pclk[16..19] (T column + scan, vis load, records, tail)
  unsigned long long tm = a.pclk && tid == 0 ? wall_clock64() : 0;
  auto mark = [&](int ph) {
    if (a.pclk && tid == 0) {
      const unsigned long long now = wall_clock64();
      atomicAdd(&a.pclk[ph], now - tm);
      tm = now;
    }
  };
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem);  // [MV_SEG + 1]
  uint32_t* sb = pre + MV_SEG + 1;                    // [MV_SEG]
  uint32_t* visL = sb + MV_SEG;                       // [BP]
  uint32_t* vis0 = visL + BP;                         // [BP]
  uint32_t* ctl = vis0 + BP;                          // [64]: [0..15] scan words, [1] base, [8..23] counts
  uint32_t* gt = ctl + 64;                            // [GT_WORDS]
  // the level's records go to the pool run of their fine bin (2^BSF nodes): cursors per
  // fine bin of this coarse bin, reserved once per wave per fine bin
  const uint32_t FS = a.BSC - a.BSF, NF = 1u << FS, f0 = c << FS;
  uint32_t* fcur = ctl + 32;  // [NF <= 16] records appended this level
  uint32_t* fbase = ctl + 48;  // [NF] the fine bins' pool fills before this level
  if (tid < NF) {
    fcur[tid] = 0;
    fbase[tid] = f0 + tid - a.flo < a.fno ? a.pused[f0 + tid - a.flo] : 0u;
  }
  bool loaded = false;  // vis is read only by bins that receive records at this level
  for (uint32_t c0 = 0; c0 < G; c0 += MV_SEG) {
    const uint32_t gc = min(MV_SEG, G - c0);
    for (uint32_t i = tid; i < gc; i += MV_AT) {
      const uint32_t st = mv_t(a, c0 + i, 1 + c);
      pre[i] = mv_t(a, c0 + i, 2 + c) - st;  // bin starts are exclusive; entry 1 + nbc is the run's total
      sb[i] = mv_t(a, c0 + i, 0) + st;
    }
    __syncthreads();
    const uint32_t ct = mv_block_scan(pre, gc, ctl);
    mark(16);
    if (ct == 0) continue;  // (uniform)
    if (tid == 0) pre[gc] = ct;
    if (!loaded) {
      for (uint32_t i = tid; i < GT_WORDS; i += MV_AT) gt[i] = a.gt[i];
      for (uint32_t i = tid; i < nv; i += MV_AT) {
        const uint32_t m = a.vis[v0 + i];
        visL[i] = m;
        vis0[i] = m;
      }
      loaded = true;
    }
    __syncthreads();
    mark(17);
    // MV_AR records per thread per trip: their searches and area loads are issued
    // together, so a trip waits for one memory round trip, not MV_AR
    constexpr uint32_t MV_AR = 4;
    for (uint32_t r0 = 0; r0 < ct; r0 += MV_AT * MV_AR) {
      unsigned long long rec[MV_AR];
#pragma unroll
      for (uint32_t k = 0; k < MV_AR; ++k) {
        const uint32_t r = r0 + k * MV_AT + tid;
        uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pre[mid] <= r) lo = mid; else hi = mid;
        }
        rec[k] = r < ct ? a.area[sb[lo] + (r - pre[lo])] : ~0ull;
      }
#pragma unroll
      for (uint32_t k = 0; k < MV_AR; ++k) {
        const bool live = r0 + k * MV_AT + tid < ct;
        if (!live) continue;
        uint32_t vl = (uint32_t)(rec[k] >> UB) & BPm;
        if (GS_OOB(vl, nv, a.err, "multi record node")) vl = 0;
        const uint32_t m = (uint32_t)(rec[k] >> (UB + BSC));
        atomicOr(&visL[vl], m);
        const uint32_t fb = vl >> a.BSF;
        if (f0 + fb - a.flo >= a.fno) continue;  // kept fine bins only
        // the record's place in its fine bin's run: one LDS atomic per lane (measured faster
        // than one per wave and fine bin by ballots: 19.5-19.7 vs 21.2-24.5 us per launch at C4)
        const size_t pp = (size_t)fbase[fb] + atomicAdd(&fcur[fb], 1u);
        if (pp < a.pcap)
          a.pool[(size_t)(f0 + fb - a.flo) * a.pcap + pp] =
              mv_pool_rec(a, (uint32_t)rec[k] & ((1u << UB) - 1), vl & ((1u << a.BSF) - 1), d + 1, m);
      }
    }
    __syncthreads();
    mark(18);
  }
  __syncthreads();
  if (tid < NF && f0 + tid - a.flo < a.fno) {  // each kept fine bin's pool fill
    const uint32_t fl = f0 + tid - a.flo;
    const uint32_t used = fbase[tid], n = fcur[tid];
    const bool over = (size_t)used + n > a.pcap;
    if (over) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_POOL);
    if (n) a.pused[fl] = over ? (uint32_t)a.pcap : used + n;
  }
  if (!loaded) {  // no records: no first arrivals in this bin
    mark(19);
    return;
  }
  // first arrivals (hop d + 1) become next-level entries, in node order
  uint32_t cntp = 0;
  for (uint32_t i = tid; i < nv; i += MV_AT) {
    const uint32_t nw = visL[i] & ~vis0[i];
    if (nw) cntp += mv_parts(gt, v0 + i, nw, a.bucket[v0 + i], nullptr, 0);
  }
  const uint32_t incl = wave_incl_scan(cntp);
  if ((tid & 63) == 63) ctl[8 + (tid >> 6)] = incl;
  __syncthreads();
  uint32_t off = 0, tnew = 0;
  for (uint32_t k = 0; k < MV_AT / 64; ++k) {
    if (k < (tid >> 6)) off += ctl[8 + k];
    tnew += ctl[8 + k];
  }
  if (tnew == 0) {
    mark(19);
    return;
  }
  if (tid == 0) {
    const uint32_t base = atomicAdd(&a.lvl[d + 1], tnew);
    ctl[1] = base;
    if ((size_t)base + tnew > a.q_cap) { atomicOr(a.err, ERR_MV_CAP | ERR_MVD_Q); ctl[1] = 0xFFFFFFFFu; }
  }
  __syncthreads();
  if (ctl[1] == 0xFFFFFFFFu) return;
  uint32_t pos = ctl[1] + off + incl - cntp;
  for (uint32_t i = tid; i < nv; i += MV_AT) {
    const uint32_t nw = visL[i] & ~vis0[i];
    if (!nw) continue;
    const uint32_t v = v0 + i;
    a.vis[v] = visL[i];
    pos += mv_parts(gt, v, nw, a.bucket[v], qnxt, pos);
  }
  mark(19);
}

// ------------------------------------------------------------ small levels ----
constexpr uint32_t MV_ST = 1024;     // threads of the small-level workgroup
constexpr uint32_t MV_SMALL_LP = 8192;  // fine bins up to which the small kernel keeps pool fills in LDS
constexpr uint32_t MV_SMALL = 1024;  // frontier entries at most for a head level (default; GS_MV_SMALL)
constexpr uint32_t MV_SQ = 2048;     // frontier entries of a level kept in the small kernel's LDS queue
enum : uint32_t { MV_HEAD = 0, MV_TAIL = 1, MV_POLL = 2 };  // small-kernel modes


// Levels run inside ONE workgroup, level after level, with no launch between them: every
// entry is expanded (mv_expand_entry), each record ORs its slots into vis with a
// device-scope atomic -- the atomic that sets a slot's bit is that slot's first arrival
// (hop d + 1, gossip.rs:594-600) -- new bits become next-level entries (an LDS queue of
// MV_SQ entries, the rest in global memory), and the record is appended to its fine bin's
// pool run. Modes:
//   MV_HEAD  the round's first levels: seeds the group (lvl, pool fills, vis of the seed
//            nodes, the first queue), runs while a level has at most a.small entries,
//            leaves the level where it stopped in dpair[0] for the expand/apply pairs;
//   MV_TAIL  from level dpair[pi] to the end of the BFS whatever the level sizes (the host
//            enqueued pairs by the previous round's level profile; a level the pairs did not
//            take is expanded here, slowly but correctly); writes the round's level profile
//            to host-mapped memory (hprof) for the next round's prediction;
//   MV_POLL  from level d0 while levels have at most a.small entries (the polled loop).
// Every mode reports (level, entries) where it stopped in hstate.
template <int ASZP>
__global__ __launch_bounds__(MV_ST) void k_mv_small(MvArgs a, uint32_t mode, uint32_t d0, uint32_t pi,
                                                    uint2* __restrict__ q0, uint2* __restrict__ q1,
                                                    uint32_t* __restrict__ hstate, const uint2* __restrict__ seeds,
                                                    uint32_t nseed, uint32_t seq) {
  // (when LP) [fno] the pool fills: the records' pool places come from LDS atomics, the
  // global fills are written once at the end
  extern __shared__ __attribute__((aligned(16))) uint32_t lp[];
  __shared__ uint2 qL[2][MV_SQ];
  __shared__ MvSlots S;
  __shared__ uint32_t gt[GT_WORDS], cnt_s;
  const uint32_t tid = threadIdx.x;
  const bool LP = a.fno <= MV_SMALL_LP;  // (uniform; beyond, device-scope atomics on a.pused)
  mv_slots_load(a, S, tid, MV_ST);
  for (uint32_t i = tid; i < GT_WORDS; i += MV_ST) gt[i] = a.gt[i];
  uint32_t d = mode == MV_TAIL ? a.dpair[pi] : d0;
  bool inL = false;  // the current level's entries [0, MV_SQ) are in qL[d & 1]
  if (mode == MV_HEAD) {  // the group's round starts here: no memsets of lvl / pool fills, no seed launch
    for (uint32_t i = tid; i < 256; i += MV_ST) a.lvl[i] = i == 0 ? nseed : 0u;
    for (uint32_t f = tid; f < a.fno; f += MV_ST) {
      a.pused[f] = 0;
      if (LP) lp[f] = 0;
    }
    if (tid == 0) a.ctr[0] = 0;
    if (tid < nseed) {
      const uint2 sd = seeds[tid];  // distinct origins (vis was cleared before this kernel)
      qL[0][tid] = sd;
      a.vis[sd.x & 0xFFFFFFu] = sd.y;
    }
    inL = true;
    __syncthreads();  // (full: the seeds' vis stores land before any vis atomic)
  } else if (LP) {
    for (uint32_t f = tid; f < a.fno; f += MV_ST) lp[f] = mv_ld(&a.pused[f]);
  }
  // GS_PHASE_PROFILE: section clocks of thread 0 at pclk[0..4] (setup, expand loads,
  // atomics + places, Lt + barrier; [4] levels)
  unsigned long long tm = a.pclk && tid == 0 ? wall_clock64() : 0;
  auto mark = [&](int ph) {
    if (a.pclk && tid == 0) {
      const unsigned long long now = wall_clock64();
      atomicAdd(&a.pclk[ph], now - tm);
      tm = now;
    }
  };
  uint32_t qn = mode == MV_HEAD ? nseed : (d < 256 ? a.lvl[d] : 0u);
  const uint32_t lim = mode == MV_TAIL ? 0xFFFFFFFFu : a.small;
  __syncthreads();
  mark(0);
  while (qn > 0 && qn <= lim && d < 254) {
    const uint2* qg = (d & 1) ? q1 : q0;
    uint2* qgn = (d & 1) ? q0 : q1;
    const uint2* ql = qL[d & 1];
    uint2* qln = qL[(d + 1) & 1];
    if (tid == 0) {
      cnt_s = 0;
      if (a.pclk) atomicAdd(&a.pclk[4], 1ull);
    }
    lds_barrier();
    for (uint32_t i0 = 0; i0 < qn; i0 += MV_ST) {
      const uint32_t i = i0 + tid;
      uint32_t row[ASZP], acc[ASZP], u = 0;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) { row[s] = 0; acc[s] = 0; }
      if (i < qn) mv_expand_entry<ASZP>(a, inL && i < MV_SQ ? ql[i] : qg[i], S, row, acc, u);
      if (a.pclk && i0 == 0) {  // (profiling only: wait for the entry's loads)
        uint32_t x = 0;
#pragma unroll
        for (int s = 0; s < ASZP; ++s) x |= acc[s];
        if (x == 0xFFFFFFFFu) atomicOr(a.err, 0u);
        mark(1);
      }
      // every global access of the entry is issued before any result is used (one wait,
      // not one round trip per pushed-to peer): the vis atomics, the peers' buckets and,
      // without LDS fills, the pool-place atomics
      uint32_t old[ASZP], pp[ASZP], bw[ASZP];
#pragma unroll
      for (int s = 0; s < ASZP; ++s) old[s] = acc[s] ? atomic_or_wg(&a.vis[row[s]], acc[s]) : 0xFFFFFFFFu;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) bw[s] = acc[s] ? (uint32_t)a.bucket[row[s]] : 0u;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        const uint32_t f = (row[s] >> a.BSF) - a.flo;
        const bool kept = acc[s] && f < a.fno;  // kept bins only
        pp[s] = !kept ? 0xFFFFFFFFu : LP ? atomicAdd(&lp[f], 1u) : atomic_add_wg(&a.pused[f], 1u);
      }
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        if (!acc[s]) continue;
        const uint32_t w = row[s];
        const uint32_t nw = acc[s] & ~old[s];
        if (pp[s] != 0xFFFFFFFFu) {
          const uint32_t f = (w >> a.BSF) - a.flo;
          if (pp[s] < a.pcap)
            a.pool[(size_t)f * a.pcap + pp[s]] = mv_pool_rec(a, u, w & ((1u << a.BSF) - 1), d + 1, acc[s]);
          else
            atomicOr(a.err, ERR_MV_CAP | ERR_MVD_POOL);
        }
        if (nw) {  // this thread's first arrivals at w (another thread may add more bits to w)
          const uint32_t n = mv_parts(gt, w, nw, bw[s], nullptr, 0);
          const uint32_t base = atomicAdd(&cnt_s, n);
          if ((size_t)base + n <= a.q_cap) {
            mv_parts_to(gt, w, nw, bw[s], [&](uint32_t k, uint2 x) {
              if (base + k < MV_SQ) qln[base + k] = x;
              else qgn[base + k] = x;
            });
          } else {
            atomicOr(a.err, ERR_MV_CAP | ERR_MVD_Q);
          }
        }
      }
    }
    lds_barrier();
    mark(2);
    qn = min(cnt_s, (uint32_t)a.q_cap);
    ++d;
    if (tid == 0) a.lvl[d] = qn;
    inL = true;
    if (qn > MV_SQ) __syncthreads();  // (entries beyond the LDS queue went to global memory)
    else lds_barrier();
    mark(3);
  }
  if (LP)
    for (uint32_t f = tid; f < a.fno; f += MV_ST) a.pused[f] = min(lp[f], (uint32_t)a.pcap);
  if (qn > 0 && inL && mode != MV_TAIL) {  // the next level's entries for expand: the LDS part to global memory
    uint2* qg = (d & 1) ? q1 : q0;
    for (uint32_t i = tid; i < min(qn, MV_SQ); i += MV_ST) qg[i] = qL[d & 1][i];
  }
  if (mode == MV_TAIL && qn > 0 && tid == 0) atomicOr(a.err, ERR_DEPTH);  // level 254 not empty
  if (tid == 0) {
    if (mode == MV_HEAD) a.dpair[0] = d;
    if (mode == MV_TAIL) {  // the round's level profile for the host's next prediction
      uint32_t* hp = a.hprof;
      const uint32_t nl = min(d, 255u);
      // seqlock: 0 (in progress, the host skips it) before the sizes, the new seq after
      __hip_atomic_store(&hp[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __atomic_thread_fence(__ATOMIC_RELEASE);  // (the 0 is visible before any size)
      for (uint32_t k = 0; k < nl; ++k) __hip_atomic_store(&hp[2 + k], a.lvl[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&hp[1], nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&hp[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(&hstate[1], qn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&hstate[0], d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // the host polls this word
  }
  if (tid == 0 && mode != MV_TAIL)  // per-level sizes for the polled loop / diagnostics (tid 0 wrote lvl[])
    for (uint32_t k = d0; k < d && k < 256; ++k)
      __hip_atomic_store(&a.hlvl[k], a.lvl[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// --------------------------------------------------------------- gather ----
constexpr uint32_t MV_GC = 12;        // records per gather thread kept in registers between the passes
constexpr uint32_t MV_GLDS_DEF = 78 * 1024;  // gather LDS: two workgroups per CU (GS_MV_GLDS_KB: tuning)
static uint32_t mv_glds() {
  static const uint32_t v = [] {
    const char* x = std::getenv("GS_MV_GLDS_KB");
    return x ? std::min<uint32_t>(160, std::max<uint32_t>(16, (uint32_t)std::strtoul(x, nullptr, 10))) * 1024u : MV_GLDS_DEF;
  }();
  return v;
}
constexpr uint32_t MV_WSCR = 64 + CACHE_CAP;  // fused consume: per-wave LDS scratch (u32)
constexpr uint32_t MV_CSCR = (MV_GT / 64) * MV_WSCR * 4;  // bytes of all waves' scratch

__host__ __device__ inline size_t mv_gather_fixed_bytes(uint32_t BSF) {
  return 4 * (2 * (((size_t)1 << BSF) + 1) + 16 + 32);
}

// The LDS CSR of one fine bin's records: cn[i] .. cn[i + 1] (minus the range base) index
// node i's records keys[] = hop << 24 | src and msk[] = slot masks.
struct MvCsr {
  uint32_t *cn, *cur, *ctl, *sorg, *keys, *msk;
};

// After the last level, per kept fine bin f (local index; node base v0): the bin's pool
// (records of every level, mv_pool_rec) as an LDS CSR by destination. Nodes whose records
// exceed gcap are taken in consecutive ranges; body(lo, hi, base) runs on each range (all
// threads; no barrier inside body is needed, one follows it).
template <class Body>
__device__ inline void mv_bin_csr(const MvArgs& a, uint32_t f, uint32_t nv, uint32_t gcap, const MvCsr& L,
                                  Body body) {
  const uint32_t tid = threadIdx.x, UB = a.UB, BSF = a.BSF, BP = 1u << BSF, BPm = BP - 1;
  const uint32_t um = (1u << UB) - 1, MS = UB + BSF + 8;
  unsigned long long tm = a.pclk && tid == 0 ? wall_clock64() : 0;
  auto mark = [&](int ph) {
    if (a.pclk && tid == 0) {
      const unsigned long long now = wall_clock64();
      atomicAdd(&a.pclk[ph], now - tm);
      tm = now;
    }
  };
  uint32_t *cn = L.cn, *cur = L.cur, *ctl = L.ctl, *keys = L.keys, *msk = L.msk;
  const unsigned long long* pool = a.pool + (size_t)f * a.pcap;  // (f: local kept-bin index)
  for (uint32_t i = tid; i <= BP; i += MV_GT) cn[i] = 0;
  if (tid < a.Sg) L.sorg[tid] = a.origin[a.s0 + tid];
  const uint32_t Etot = min(a.pused[f], (uint32_t)a.pcap);
  if (a.pclk && tid == 0) atomicAdd(&a.pclk[10], (unsigned long long)Etot);  // (profiling: pool records)
  auto key_of = [&](unsigned long long rec) {
    return (((uint32_t)(rec >> (UB + BSF)) & 0xFFu) << 24) | ((uint32_t)rec & um);
  };
  __syncthreads();
  // 1. count per node; the first MV_GC records of each thread stay in registers (key, mask, node)
  uint32_t kc[MV_GC], mc[MV_GC], vc[MV_GC];
#pragma unroll
  for (uint32_t j = 0; j < MV_GC; ++j) {
    const uint32_t t = tid + j * MV_GT;
    kc[j] = 0; mc[j] = 0; vc[j] = 0xFFFFFFFFu;
    if (t < Etot) {
      const unsigned long long rec = pool[t];
      kc[j] = key_of(rec);
      mc[j] = (uint32_t)(rec >> MS);
      vc[j] = (uint32_t)(rec >> UB) & BPm;
    }
  }
#pragma unroll
  for (uint32_t j = 0; j < MV_GC; ++j)
    if (vc[j] != 0xFFFFFFFFu) atomicAdd(&cn[vc[j]], 1u);
  for (uint32_t t = tid + MV_GC * MV_GT; t < Etot; t += MV_GT) atomicAdd(&cn[(uint32_t)(pool[t] >> UB) & BPm], 1u);
  __syncthreads();
  const uint32_t E2 = mv_block_scan(cn, BP, ctl);
  if (tid == 0) cn[BP] = E2;
  __syncthreads();
  mark(12);
  // 2. node ranges whose records fit the LDS CSR (one range unless the bin is heavy); the
  // register-held records are placed in the first range only (they are dead afterwards:
  // later ranges re-read the pool), so they do not stay live across body
  auto range = [&](uint32_t lo) {
    if (tid == 0) {
      // the largest h with cn[h] - cn[lo] <= gcap (cn is non-decreasing): usually the whole bin
      uint32_t h = nv;
      if (cn[nv] - cn[lo] > gcap) {
        uint32_t l2 = lo, h2 = nv;  // cn[l2] - cn[lo] <= gcap < cn[h2] - cn[lo]
        while (h2 - l2 > 1) {
          const uint32_t mid = (l2 + h2) >> 1;
          if (cn[mid] - cn[lo] <= gcap) l2 = mid; else h2 = mid;
        }
        h = l2;
      }
      if (h == lo) { atomicOr(a.err, ERR_MV_CAP | ERR_MVD_CSR); h = nv; }  // one node beyond the LDS CSR
      ctl[15] = h;
      ctl[14] = 0;  // body's heavy-node count (k_mv_gather)
    }
    __syncthreads();
    const uint32_t hi = ctl[15];
    for (uint32_t i = lo + tid; i < hi; i += MV_GT) cur[i] = cn[i] - cn[lo];
    __syncthreads();
    return hi;
  };
  auto place_pool = [&](uint32_t lo, uint32_t hi, uint32_t t0) {
    for (uint32_t t = tid + t0; t < Etot; t += MV_GT) {
      const unsigned long long rec = pool[t];
      const uint32_t vl = (uint32_t)(rec >> UB) & BPm;
      if (vl < lo || vl >= hi) continue;
      const uint32_t p = atomicAdd(&cur[vl], 1u);
      if (p < gcap) {
        keys[p] = key_of(rec);
        msk[p] = (uint32_t)(rec >> MS);
      }
    }
    __syncthreads();
  };
  uint32_t hi = range(0);
#pragma unroll
  for (uint32_t j = 0; j < MV_GC; ++j) {
    const uint32_t vl = vc[j];
    if (vl >= hi) continue;  // (also the empty marker)
    const uint32_t p = atomicAdd(&cur[vl], 1u);
    if (p < gcap) { keys[p] = kc[j]; msk[p] = mc[j]; }
  }
  place_pool(0, hi, MV_GC * MV_GT);
  mark(13);
  body(0u, hi, 0u);
  __syncthreads();
  mark(11);
  for (uint32_t lo = hi; lo < nv; lo = hi) {
    hi = range(lo);
    place_pool(lo, hi, 0);
    mark(13);
    body(lo, hi, cn[lo]);
    __syncthreads();
    mark(11);
  }
}

__device__ inline MvCsr mv_csr_lds(unsigned char* smem, uint32_t BP, uint32_t gcap) {
  MvCsr L;
  L.cn = reinterpret_cast<uint32_t*>(smem);  // [BP + 1] records per node -> CSR starts
  L.cur = L.cn + BP + 1;                     // [BP + 1] placement cursors
  L.ctl = L.cur + BP + 1;                    // [16]
  L.sorg = L.ctl + 16;                       // [32]
  L.keys = L.sorg + 32;                      // [gcap] hop << 24 | src
  L.msk = L.keys + gcap;                     // [gcap] slot masks
  return L;
}

// Slot j's records of one node (list r0 .. r1 of the bin's CSR): the count c and the
// first 16 matches in list order in rk[0 .. min(c, 16)) (~0 beyond). A list of <= 64
// records is filtered to a bitmap (one LDS load and two ALU ops per record), then the
// matches are extracted in lockstep over the wave (t = 0, 1, ...: no per-lane register
// index); a longer list collects its matches record by record. All lanes of the wave
// must be active (the extraction bound is a wave maximum).
__device__ inline void mv_pair_records(const MvCsr& L, uint32_t r0, uint32_t r1, uint32_t j, uint32_t (&rk)[16],
                                       uint32_t& c) {
#pragma unroll
  for (int t = 0; t < 16; ++t) rk[t] = 0xFFFFFFFFu;
  const uint32_t Ln = r1 - r0;
  uint32_t blo = 0, bhi = 0;
  c = 0;
  if (Ln <= 64) {  // 4 independent LDS loads per step (the list is followed by >= 3 readable words)
    for (uint32_t k = 0; k < Ln; k += 4) {
      const uint32_t m0 = L.msk[r0 + k], m1 = L.msk[r0 + k + 1], m2 = L.msk[r0 + k + 2], m3 = L.msk[r0 + k + 3];
      const uint32_t b = ((m0 >> j) & 1u) | (((m1 >> j) & 1u) << 1) | (((m2 >> j) & 1u) << 2) | (((m3 >> j) & 1u) << 3);
      const uint32_t bm = Ln - k >= 4 ? b : b & ((1u << (Ln - k)) - 1);
      if (k < 32) blo |= bm << k; else bhi |= bm << (k - 32);
    }
    c = (uint32_t)(__popc(blo) + __popc(bhi));
  } else {
    for (uint32_t r = r0; r < r1; ++r) {
      if (!((L.msk[r] >> j) & 1u)) continue;
      const uint32_t key = L.keys[r];
#pragma unroll
      for (int t = 0; t < 16; ++t) rk[t] = c == (uint32_t)t ? key : rk[t];
      ++c;
    }
  }
  const uint32_t wx = active_max<5>(min(c, 16u));
#pragma unroll
  for (uint32_t t = 0; t < 16; ++t) {
    if (t >= wx) break;
    if (blo | bhi) {
      const uint32_t pos = blo ? (uint32_t)__builtin_ctz(blo) : 32u + (uint32_t)__builtin_ctz(bhi);
      if (blo) blo &= blo - 1; else bhi &= bhi - 1;
      rk[t] = L.keys[r0 + pos];
    }
  }
}

// The smallest hop among slot j's records of the node (rk holds them all when c <= 16).
__device__ inline uint32_t mv_pair_hop(const MvCsr& L, uint32_t r0, uint32_t r1, uint32_t j, const uint32_t (&rk)[16],
                                       uint32_t c) {
  uint32_t mh = 0xFFu;
  if (c <= 16) {
#pragma unroll
    for (int t = 0; t < 16; ++t) mh = min(mh, rk[t] >> 24);
  } else {
    for (uint32_t r = r0; r < r1; ++r)
      if ((L.msk[r] >> j) & 1u) mh = min(mh, L.keys[r] >> 24);
  }
  return mh;
}

// Per (slot, node) of the fine bin: in-degree, the inbound rows and the hop (the step
// API's gs_run_gossip, and gs_round unless GS_MV_FUSED=1). A lane holds its node's slot
// masks in registers, 32 records at a time, and per slot builds a 32-record bitmap from
// them (two ALU ops per record), then appends the slot's records in list order, one per
// set bit (round 4; before, every slot re-read and re-tested every record from LDS:
// ~21 instructions per (slot, record) for ~4.7 set bits per record at C5). Lanes hold
// consecutive nodes, so a slot's row t of every single-chunk node is stored by the same
// instruction.
// A node with more than MV_GH records (all slots) is deferred to a whole wave: stake
// weights make in-degrees power-law, and one such node in a wave of lanes held the
// other 63 lanes for its whole list (every slot). (256; 4 under GS_FLAG_NARROW_WAVE_PATH)
__global__ __launch_bounds__(MV_GT) void k_mv_gather(MvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // (local kept-bin index, in dispatch order: stakes fall with node id, so the low bins
  // hold the hubs' long lists; contiguous ranges per XCD left XCD 0 the heavy bins, C5's
  // gather 5.70 vs 4.41 ms per round)
  const uint32_t f = blockIdx.x;
  if (f >= a.fno) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, BP = 1u << a.BSF, Sg = a.Sg, v0 = (a.flo + f) << a.BSF;
  if (v0 >= a.vhi) return;
  const uint32_t nv = min(BP, a.vhi - v0), gcap = a.gcap;
  if (a.clear_vis)  // (the BFS is over and the gather does not read vis)
    for (uint32_t i = tid; i < nv; i += MV_GT) a.vis[v0 + i] = 0;
  const MvCsr L = mv_csr_lds(smem, BP, gcap);
  bool over = false;
  mv_bin_csr(a, f, nv, gcap, L, [&](uint32_t lo, uint32_t hi, uint32_t base) {
    const unsigned long long tb = a.pclk && tid == 0 ? wall_clock64() : 0;
    uint32_t* hvl = L.cur;  // the placement cursors are dead here: the heavy-node list
    for (uint32_t i = lo + tid; i < hi; i += MV_GT) {
      const uint32_t v = v0 + i, r0 = L.cn[i] - base, r1 = min(L.cn[i + 1] - base, gcap);
      if (r1 - r0 > a.gh) {
        hvl[atomicAdd(&L.ctl[14], 1u)] = i;
        continue;
      }
      const uint32_t vo = v - a.vlo;
      uint32_t A[32];  // slot masks of 32 records (>= 31 records of slack follow the CSR)
#pragma unroll
      for (int t = 0; t < 32; ++t) A[t] = L.msk[r0 + t];
      for (uint32_t j = 0; j < Sg; ++j) {
        uint32_t* __restrict__ row = a.inb + (size_t)(a.s0 + j) * a.NP + vo;
        uint32_t cc = 0, mh = 0xFFu;
        for (uint32_t rb = r0; rb < r1; rb += 32) {
          if (r1 - r0 > 32 && (rb != r0 || j)) {  // (nodes of more than one chunk)
#pragma unroll
            for (int t = 0; t < 32; ++t) A[t] = L.msk[rb + t];
          }
          uint32_t b = 0;
#pragma unroll
          for (int t = 0; t < 32; ++t) b |= ((A[t] >> j) & 1u) << t;
          if (r1 - rb < 32) b &= (1u << (r1 - rb)) - 1u;
          while (b) {  // four set bits per trip: four LDS loads, then their stores
            uint32_t k[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              ok[u] = b != 0;
              k[u] = L.keys[rb + (uint32_t)__builtin_ctz(b | 0x80000000u)];  // (b = 0: record 31, in the slack)
              b &= b - 1u;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (!ok[u]) break;
              if (cc < a.capin) row[(size_t)cc * a.PAIRS] = k[u];
              mh = min(mh, k[u] >> 24);
              ++cc;
            }
          }
        }
        const size_t p = (size_t)(a.s0 + j) * a.NP + vo;
        over |= cc > a.capin;
        a.cnt[p] = cc;
        a.hops[p] = (uint8_t)(v == L.sorg[j] ? 0u : (cc ? mh : 0xFFu));
      }
    }
    __syncthreads();
    const unsigned long long tl = a.pclk && tid == 0 ? wall_clock64() : 0;
    if (a.pclk && tid == 0) atomicAdd(&a.pclk[14], tl - tb);  // (phase clocks: the light nodes, [15] the heavy)
    // heavy nodes, one per wave: 64 records per step, each slot's ranks by ballot
    const uint32_t nh = L.ctl[14];
    for (uint32_t h = tid >> 6; h < nh; h += MV_GT / 64) {
      const uint32_t i = hvl[h];
      const uint32_t v = v0 + i, r0 = L.cn[i] - base, r1 = min(L.cn[i + 1] - base, gcap);
      for (uint32_t j = 0; j < Sg; ++j) {
        const size_t p = (size_t)(a.s0 + j) * a.NP + (v - a.vlo);
        uint32_t cc = 0, mh = 0xFFu;
        for (uint32_t rb = r0; rb < r1; rb += 64) {
          const uint32_t r = rb + lane;
          const bool b = r < r1 && ((L.msk[r] >> j) & 1u);
          const uint32_t k = b ? L.keys[r] : 0xFFFFFFFFu;
          const uint64_t bal = __ballot(b);
          const uint32_t pos =
              cc + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          if (b && pos < a.capin) a.inb[(size_t)pos * a.PAIRS + p] = k;
          mh = min(mh, k >> 24);
          cc += (uint32_t)__popcll(bal);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) mh = min(mh, (uint32_t)__shfl_xor((int)mh, off));
        if (lane == 0) {
          over |= cc > a.capin;
          a.cnt[p] = cc;
          a.hops[p] = (uint8_t)(v == L.sorg[j] ? 0u : (cc ? mh : 0xFFu));
        }
      }
    }
    if (a.pclk) {
      __syncthreads();
      if (tid == 0) atomicAdd(&a.pclk[15], wall_clock64() - tl);
    }
  });
  if (over) atomicOr(a.err, ERR_INBOUND);
}

// After a pair's consume: in-degree recorded, a due prune queued (k_cg_prune finds it by
// its meta word), else the previous round's pruned-len and prune count cleared.
__device__ inline void mv_after_consume(const MvArgs& a, uint32_t q, uint32_t meta, uint32_t c, uint32_t len,
                                        uint32_t up) {
  const bool due = up >= MIN_NUM_UPSERTS;
  const uint32_t nm = due ? (len | (up << 8) | (meta & 0xFF0000u)) : (len | (up << 8));
  if (nm != meta) a.cmeta[q] = nm;
  if (!due) a.prune_round[q] = 0;
  if (a.record && c) a.ingress_acc[q] += c;
}

// gs_round's gather + consume_messages (gossip.rs:601-607, 618-653): per (slot, node)
// of the fine bin, the pair's records are filtered from the node's LDS list straight
// into registers (the inbound rows are never written), then the received-cache update
// of gs_consume_dev.h; in-degree and hop as in k_mv_gather. Lanes walk nodes, so the
// cache rows stay coalesced. Pairs with in-degree > lane_c are taken by the whole wave
// (records compacted by ballot, sorted across lanes), > wave_c by one lane.
__global__ __launch_bounds__(MV_GT) __attribute__((amdgpu_waves_per_eu(4))) void k_mv_consume(MvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // (local kept-bin index, in dispatch order: stakes fall with node id, so the low bins
  // hold the hubs' long lists; contiguous ranges per XCD left XCD 0 the heavy bins, C5's
  // gather 5.70 vs 4.41 ms per round)
  const uint32_t f = blockIdx.x;
  if (f >= a.fno) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63, BP = 1u << a.BSF, Sg = a.Sg, v0 = (a.flo + f) << a.BSF;
  if (v0 >= a.vhi) return;
  const uint32_t nv = min(BP, a.vhi - v0), gcap = a.gcap_c;
  if (a.clear_vis)
    for (uint32_t i = tid; i < nv; i += MV_GT) a.vis[v0 + i] = 0;
  uint32_t* wscr = reinterpret_cast<uint32_t*>(smem) + (tid >> 6) * MV_WSCR;  // [64] keys, [CACHE_CAP] cache
  const MvCsr L = mv_csr_lds(smem + MV_CSCR, BP, gcap);
  const size_t PAIRS = a.PAIRS;
  uint32_t over = 0, errf = 0;
  mv_bin_csr(a, f, nv, gcap, L, [&](uint32_t lo, uint32_t hi, uint32_t base) {
    for (uint32_t i0 = lo; i0 < hi; i0 += MV_GT) {  // block-uniform trip count
      const uint32_t i = i0 + tid;
      const bool in = i < hi;
      const uint32_t v = v0 + i;
      const uint32_t r0 = in ? L.cn[i] - base : 0u, r1 = in ? min(L.cn[i + 1] - base, gcap) : 0u;
      for (uint32_t j = 0; j < Sg; ++j) {
        const uint32_t q = (a.s0 + j) * a.NP + (v - a.vlo);
        const uint32_t meta = in ? ntl(&a.cmeta[q]) : 0u;  // in flight during the filter
        uint32_t rk[16], c;
        mv_pair_records(L, r0, r1, j, rk, c);
        const uint32_t mh = mv_pair_hop(L, r0, r1, j, rk, c);
        if (in) {
          a.cnt[q] = c;
          a.hops[q] = (uint8_t)(v == L.sorg[j] ? 0u : (c ? mh : 0xFFu));
          if (c > a.capin) { over = 1; c = a.capin; }
        }
        uint32_t len = meta & 0xFF, up = (meta >> 8) & 0xFF;
        const bool heavy = in && c > a.lane_c;
        if (in && !heavy) {
          if (c) {
            const uint32_t wc = active_max<5>(c);
            uint32_t kc0[8];
            cache_prefetch(a.ckey, PAIRS, q, len, kc0);
            sort_ranked(rk, wc);
            cache_update_lane(a.ckey, PAIRS, q, rk, c, wc, kc0, len, up, errf);
          }
          mv_after_consume(a, q, meta, c, len, up);
        }
        uint64_t hv = __ballot(heavy);
        while (hv) {  // the wave's heavy pairs, one at a time
          const int hl = __ffsll((long long)hv) - 1;
          hv &= hv - 1;
          const uint32_t hq = (uint32_t)__shfl((int)q, hl);
          const uint32_t hmeta = (uint32_t)__shfl((int)meta, hl);
          const uint32_t hc = (uint32_t)__shfl((int)c, hl);
          const uint32_t h0 = (uint32_t)__shfl((int)r0, hl), h1 = (uint32_t)__shfl((int)r1, hl);
          uint32_t hlen = hmeta & 0xFF, hup = (hmeta >> 8) & 0xFF;
          if (hc <= a.wave_c) {
            uint32_t nb = 0;  // compact the pair's records into wscr[0..hc), then sort across lanes
            for (uint32_t rb = h0; rb < h1; rb += 64) {
              const uint32_t r = rb + lane;
              const bool m = r < h1 && ((L.msk[r] >> j) & 1u);
              const uint64_t bm = __ballot(m);
              const uint32_t pos = nb + (uint32_t)__popcll(bm & ((1ull << lane) - 1));
              if (m && pos < 64) wscr[pos] = L.keys[r];
              nb += (uint32_t)__popcll(bm);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const uint32_t key = wave_sort(lane < hc ? wscr[lane] : 0xFFFFFFFFu);
            __builtin_amdgcn_wave_barrier();
            cache_update_wave(a.ckey, PAIRS, hq, key, hc, hlen, hup, wscr + 64, errf);
          } else {
            cache_update_serial(a.ckey, PAIRS, hq, hc, hlen, hup, errf, [&](uint32_t k, uint32_t prev) {
              uint32_t best = 0xFFFFFFFFu;
              for (uint32_t r = h0; r < h1; ++r) {
                if (!((L.msk[r] >> j) & 1u)) continue;
                const uint32_t x = L.keys[r];
                if ((k == 0 || x > prev) && x < best) best = x;
              }
              return best;
            });
          }
          if (lane == 0) mv_after_consume(a, hq, hmeta, hc, hlen, hup);
        }
      }
    }
  });
  if (over) atomicOr(a.err, ERR_INBOUND);
  if (errf) atomicOr(a.err, errf);
}

// ------------------------------------------ frontier exchange (node-range partition) ----
// A frontier-exchange partition rank (GS_FLAG_FRONTIER_EXCHANGE) expands only the frontier
// entries of the nodes it owns; level d's push records (the expand runs, binned by coarse
// destination bin) go to the rank owning each bin, which applies them (k_mv_apply: first
// arrivals in its LDS copy of the bin's visited masks, pool records, its own next-level
// entries). Ranks own whole coarse bins, so a bin's records go to one rank.

// Records per coarse bin in level d's G expand runs (the T column of bin c).
// (G = ~0: level d's slices, from its size on the device -- the asynchronous level loop)
__device__ inline uint32_t mvx_slices(const MvArgs& a, uint32_t G, uint32_t d) {
  return G != 0xFFFFFFFFu ? G : min((a.lvl[d] + a.XT - 1) / a.XT, (uint32_t)a.rows_cap);
}

__global__ __launch_bounds__(256) void k_mvx_bincount(MvArgs a, uint32_t G, uint32_t d, uint32_t* __restrict__ bincnt) {
  __shared__ uint32_t part[4];
  const uint32_t c = blockIdx.x;
  G = mvx_slices(a, G, d);
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < G; i += 256) {
    s += mv_t(a, i, 2 + c) - mv_t(a, i, 1 + c);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bincnt[c] = part[0] + part[1] + part[2] + part[3];
}

// Bin c's segments of the G expand runs, copied contiguously (slice order) to out[rpos[c]..],
// and its record count to out[hpos[c]]: the header word of the owner's message.
// (rpos[c] = ~0: the owner's message outgrew its slot -- the header says 0 records)
__global__ __launch_bounds__(256) void k_mvx_pack(MvArgs a, uint32_t G, uint32_t d,
                                                  const unsigned long long* __restrict__ hpos,
                                                  const unsigned long long* __restrict__ rpos,
                                                  const uint32_t* __restrict__ bincnt,
                                                  unsigned long long* __restrict__ out) {
  __shared__ uint32_t pre[MV_SEG + 1], sb[MV_SEG], wsum[16];
  const uint32_t c = blockIdx.x, tid = threadIdx.x;
  G = mvx_slices(a, G, d);
  const bool skip = rpos[c] == ~0ull;
  if (tid == 0) out[hpos[c]] = skip ? 0u : bincnt[c];
  if (skip) return;
  size_t dst = rpos[c];
  for (uint32_t c0 = 0; c0 < G; c0 += MV_SEG) {
    const uint32_t gc = min(MV_SEG, G - c0);
    for (uint32_t i = tid; i < gc; i += 256) {
      const uint32_t st = mv_t(a, c0 + i, 1 + c);
      pre[i] = mv_t(a, c0 + i, 2 + c) - st;
      sb[i] = mv_t(a, c0 + i, 0) + st;
    }
    __syncthreads();
    const uint32_t ct = mv_block_scan(pre, gc, wsum);
    if (tid == 0) pre[gc] = ct;
    __syncthreads();
    for (uint32_t r = tid; r < ct; r += 256) {
      uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= r) lo = mid; else hi = mid;
      }
      out[dst + r] = a.area[sb[lo] + (r - pre[lo])];
    }
    dst += ct;
    __syncthreads();
  }
}

// T row q of a received level (bin-major with stride K, as mv_t): sender q's message (words
// off[q] ..) is nbm header words (record counts of this rank's bins blo, blo + 1, ...) then the
// records, bin by bin.
// (off = null: sender q's message starts at q * cap, the asynchronous loop's fixed slots)
__global__ __launch_bounds__(64) void k_mvx_trows(const unsigned long long* __restrict__ recv,
                                                  const unsigned long long* __restrict__ off, unsigned long long cap,
                                                  uint32_t blo, uint32_t nbm, uint32_t nbc, uint32_t K,
                                                  uint32_t* __restrict__ T) {
  const uint32_t q = blockIdx.x;
  const unsigned long long o = off ? off[q] : (unsigned long long)q * cap;
  for (uint32_t b = threadIdx.x; b < blo; b += 64) T[(size_t)(1 + b) * K + q] = 0;
  if (threadIdx.x == 0) {
    T[q] = (uint32_t)(o + nbm);
    uint32_t run = 0;
    for (uint32_t i = 0; i < nbm; ++i) {
      T[(size_t)(1 + blo + i) * K + q] = run;
      run += (uint32_t)recv[o + i];
    }
    for (uint32_t b = blo + nbm; b <= nbc; ++b) T[(size_t)(1 + b) * K + q] = run;
  }
}

// The asynchronous level loop's message layout (one thread per owner rank q): q's message
// goes to the fixed slot [q * cap, (q + 1) * cap) of the send buffer -- its bins' counts, then
// their records -- so no size has to reach the host before the all-to-all. xbin[2q], xbin[2q+1]:
// q's first coarse bin and bin count; wlog[q]: the message's words (the next round's
// capacity prediction). A message larger than its slot raises ERR_MVX_CAP and is sent as
// counts of 0 (the group's BFS is then redone with exact sizes).
__global__ void k_mvx_layout(uint32_t K, const uint32_t* __restrict__ xbin, const uint32_t* __restrict__ bincnt,
                             unsigned long long cap, unsigned long long* __restrict__ hpos,
                             unsigned long long* __restrict__ rpos, unsigned long long* __restrict__ wlog,
                             uint32_t* __restrict__ err) {
  for (uint32_t q = threadIdx.x; q < K; q += blockDim.x) {
    const uint32_t f = xbin[2 * q], nb = xbin[2 * q + 1];
    unsigned long long w = nb;
    for (uint32_t i = 0; i < nb; ++i) w += bincnt[f + i];
    wlog[q] = w;
    const bool over = w > cap;
    if (over) atomicOr(err, ERR_MVX_CAP);
    unsigned long long rp = (unsigned long long)q * cap + nb;
    for (uint32_t i = 0; i < nb; ++i) {
      hpos[f + i] = (unsigned long long)q * cap + i;  // (cap >= nb: the host sizes every slot so)
      rpos[f + i] = over ? ~0ull : rp;
      rp += bincnt[f + i];
    }
  }
}

// The group's origins owned by this rank: visited masks and level-0 entries (lvl was zeroed).
__global__ void k_mvx_seed(MvArgs a, const uint2* __restrict__ seeds, uint32_t nseed, uint2* __restrict__ q0) {
  const uint32_t i = threadIdx.x;
  if (i >= nseed) return;
  const uint2 sd = seeds[i];
  const uint32_t o = sd.x & 0xFFFFFFu;
  if (o - a.vlo >= a.vhi - a.vlo) return;
  a.vis[o] = sd.y;
  q0[atomicAdd(&a.lvl[0], 1u)] = sd;
}

// fcls[w] = smallest i (1-based) with frank[w] < T[i-1] over the ascending distinct
// failure counts T[0..m); 255 when w fails in no slot.
__global__ void k_mv_fcls(const uint32_t* __restrict__ frank, const uint32_t* __restrict__ T, uint32_t m, uint32_t N,
                          uint8_t* __restrict__ fcls) {
  for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w < N; w += gridDim.x * blockDim.x) {
    const uint32_t fr = frank[w];
    uint32_t lo = 0, hi = m;  // first i with T[i] > fr
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (T[mid] > fr) hi = mid; else lo = mid + 1;
    }
    fcls[w] = (uint8_t)(lo < m ? lo + 1 : 255);
  }
}

}  // namespace

// ------------------------------------------------------------------ host ----
// Fine bins with per-pair state: all, or a partition rank's (its range starts on a bin).
uint32_t mv_kept_bins(const Engine& e) {
  return (e.NP + (1u << e.mv.BSF) - 1) >> e.mv.BSF;
}

static uint32_t ceil_log2(size_t x) {
  uint32_t l = 0;
  while (((size_t)1 << l) < x) ++l;
  return l;
}

void mv_geometry(uint32_t N, uint32_t S, uint32_t ASZ, uint32_t ASZP, MvGeom& g) {
  (void)ASZP;
  g.UB = std::max(1u, ceil_log2(N));
  g.BSC = std::min(13u, std::max(6u, g.UB > 8 ? g.UB - 8 : 0u));   // ~256 coarse bins
  if (const char* x = std::getenv("GS_MV_BSC"))  // (tuning: at C5, 12 and 11 lose to 13)
    g.BSC = std::min(13u, std::max(6u, (uint32_t)std::strtoul(x, nullptr, 10)));
  g.BSF = std::min(g.BSC, 9u);  // fine bins of <= 512 nodes (gather at C4: 301 vs 412 us with 1,024)
  // (GS_MV_BSF: tuning; at most 10 so that a partition range of whole 1,024-id bins is whole fine bins)
  if (const char* x = std::getenv("GS_MV_BSF")) g.BSF = std::min(std::min(g.BSC, 10u), std::max(6u, (uint32_t)std::strtoul(x, nullptr, 10)));
  // apply keeps one LDS cursor per fine bin of its coarse bin: at most 16 (k_mv_apply's fcur)
  g.BSF = std::max(g.BSF, g.BSC > 4 ? g.BSC - 4 : 0u);
  g.nbc = (N + (1u << g.BSC) - 1) >> g.BSC;
  g.nbf = g.nbc << (g.BSC - g.BSF);
  // slot masks: area records (src | node-in-coarse-bin | mask) and pool records (src |
  // node-in-fine-bin | hop | mask, mv_pool_rec) are 64 bits
  g.GW = std::min(28u, std::min((64u - g.UB - g.BSC) & ~3u, (64u - g.UB - g.BSF - 8) & ~3u));
  g.TW = g.nbc + 2;
  const size_t sg = std::min<size_t>(S, g.GW);
  g.q_cap = (size_t)N * std::min<size_t>(sg, 26) + 64;
  g.XT = g.nbc >= MV_XT_WIDE && mv_hist_bytes(g.nbc) + (size_t)MV_XT_L * ASZP * 8 <= 160 * 1024 ? MV_XT_L : MV_XT;
  g.rows_cap = (g.q_cap + g.XT - 1) / g.XT + 1;
  g.area_cap = std::min<size_t>(g.rows_cap * g.XT * ASZ, 0xFFFFFFF0u);  // expand slice w's run at w * XT * ASZ
  const size_t rpn = (size_t)ASZ * std::min<size_t>(sg, 4) + 16;  // pool records per node (average over a bin)
  g.pcap = ((size_t)1 << g.BSF) * rpn;
  // (slack: k_mv_gather reads masks up to 31 records past a node's list, the fused
  // consume's filters up to 3)
  g.gcap = (uint32_t)((mv_glds() - mv_gather_fixed_bytes(g.BSF)) / 8) - 32;
  g.gcap_c = (uint32_t)((mv_glds() - MV_CSCR - mv_gather_fixed_bytes(g.BSF)) / 8) - 4;
}

bool mv_supported(const MvGeom& g, uint32_t ASZP) {
  return mv_hist_bytes(g.nbc) + (size_t)g.XT * ASZP * 8 <= 160 * 1024 && mv_apply_lds_bytes(g.BSC) <= 160 * 1024 &&
         g.GW >= 4;
}

// Host-side slot groups (contiguous ranges of <= GW slots) and their tables.
void mv_build_groups(Engine& e, const std::vector<uint32_t>& origins, const std::vector<uint8_t>& obkt,
                     const std::vector<uint8_t>& bucket, std::vector<uint32_t>& gtab, std::vector<uint2>& seeds) {
  const uint32_t GW = e.mv.GW;
  const uint32_t ng = (e.S + GW - 1) / GW;
  gtab.assign((size_t)ng * GT_STRIDE, 0);
  seeds.clear();
  e.mv_groups.clear();
  for (uint32_t g = 0; g < ng; ++g) {
    const uint32_t s0 = g * GW, sg = std::min(GW, e.S - s0);
    uint32_t* t = gtab.data() + (size_t)g * GT_STRIDE;
    {  // origin -> slot mask, open addressing with two probes (mv_origin_slots)
      uint32_t* ot = t + GT_OT;
      for (uint32_t i = 0; i < 128; ++i) ot[2 * i] = 0xFFFFFFFFu;
      bool ok = true;
      for (uint32_t j = 0; j < sg; ++j) {
        const uint32_t o = origins[s0 + j], h0 = mv_ohash(o), h1 = (h0 + 1) & 127u;
        const uint32_t h = (ot[2 * h0] == o || ot[2 * h0] == 0xFFFFFFFFu) ? h0
                           : (ot[2 * h1] == o || ot[2 * h1] == 0xFFFFFFFFu) ? h1 : 128u;
        if (h == 128u) { ok = false; continue; }
        ot[2 * h] = o;
        ot[2 * h + 1] |= 1u << j;
      }
      t[GT_OTOK] = ok ? 1u : 0u;
    }
    for (uint32_t k = 0; k < (uint32_t)NB; ++k)
      for (uint32_t j = 0; j < sg; ++j)
        if (obkt[s0 + j] >= k) t[GT_OWN + k] |= 1u << j;
    uint32_t nobs = 0;
    for (uint32_t j = 0; j < sg; ++j) {
      uint32_t i = 0;
      while (i < nobs && t[GT_OBV + i] != obkt[s0 + j]) ++i;
      if (i == nobs) { t[GT_OBV + i] = obkt[s0 + j]; ++nobs; }
      t[GT_OBM + i] |= 1u << j;
    }
    t[GT_NOBS] = nobs;
    const uint32_t seed0 = (uint32_t)seeds.size();
    for (uint32_t j = 0; j < sg; ++j) {  // one seed entry per distinct origin; its own entry
      const uint32_t org = origins[s0 + j];
      size_t i = seed0;
      while (i < seeds.size() && (seeds[i].x & 0xFFFFFFu) != org) ++i;
      if (i == seeds.size()) seeds.push_back(make_uint2(org | ((uint32_t)bucket[org] << 24), 0u));
      seeds[i].y |= 1u << j;
    }
    t[GT_NSEED] = (uint32_t)seeds.size() - seed0;
    t[GT_SEED] = seed0;
    t[GT_S0] = s0;
    t[GT_SG] = sg;
    e.mv_groups.push_back({s0, sg, seed0, t[GT_NSEED]});
  }
}

// After the failure counts change: per-slot failure classes and the per-node table.
hipError_t mv_update_failures(Engine& e, const std::vector<uint32_t>& nf) {
  if (!mv_layout(e)) return hipSuccess;
  std::vector<uint32_t> T;
  for (uint32_t x : nf)
    if (x) T.push_back(x);
  std::sort(T.begin(), T.end());
  T.erase(std::unique(T.begin(), T.end()), T.end());
  if (T.size() > 254) return hipErrorInvalidValue;
  std::vector<uint8_t> fk(e.S, 0);
  for (uint32_t o = 0; o < e.S; ++o)
    if (nf[o]) fk[o] = (uint8_t)(std::lower_bound(T.begin(), T.end(), nf[o]) - T.begin() + 1);
  hipError_t r;
  if ((r = hipMemcpyAsync(e.mv_fk, fk.data(), e.S, hipMemcpyHostToDevice, e.st))) return r;
  if (!T.empty()) {
    if ((r = hipMemcpyAsync(e.mv_thr, T.data(), T.size() * 4, hipMemcpyHostToDevice, e.st))) return r;
    hipLaunchKernelGGL(k_mv_fcls, dim3(std::min<uint32_t>((e.N + 255) / 256, 4096)), dim3(256), 0, e.st, e.frank,
                       e.mv_thr, (uint32_t)T.size(), e.N, e.mv_fcls);
    if ((r = launch_own_rows(e, nullptr, nullptr))) return r;  // the rows carry their peers' failure classes
  }
  return hipStreamSynchronize(e.st);  // fk and T are host temporaries
}

MvArgs mv_args(Engine& e, const MvGroup& gr, uint32_t g) {
  MvArgs a;
  a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.own = e.own; a.fcls = e.mv_fcls; a.fk = e.mv_fk;
  a.origin = e.origin; a.mask = e.mask; a.gt = e.mv_gtab + (size_t)g * GT_STRIDE;
  a.hops = e.hops; a.cnt = e.cnt; a.inb = e.inb; a.egress = e.egress; a.err = e.err;
  a.vis = e.mv_vis; a.lvl = e.lvl; a.hlvl = e.mv_hlvl_dev; a.T = e.mv_T; a.area = e.mv_area; a.ctr = e.mv_ctr;
  a.dpair = e.mv_dpair; a.hprof = nullptr; a.clear_vis = 0;
  a.pool = e.mv_pool; a.pused = e.mv_pused;
  a.N = e.N; a.SP = e.SP; a.ASZ = e.ASZ; a.fanout = e.fanout; a.capin = e.capin; a.s0 = gr.s0; a.Sg = gr.sg;
  a.UB = e.mv.UB; a.BSC = e.mv.BSC; a.BSF = e.mv.BSF; a.nbc = e.mv.nbc; a.nbf = e.mv.nbf; a.TW = e.mv.TW;
  a.TS = (uint32_t)e.mv.rows_cap;
  a.vlo = e.vlo; a.vhi = e.vlo + e.NP; a.NP = e.NP; a.MSU = (uint32_t)e.msu;
  a.XT = e.mv.XT;
  a.xrows = 0;
  a.small = MV_SMALL;  // the one-workgroup kernel's level bound
  if (const char* sm = std::getenv("GS_MV_SMALL")) a.small = (uint32_t)std::strtoul(sm, nullptr, 10);
  if (e.prm.flags & GS_FLAG_NO_SMALL_LEVELS) a.small = 0;  // every level through expand + apply
  a.flo = e.vlo >> e.mv.BSF; a.fno = mv_kept_bins(e);
  a.ORW = e.ORW;
  a.any_fail = 0;
  for (uint32_t j = 0; j < gr.sg; ++j) a.any_fail |= e.h_nfail_any[gr.s0 + j] ? 1u : 0u;
  a.gcap = e.mv.gcap;
  a.gcap_c = e.mv.gcap_c;
  a.cmeta = e.cmeta; a.ckey = e.ckey; a.prune_round = e.prune_round; a.ingress_acc = e.ingress_acc;
  const bool narrow = (e.prm.flags & GS_FLAG_NARROW_WAVE_PATH) != 0;  // small tests reach every consume path
  a.lane_c = narrow ? 4u : 16u;
  a.wave_c = narrow ? 8u : 64u;
  a.gh = narrow ? 4u : 256u;  // C4: 291 us with no wave path, 311 at 32
  if (const char* x = std::getenv("GS_MV_GH")) a.gh = std::min<uint32_t>(4096, (uint32_t)std::strtoul(x, nullptr, 10));
  a.pclk = e.phase_clk;
  a.record = 0;
  a.PAIRS = e.PAIRS; a.area_cap = e.mv.area_cap; a.rows_cap = e.mv.rows_cap; a.q_cap = e.mv.q_cap;
  a.pcap = e.mv.pcap;
  return a;
}

// Host-mapped words the level loop polls: PENDING until the kernel that writes them
// runs. The spin checks the stream now and then, so a stream that finished (or failed)
// without writing the word ends the wait instead of hanging it.
// The wait is bounded in wall-clock time (GS_LEVEL_WAIT_S, default 60 s): a kernel that
// never finishes its level (a device-side livelock) ends in hipErrorLaunchTimeOut, which the
// engine reports with the level, instead of spinning forever.
hipError_t mv_wait(volatile uint32_t* p, hipStream_t st, uint32_t& out) {
  static const double limit_s = [] {
    const char* x = std::getenv("GS_LEVEL_WAIT_S");
    const double v = x ? std::strtod(x, nullptr) : 0.0;
    return v > 0 ? v : 60.0;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t it = 1;; ++it) {
    const uint32_t x = *p;
    if (x != MV_PENDING) { out = x; return hipSuccess; }
    if ((it & 1023) == 0) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {
        out = *p;
        return out != MV_PENDING ? hipSuccess : hipErrorUnknown;
      }
      if (q != hipErrorNotReady) return q;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
        return hipErrorLaunchTimeOut;
    }
  }
}

hipError_t level_empty(Engine& e, uint32_t d, bool& empty) {
  uint32_t x = 0;
  hipError_t r = hipMemcpyAsync(&x, e.lvl + d, 4, hipMemcpyDeviceToHost, e.st);
  if (r == hipSuccess) r = hipStreamSynchronize(e.st);
  empty = x == 0;
  return r;
}

// One expand launch (slices of e.mv.XT entries).
static void launch_expand(Engine& e, const MvArgs& a, uint32_t d, uint32_t pi, size_t lds_x, uint32_t xgrid) {
  if (e.mv.XT == MV_XT_L) {
    GS_ASZP_DISPATCH_V(e.ASZP, hipLaunchKernelGGL((k_mv_expand<A, MV_XT_L>), dim3(xgrid), dim3(MV_XT_L), lds_x, e.st, a,
                                                  d, pi, e.mv_q[0], e.mv_q[1]));
  } else {
    GS_ASZP_DISPATCH_V(e.ASZP, hipLaunchKernelGGL((k_mv_expand<A, MV_XT>), dim3(xgrid), dim3(MV_XT), lds_x, e.st, a, d,
                                                  pi, e.mv_q[0], e.mv_q[1]));
  }
}

// The small-level kernel (one workgroup, k_mv_small).
static void launch_small_levels(Engine& e, const MvArgs& a, uint32_t mode, uint32_t d0, uint32_t pi,
                                const uint2* seeds, uint32_t nseed, uint32_t seq, size_t lds_s) {
  GS_ASZP_DISPATCH_V(e.ASZP, hipLaunchKernelGGL((k_mv_small<A>), dim3(1), dim3(MV_ST), lds_s, e.st, a, mode, d0, pi,
                                                e.mv_q[0], e.mv_q[1], e.mv_hstate_dev, seeds, nseed, seq));
}

// The level loop of one slot group. Two forms:
//  - predicted (the group has a level profile from an earlier round): everything is
//    enqueued at once and the host never waits -- the head kernel (seed + levels of at
//    most a.small entries), one expand/apply pair per level the profile had above the
//    tail threshold (each pair reads its level from dpair on the device, so a pair past
//    the BFS's end is a no-op), and the tail kernel, which finishes the BFS whatever is
//    left (and publishes this round's profile). Levels per round barely change between
//    rounds (the active sets rotate slowly), so the pairs fit.
//  - polled (no profile yet): the host enqueues level d after seeing level d - lag's size.
static hipError_t mv_group_polled(Engine& e, MvArgs& a, const MvGroup& gr, uint32_t lag, uint32_t& nlev) {
  hipError_t r;
  const size_t lds_x = mv_hist_bytes(e.mv.nbc) + (size_t)e.mv.XT * e.ASZP * 8;
  const size_t lds_a = mv_apply_lds_bytes(e.mv.BSC);
  const uint32_t fno = mv_kept_bins(e);
  const size_t lds_s = fno <= MV_SMALL_LP ? (size_t)fno * 4 : 0;
  const uint32_t agrid = ((e.mv.nbc + 7) / 8) * 8, xgrid = 2048;
  volatile uint32_t* hl = e.mv_hlvl;        // host-mapped: expand(d) writes lvl[d]
  volatile uint32_t* hs = e.mv_hlvl + 256;  // host-mapped: the small-level kernel's (level, entries)
  uint32_t d = 0;
  bool head = true;
  for (;;) {
    // small levels in one workgroup, until the frontier is empty or large
    hs[0] = MV_PENDING;
    launch_small_levels(e, a, head ? MV_HEAD : MV_POLL, d, 0u, e.mv_seed + gr.seed0, gr.nseed, 0u, lds_s);
    head = false;
    e.bfs_level = d;
    if ((r = mv_wait(hs, e.st, d))) return r;
    if (hs[1] == 0) { nlev = d; return hipSuccess; }
    if (d >= 254) return hipErrorNotSupported;  // frontier still non-empty after 254 levels
    // large levels: expand + apply; the frontier size of level x is polled `lag` levels late
    const uint32_t dl = d;
    for (;; ++d) {
      if (d >= 254) {  // levels through 253 enqueued: the hops fit u8 iff level 254 is empty
        bool empty = false;
        if ((r = level_empty(e, 254, empty))) return r;
        if (!empty) return hipErrorNotSupported;
        nlev = d;
        return hipSuccess;
      }
      hl[d] = MV_PENDING;
      launch_expand(e, a, d, MV_NOPAIR, lds_x, xgrid);
      hipLaunchKernelGGL(k_mv_apply, dim3(agrid), dim3(MV_AT), lds_a, e.st, a, d, MV_NOPAIR, e.mv_q[0], e.mv_q[1]);
      if (d >= dl + lag) {
        uint32_t x = 0;
        e.bfs_level = d - lag;
        if ((r = mv_wait(hl + (d - lag), e.st, x))) return r;
        if (x == 0) { nlev = d + 1; return hipSuccess; }
        if (x <= a.small) { ++d; break; }  // levels d - 1, d are enqueued; small levels from d + 1
      }
    }
  }
}

// Dynamic-LDS limits of the level kernels (once per engine) and the persistent kernel's grid.
static hipError_t mv_attrs(Engine& e) {
  hipError_t r = hipSuccess;
  const size_t lds_x = mv_hist_bytes(e.mv.nbc) + (size_t)e.mv.XT * e.ASZP * 8;
  const size_t lds_a = mv_apply_lds_bytes(e.mv.BSC);
  const size_t lds_g = mv_glds();
  const uint32_t fno = mv_kept_bins(e);
  const size_t lds_s = fno <= MV_SMALL_LP ? (size_t)fno * 4 : 0;
  if (!e.mv_attr_set) {
    GS_ASZP_DISPATCH(e.ASZP, {
      r = e.mv.XT == MV_XT_L
              ? hipFuncSetAttribute((const void*)k_mv_expand<A, MV_XT_L>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds_x)
              : hipFuncSetAttribute((const void*)k_mv_expand<A, MV_XT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds_x);
    });
    if (r != hipSuccess) return r;
    if ((r = hipFuncSetAttribute((const void*)k_mv_apply, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a)))
      return r;
    if ((r = hipFuncSetAttribute((const void*)k_mv_gather, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g)))
      return r;
    if ((r = hipFuncSetAttribute((const void*)k_mv_consume, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g)))
      return r;
    GS_ASZP_DISPATCH(e.ASZP, {
      r = hipFuncSetAttribute((const void*)k_mv_small<A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_s);
    });
    if (r != hipSuccess) return r;
    e.mv_attr_set = true;
  }
  return r;
}

hipError_t launch_bfs_multi(Engine& e, bool record, bool consume) {
  hipError_t r = hipSuccess;
  const size_t lds_x = mv_hist_bytes(e.mv.nbc) + (size_t)e.mv.XT * e.ASZP * 8;
  const size_t lds_a = mv_apply_lds_bytes(e.mv.BSC);
  const size_t lds_g = mv_glds();
  const uint32_t fno = mv_kept_bins(e);
  const size_t lds_s = fno <= MV_SMALL_LP ? (size_t)fno * 4 : 0;
  if ((r = mv_attrs(e))) return r;
  const uint32_t agrid = ((e.mv.nbc + 7) / 8) * 8;
  const uint32_t ggrid = fno;
  const uint32_t xgrid = 2048;
  uint32_t lag = 2;
  if (const char* x = std::getenv("GS_MV_LAG")) lag = std::max<uint32_t>(1, (uint32_t)std::strtoul(x, nullptr, 10));
  static const bool polled_only = std::getenv("GS_MV_POLLED") && std::getenv("GS_MV_POLLED")[0] == '1';
  static const uint32_t tail_env = [] {  // levels the profile had at or below this run in the tail kernel
    const char* x = std::getenv("GS_MV_TAIL");
    return x ? (uint32_t)std::strtoul(x, nullptr, 10) : 0xFFFFFFFFu;
  }();
  for (uint32_t g = 0; g < (uint32_t)e.mv_groups.size(); ++g) {
    const MvGroup& gr = e.mv_groups[g];
    MvArgs a = mv_args(e, gr, g);
    a.record = record ? 1u : 0u;
    uint32_t* hp = e.mv_prof + (size_t)g * MV_PROF_WORDS;
    a.hprof = e.mv_prof_dev + (size_t)g * MV_PROF_WORDS;
    {  // the newest published profile of this group (a tail kernel of an earlier round)
      volatile uint32_t* vp = hp;
      const uint32_t sq = vp[0];
      if (sq != e.mv_prof_seen[g] && sq != 0) {
        std::atomic_thread_fence(std::memory_order_acquire);
        const uint32_t nl = std::min<uint32_t>((uint32_t)vp[1], 255u);
        std::vector<uint32_t> pv(nl);
        for (uint32_t k = 0; k < nl; ++k) pv[k] = vp[2 + k];
        std::atomic_thread_fence(std::memory_order_acquire);
        if (vp[0] == sq) {  // (not rewritten meanwhile: a rewrite sets 0 first, then a new seq)
          e.mv_pred[g] = std::move(pv);
          e.mv_prof_seen[g] = sq;
        }
      }
    }
    hipEvent_t t0;
    e.tbegin("bfs", &t0);
    // the persistent BFS (gs_bfs_pers.hip) keeps the visited masks in LDS: vis stays as it is
    const bool pers = pb_usable(e) && !e.mv_diag;
    if (!pers && !e.mv_vis_clean && (r = hipMemsetAsync(e.mv_vis, 0, (size_t)e.N * 4, e.st))) return r;
    if (!pers) e.mv_vis_clean = false;
    uint32_t nlev = 254;  // (the gather reads the levels' sizes; empty levels end the BFS)
    const std::vector<uint32_t>& pv = e.mv_pred[g];
    if (pers) {
      if ((r = launch_bfs_pers(e, a, gr))) return r;
    } else if (pv.empty() || polled_only || e.mv_diag) {
      if ((r = mv_group_polled(e, a, gr, lag, nlev))) return r;
      if (!polled_only) {  // this round's sizes seed the prediction
        // (levels enqueued after the one that ended the BFS may not have run yet: PENDING = 0)
        std::vector<uint32_t> p2(nlev);
        for (uint32_t k = 0; k < nlev; ++k) {
          const uint32_t x = e.mv_hlvl[k];
          p2[k] = x == MV_PENDING ? 0u : x;
        }
        while (!p2.empty() && p2.back() == 0) p2.pop_back();
        e.mv_pred[g] = std::move(p2);
      }
    } else {
      // the head kernel stops at the first level above a.small; pairs then take the levels
      // the profile had above the tail threshold
      const uint32_t tail_thr = tail_env != 0xFFFFFFFFu ? tail_env : 2048u;
      uint32_t k0 = 0;
      while (k0 < pv.size() && pv[k0] <= a.small) ++k0;
      uint32_t k1 = (uint32_t)pv.size();  // one past the last level above the tail threshold
      while (k1 > k0 && pv[k1 - 1] <= tail_thr) --k1;
      const uint32_t npairs = std::min<uint32_t>(k1 - k0 + mv_margin(), 250);
      launch_small_levels(e, a, MV_HEAD, 0u, 0u, e.mv_seed + gr.seed0, gr.nseed, 0u, lds_s);
      static const bool full_grid = std::getenv("GS_MV_XGRID_FULL") && std::getenv("GS_MV_XGRID_FULL")[0] == '1';
      for (uint32_t i = 0; i < npairs; ++i) {
        // the pair's expand grid from the predicted level (+25 %; slices beyond it are taken by
        // the grid-stride loop): small levels launch a few workgroups instead of 2,048
        const uint32_t pl = k0 + i < pv.size() ? pv[k0 + i] : 0u;
        const uint32_t gp = (uint32_t)(((size_t)pl + e.mv.XT - 1) / e.mv.XT);
        const uint32_t xg = full_grid ? xgrid : std::min<uint32_t>(xgrid, std::max<uint32_t>(16, gp + gp / 4 + 8));
        launch_expand(e, a, 0u, i, lds_x, xg);
        hipLaunchKernelGGL(k_mv_apply, dim3(agrid), dim3(MV_AT), lds_a, e.st, a, 0u, i, e.mv_q[0], e.mv_q[1]);
      }
      const uint32_t seq = ++e.mv_seq ? e.mv_seq : ++e.mv_seq;  // (never 0)
      launch_small_levels(e, a, MV_TAIL, 0u, npairs, nullptr, 0u, seq, lds_s);
    }
    e.tend("bfs", t0);
    e.tbegin(consume ? "gather_consume" : "gather", &t0);
    // an unpartitioned engine's fine bins cover every node: the gather leaves vis zeroed
    // for the next BFS (one memset launch less per group and round)
    a.clear_vis = e.part_on || pers ? 0u : 1u;
    if (consume) hipLaunchKernelGGL(k_mv_consume, dim3(ggrid), dim3(MV_GT), lds_g, e.st, a);
    else hipLaunchKernelGGL(k_mv_gather, dim3(ggrid), dim3(MV_GT), lds_g, e.st, a);
    if (!pers) e.mv_vis_clean = a.clear_vis != 0;
    e.tend(consume ? "gather_consume" : "gather", t0);
    if (e.mv_diag) {  // GS_MV_DIAG=1: entries and records of the group's BFS (diagnostics)
      std::vector<uint32_t> pu(fno);
      if ((r = hipMemcpyAsync(pu.data(), e.mv_pused, pu.size() * 4, hipMemcpyDeviceToHost, e.st))) return r;
      if ((r = hipStreamSynchronize(e.st))) return r;
      volatile uint32_t* hl = e.mv_hlvl;
      size_t ent = 0, rec = 0, mx = 0;
      for (uint32_t d = 0; d < nlev; ++d) ent += hl[d];
      for (uint32_t x : pu) { rec += x; mx = std::max<size_t>(mx, x); }
      std::fprintf(stderr, "GS_MV_DIAG group %u: levels %u, entries %zu, records %zu (max %zu per fine bin)\n", g,
                   nlev, ent, rec, mx);
      std::fprintf(stderr, "GS_MV_DIAG levels (entries):");
      for (uint32_t d = 0; d < nlev; ++d) std::fprintf(stderr, " %u", hl[d]);
      std::fprintf(stderr, "\n");
    }
  }
  return hipGetLastError();
}

// ------------------------------------------ frontier exchange: host side ----
// The owner of coarse bin c, and rank q's first bin and bin count (ranks own whole bins).
static uint32_t mvx_owner(const Engine& e, uint32_t c) {
  return (uint32_t)(((size_t)c << e.mv.BSC) / e.part_C);
}
static void mvx_bins(const Engine& e, uint32_t q, uint32_t& first, uint32_t& nb) {
  const size_t lo = std::min<size_t>(e.N, (size_t)q * e.part_C), hi = std::min<size_t>(e.N, lo + e.part_C);
  first = (uint32_t)(lo >> e.mv.BSC);
  nb = (uint32_t)(((hi + (1u << e.mv.BSC) - 1) >> e.mv.BSC) - first);
  if (hi <= lo) nb = 0;
}

hipError_t mvx_begin(Engine& e, uint32_t g, uint32_t& n_local) {
  hipError_t r;
  if ((r = mv_attrs(e))) return r;
  const MvGroup& gr = e.mv_groups[g];
  MvArgs a = mv_args(e, gr, g);
  if ((r = hipMemsetAsync(e.mv_vis, 0, (size_t)e.N * 4, e.st))) return r;
  if ((r = hipMemsetAsync(e.lvl, 0, 256 * 4, e.st))) return r;
  if ((r = hipMemsetAsync(e.mv_pused, 0, (size_t)mv_kept_bins(e) * 4, e.st))) return r;
  if (gr.nseed > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_mvx_seed, dim3(1), dim3(1024), 0, e.st, a, e.mv_seed + gr.seed0, gr.nseed, e.mv_q[0]);
  if ((r = hipMemcpyAsync(e.h_err + 1, e.lvl, 4, hipMemcpyDeviceToHost, e.st))) return r;
  if ((r = hipStreamSynchronize(e.st))) return r;
  n_local = e.h_err[1];
  return hipGetLastError();
}

hipError_t mvx_expand(Engine& e, uint32_t g, uint32_t d, uint32_t n_local, std::vector<uint64_t>& words_to) {
  hipError_t r;
  MvArgs a = mv_args(e, e.mv_groups[g], g);
  const uint32_t nbc = e.mv.nbc, K = e.part_K;
  const uint32_t G = (n_local + e.mv.XT - 1) / e.mv.XT;
  if ((size_t)n_local > e.mv.q_cap || G > e.mv.rows_cap) return hipErrorInvalidValue;
  std::vector<uint32_t> cnt(nbc, 0);
  if (G) {
    const size_t lds_x = mv_hist_bytes(nbc) + (size_t)e.mv.XT * e.ASZP * 8;
    launch_expand(e, a, d, MV_NOPAIR, lds_x, std::min<uint32_t>(G, 2048));
    hipLaunchKernelGGL(k_mvx_bincount, dim3(nbc), dim3(256), 0, e.st, a, G, d, e.x_bincnt);
    if ((r = hipMemcpyAsync(cnt.data(), e.x_bincnt, nbc * 4, hipMemcpyDeviceToHost, e.st))) return r;
    if ((r = hipStreamSynchronize(e.st))) return r;
  } else {
    if ((r = hipMemsetAsync(e.x_bincnt, 0, nbc * 4, e.st))) return r;
  }
  // message to rank q: the counts of q's bins (one u64 word each), then their records in bin order
  std::vector<unsigned long long> pos(2 * (size_t)nbc);
  words_to.assign(K, 0);
  std::vector<uint64_t> start(K + 1, 0);
  for (uint32_t q = 0; q < K; ++q) {
    uint32_t f, nb;
    mvx_bins(e, q, f, nb);
    uint64_t w = nb;
    for (uint32_t i = 0; i < nb; ++i) w += cnt[f + i];
    words_to[q] = w;
    start[q + 1] = start[q] + w;
  }
  if (start[K] > e.x_send_cap) return hipErrorInvalidValue;
  for (uint32_t q = 0; q < K; ++q) {
    uint32_t f, nb;
    mvx_bins(e, q, f, nb);
    uint64_t rp = start[q] + nb;
    for (uint32_t i = 0; i < nb; ++i) {
      pos[f + i] = start[q] + i;       // header word
      pos[nbc + f + i] = rp;           // records
      rp += cnt[f + i];
    }
  }
  if ((r = hipMemcpyAsync(e.x_pos, pos.data(), pos.size() * 8, hipMemcpyHostToDevice, e.st))) return r;
  hipLaunchKernelGGL(k_mvx_pack, dim3(nbc), dim3(256), 0, e.st, a, G, d, e.x_pos, e.x_pos + nbc, e.x_bincnt, e.x_send);
  e.x_send_words = start[K];
  if ((r = hipStreamSynchronize(e.st))) return r;  // (pos is a host temporary)
  return hipGetLastError();
}

hipError_t mvx_apply(Engine& e, uint32_t g, uint32_t d, const unsigned long long* recv,
                     const std::vector<uint64_t>& words_from, uint32_t& n_next) {
  hipError_t r;
  MvArgs a = mv_args(e, e.mv_groups[g], g);
  const uint32_t K = e.part_K;
  std::vector<unsigned long long> off(K + 1, 0);
  for (uint32_t q = 0; q < K; ++q) off[q + 1] = off[q] + words_from[q];
  if (off[K] > 0xFFFFFFF0ull) return hipErrorInvalidValue;  // (T rows hold u32 record places)
  uint32_t blo, nbm;
  mvx_bins(e, e.part_rank, blo, nbm);
  if ((r = hipMemcpyAsync(e.x_off, off.data(), (K + 1) * 8, hipMemcpyHostToDevice, e.st))) return r;
  hipLaunchKernelGGL(k_mvx_trows, dim3(K), dim3(64), 0, e.st, recv, e.x_off, 0ull, blo, nbm, e.mv.nbc, K, e.x_T);
  a.T = e.x_T;
  a.TS = K;
  a.area = const_cast<unsigned long long*>(recv);
  a.xrows = K;
  const size_t lds_a = mv_apply_lds_bytes(e.mv.BSC);
  const uint32_t agrid = ((e.mv.nbc + 7) / 8) * 8;
  hipLaunchKernelGGL(k_mv_apply, dim3(agrid), dim3(MV_AT), lds_a, e.st, a, d, MV_NOPAIR, e.mv_q[0], e.mv_q[1]);
  if ((r = hipMemcpyAsync(e.h_err + 1, e.lvl + d + 1, 4, hipMemcpyDeviceToHost, e.st))) return r;
  if ((r = hipStreamSynchronize(e.st))) return r;
  n_next = e.h_err[1];
  return hipGetLastError();
}

// ---------------------------------- frontier exchange, asynchronous level loop ----
// Level d without a host wait: expand (its grid-stride loop reads the level size on the
// device), per-bin counts, the fixed-slot layout and the pack into `send` (K slots of `cap`
// words). The all-to-all that follows moves equal slots, so the host needs no size.
hipError_t mvx_expand_async(Engine& e, uint32_t g, uint32_t d, unsigned long long cap, unsigned long long* send) {
  MvArgs a = mv_args(e, e.mv_groups[g], g);
  const uint32_t nbc = e.mv.nbc, K = e.part_K;
  const size_t lds_x = mv_hist_bytes(nbc) + (size_t)e.mv.XT * e.ASZP * 8;
  launch_expand(e, a, d, MV_NOPAIR, lds_x, 2048);
  hipLaunchKernelGGL(k_mvx_bincount, dim3(nbc), dim3(256), 0, e.st, a, 0xFFFFFFFFu, d, e.x_bincnt);
  hipLaunchKernelGGL(k_mvx_layout, dim3(1), dim3(64), 0, e.st, K, e.x_bins, e.x_bincnt, cap, e.x_pos, e.x_pos + nbc,
                     e.x_wlog + (size_t)d * K, e.err);
  hipLaunchKernelGGL(k_mvx_pack, dim3(nbc), dim3(256), 0, e.st, a, 0xFFFFFFFFu, d, e.x_pos, e.x_pos + nbc, e.x_bincnt,
                     send);
  return hipGetLastError();
}

// Level d's apply of what every rank sent (K slots of `cap` words in `recv`): T rows from the
// slots' headers, then k_mv_apply; the next level's own entries count stays on the device.
hipError_t mvx_apply_async(Engine& e, uint32_t g, uint32_t d, const unsigned long long* recv, unsigned long long cap) {
  MvArgs a = mv_args(e, e.mv_groups[g], g);
  const uint32_t K = e.part_K;
  uint32_t blo, nbm;
  mvx_bins(e, e.part_rank, blo, nbm);
  hipLaunchKernelGGL(k_mvx_trows, dim3(K), dim3(64), 0, e.st, recv, nullptr, cap, blo, nbm, e.mv.nbc, K, e.x_T);
  a.T = e.x_T;
  a.TS = K;
  a.area = const_cast<unsigned long long*>(recv);
  a.xrows = K;
  const size_t lds_a = mv_apply_lds_bytes(e.mv.BSC);
  const uint32_t agrid = ((e.mv.nbc + 7) / 8) * 8;
  hipLaunchKernelGGL(k_mv_apply, dim3(agrid), dim3(MV_AT), lds_a, e.st, a, d, MV_NOPAIR, e.mv_q[0], e.mv_q[1]);
  return hipGetLastError();
}

// Every rank's first coarse bin and bin count (k_mvx_layout's xbin), once per engine.
hipError_t mvx_upload_bins(Engine& e) {
  std::vector<uint32_t> xb(2 * (size_t)e.part_K);
  for (uint32_t q = 0; q < e.part_K; ++q) mvx_bins(e, q, xb[2 * q], xb[2 * q + 1]);
  hipError_t r = hipMemcpyAsync(e.x_bins, xb.data(), xb.size() * 4, hipMemcpyHostToDevice, e.st);
  if (r == hipSuccess) r = hipStreamSynchronize(e.st);  // (xb is a host temporary)
  return r;
}

// After the group's last level: gather + consume of its own nodes straight from the LDS CSR
// (k_mv_consume, as the replicated partition's round; no inbound rows are written).
hipError_t mvx_gather_consume(Engine& e, uint32_t g, bool record) {
  MvArgs a = mv_args(e, e.mv_groups[g], g);
  a.record = record ? 1u : 0u;
  // as gs_round: the gather's inbound rows, consumed by k_cg_consume at gs_part_xround_finish
  // (GS_MV_FUSED=1: fused gather + consume here; at C5 14.2 vs ~10 ms per round)
  if (e.mv_fused) hipLaunchKernelGGL(k_mv_consume, dim3(mv_kept_bins(e)), dim3(MV_GT), mv_glds(), e.st, a);
  else hipLaunchKernelGGL(k_mv_gather, dim3(mv_kept_bins(e)), dim3(MV_GT), mv_glds(), e.st, a);
  return hipGetLastError();
}

}  // namespace gs
