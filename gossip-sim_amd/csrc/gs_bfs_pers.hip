// gs_bfs_pers.hip -- the multi-source frontier BFS (Cluster::run_gossip, gossip.rs:494-615;
// gs_bfs_multi.hip) as ONE persistent launch per slot group, levels separated by grid
// barriers instead of kernel boundaries (round 6).
//
// Why: the launched level loop (head kernel, one expand + apply pair per level, tail
// kernel) pays ~15-30 us per level however small the level is -- two launches, a global
// frontier queue written by apply and read back by expand, a T-row walk, device-scope
// atomics on the visited masks -- and C4's BFS has 19 levels.
//
// Owner-computes: workgroup g of G (one per CU, G a power of two) owns the fine bins
// {g, g + G, g + 2G, ...} (2^BSF nodes each: interleaved, so the hub-heavy low ids spread
// over every workgroup). It keeps its nodes' visited slot masks in LDS for the whole BFS,
// appends the records pushed to its nodes to their fine bins' pools, and expands the
// frontier entries of its own nodes. Per level L (the entries whose slots first reached
// their node at hop L):
//   expand   each workgroup expands its level-L entries (mv_expand_entry: first `fanout`
//            unpruned non-origin ring slots per slot, failed peers burn a slot,
//            push_active_set.rs:128-141, gossip.rs:527-541) in chunks of CH entries; a
//            chunk takes a slice number from the level's counter, ranks its records by
//            destination workgroup in LDS and writes them as one contiguous run at the
//            slice's fixed place, with a T row (run base, per-destination starts, total);
//   barrier  (every slice of level L is written and drained; sc1 stores, sc1 loads:
//            cdna_hip_programming.md Guideline 16's write-through form, no fences);
//   receive  each workgroup walks its T column over the level's slices and ORs every
//            record's slot mask into its LDS masks -- new bits are first arrivals at hop
//            L + 1 (gossip.rs:594-600) -- and appends the record, stamped with hop L + 1,
//            to its fine bin's pool (the layout k_mv_gather reads);
//   entries  new bits of its nodes become level-(L + 1) entries (one per distinct entry
//            k, mv_parts), in node order, kept in LDS (overflow: the workgroup's global
//            region).
// The BFS ends at the first level with no slices anywhere (a grid-uniform count). Results
// equal the launched loop's bit for bit: the same entries, records, pools and egress.
#include <fcntl.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>

#include "gs_device.h"
#include "gs_internal.h"
#include "gs_mv_dev.h"

namespace gs {

namespace {

constexpr uint32_t PB_T = 1024;   // threads per workgroup (one workgroup per CU)
constexpr uint32_t PB_SEG = 1024; // T-column slices per receive batch
constexpr uint32_t PB_EC = 1024;  // level entries kept in LDS (beyond: the workgroup's global region)
// control block (pb_blk): barrier shard counters at 64 s (s < 8), top counter 512,
// generation 576; the slice counter of level L at 1024 + L. Zeroed before every launch.
constexpr uint32_t PB_BLK_WORDS = 1280;
// dynamic LDS header: the group's slots (MvSlots), its table (GT_WORDS), 16 control words
constexpr uint32_t PB_HDR_SLOTS = (uint32_t)((sizeof(MvSlots) + 15) & ~(size_t)15);
constexpr uint32_t PB_HDR = PB_HDR_SLOTS + 4 * GT_WORDS + 64;

struct PbArgs {
  MvArgs a;
  const uint2* seeds;
  uint32_t nseed;
  uint32_t G, GL;         // workgroups (= 1 << GL)
  uint32_t FPW, LB;       // fine bins per workgroup (power of two), local node index bits
  uint32_t CH;            // entries per expand chunk (slice)
  uint32_t stage_bytes;   // LDS bytes of the stage region (>= CH * ASZ records and the receive's T column)
  uint32_t rows_cap;      // slices per level at most
  uint32_t TS;            // T: rows_cap (bin-major, entry b of slice w at b * TS + w)
  uint32_t* T[2];         // per level parity: [G + 2][TS]
  unsigned long long* area[2];  // per level parity: slice w's run at w * CH * ASZ
  size_t area_cap;
  uint32_t* blk;          // control block
  uint2* gq;              // [G][gq_cap] level entries beyond PB_EC
  uint32_t gq_cap;
  unsigned long long* tr; // GS_PB_TRACE: per level [16]: WG 0's expand start, max expand / barrier /
                          // receive / entries durations over workgroups, entries, records
};

__device__ inline void st_agent32(uint32_t* p, uint32_t x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agent64(unsigned long long* p, unsigned long long x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline uint32_t ld_agent32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long ld_agent64(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid barrier (counter form, sharded by blockIdx & 7; every counter on a 256-B line of its
// own: the pollers' loads do not contend with the arrivals): every wave drains its stores
// (write-through sc1 stores and device-scope atomics: s_waitcnt vmcnt(0)) before the
// workgroup barrier, thread 0 arrives on its shard, the last of a shard on the top
// counter, the last shard publishes generation e; thread 0 polls it relaxed. The block is
// zeroed before every launch, so epochs start at 1. A spin is bounded (~1 s): on expiry
// ERR_SYNC is raised and the workgroup goes on (the engine is then refused).
constexpr uint32_t PB_BAR_STR = 64, PB_BAR_TOP = 8 * PB_BAR_STR, PB_BAR_GEN = 9 * PB_BAR_STR, PB_SLICES = 1024;
__device__ inline void pb_grid_sync(uint32_t* bar, uint32_t e, uint32_t G, uint32_t* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t sh = blockIdx.x & 7u, ns = min(G, 8u), cs = (G - sh + 7u) / 8u;
    const uint32_t r = __hip_atomic_fetch_add(&bar[PB_BAR_STR * sh], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r + 1u == e * cs) {
      const uint32_t t = __hip_atomic_fetch_add(&bar[PB_BAR_TOP], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t + 1u == e * ns) __hip_atomic_store(&bar[PB_BAR_GEN], e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (uint32_t it = 0; __hip_atomic_load(&bar[PB_BAR_GEN], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e; ++it) {
      if (it > (1u << 22)) {
        atomicOr(err, ERR_SYNC);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// mv_block_scan with LDS-only barriers: global stores in flight (T rows, records, egress)
// are not waited for -- the grid barrier drains them once per level.
__device__ inline uint32_t pb_block_scan(uint32_t* h, uint32_t n, uint32_t* wsum) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = PB_T >> 6;
  const uint32_t per = (n + PB_T - 1) / PB_T;
  const uint32_t lo = min(n, tid * per), hi = min(n, lo + per);
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += h[i];
  const uint32_t incl = wave_incl_scan(s);
  if (lane == 63) wsum[wid] = incl;
  lds_barrier();
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
  lds_barrier();
  return tot;
}

__device__ inline void st_entry(uint2* p, uint2 x) {  // (sc1: read back by other waves of the workgroup)
  st_agent64(reinterpret_cast<unsigned long long*>(p), (unsigned long long)x.x | ((unsigned long long)x.y << 32));
}
__device__ inline uint2 ld_entry(const uint2* p) {
  const unsigned long long v = ld_agent64(reinterpret_cast<const unsigned long long*>(p));
  return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}

// One frontier entry per LW lanes (lane j of the group: slot j), for a workgroup's levels of
// at most PB_T / LW entries: the slots' selections run side by side instead of one after
// another in one lane (a 13-slot entry was a ~6-9 us VALU chain of one lane, and C4's first
// levels hold 1-36 entries per workgroup). Per slot the selection of mv_expand_entry:
// taken_slots (push_active_set.rs:128-141: the first `fanout` unpruned non-origin ring
// slots in FIFO order), then failed peers burn their slot (gossip.rs:527-541); the slot's
// egress byte. Lane j < ASZP returns ring slot j's record (its peer and the slots that push
// to it) in row[0] / acc[0].
template <int ASZP, uint32_t LW>
__device__ inline void pb_expand_wide(const MvArgs& a, uint2 ent, bool valid, const MvSlots& S, uint32_t (&row)[ASZP],
                                      uint32_t (&acc)[ASZP], uint32_t& u) {
  constexpr int TQ = (mv_orw<ASZP>() - ASZP) / 4;
  const uint32_t lane = threadIdx.x & 63, j = lane & (LW - 1), gb = lane & ~(LW - 1);
  u = ent.x & 0xFFFFFFu;
  const uint32_t k = ent.x >> 24, M = valid ? ent.y : 0u;
  if (GS_OOB(u, a.N, a.err, "pbfs wide node")) u = 0;
  const bool inM = (M >> j) & 1u;
  uint32_t rw[ASZP];
  const uint32_t* orow = a.own + (size_t)u * a.ORW;
  load_row<ASZP>(orow, rw);
  uint32_t tail[4 * TQ];
  {
    const uint4* t4 = reinterpret_cast<const uint4*>(orow + ASZP);
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const uint4 x = t4[q];
      tail[4 * q] = x.x; tail[4 * q + 1] = x.y; tail[4 * q + 2] = x.z; tail[4 * q + 3] = x.w;
    }
  }
  const uint32_t pm = inM ? a.mask[(size_t)u * a.MSU + a.s0 + j] : 0u;
  uint32_t hv = tail[0] & 0xFFFFu, fc[ASZP];
  if ((tail[0] >> 16) == k) {
#pragma unroll
    for (int s = 0; s < ASZP; ++s) fc[s] = (tail[1 + s / 4] >> (8 * (s % 4))) & 0xFFu;
  } else {  // an origin of lower bucket: entry min(bucket[u], bucket[origin])
    const uint32_t ent_i = u * NB + k;
    hv = a.hl[ent_i];
    load_row<ASZP>(a.peers + (size_t)ent_i * ASZP, rw);
#pragma unroll
    for (int s = 0; s < ASZP; ++s) fc[s] = a.any_fail ? a.fcls[rw[s]] : 0xFFu;
  }
  uint32_t tk = 0;
  if (inM) {
    tk = taken_slots<ASZP>(rw, hv & 0xFF, hv >> 8, a.ASZ, pm, S.sorg[j], a.fanout);
    const uint32_t f = S.sfk[j];
    if (f) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if (fc[s] <= f) tk &= ~(1u << s);
    }
    if (u - a.vlo < a.vhi - a.vlo) a.egress[(size_t)(u - a.vlo) * a.SP + a.s0 + j] = (uint8_t)__popc(tk);
  }
  uint32_t mr = 0, ma = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    const uint64_t b = __ballot((tk >> s) & 1u);
    const uint32_t m = (uint32_t)(b >> gb) & (LW == 32 ? 0xFFFFFFFFu : 0xFFFFu);
    if (j == (uint32_t)s) { ma = m; mr = rw[s]; }
  }
#pragma unroll
  for (int s = 0; s < ASZP; ++s) { row[s] = 0; acc[s] = 0; }
  row[0] = mr;
  acc[0] = ma;
}

template <int ASZP>
__global__ __launch_bounds__(PB_T, 1) void k_mv_pbfs(PbArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  // (everything in the dynamic LDS: no static shared memory shifts its 16-byte base)
  MvSlots& S = *reinterpret_cast<MvSlots*>(lds);
  uint32_t* gt = reinterpret_cast<uint32_t*>(lds + PB_HDR_SLOTS);
  uint32_t* sh = gt + GT_WORDS;
  unsigned char* smem = lds + PB_HDR;
  const MvArgs& a = p.a;
  const uint32_t tid = threadIdx.x, g = blockIdx.x, G = p.G, GL = p.GL;
  const uint32_t BSF = a.BSF, BPm = (1u << BSF) - 1, UB = a.UB, LB = p.LB;
  const uint32_t FPW = p.FPW, NO = FPW << BSF, ASZ = a.ASZ, CH = p.CH;
  const unsigned long long UBm = (1ull << UB) - 1, LBm = (1ull << LB) - 1;
  // LDS: stage [stage_bytes] (expand: CH * ASZ u64 records; receive: the T column's counts and
  // run starts, then the level's touched nodes) | visL [NO] | visP [NO] | hist [G + 16] |
  // fcur [FPW, padded to 4] | ent [PB_EC] u64 | bk [NO] u8 | (GS_PB_TRACE table)
  unsigned long long* stage = reinterpret_cast<unsigned long long*>(smem);
  uint32_t* visL = reinterpret_cast<uint32_t*>(smem + p.stage_bytes);
  uint32_t* visP = visL + NO;
  uint32_t* hist = visP + NO;
  uint32_t* fcur = hist + G + 16;
  uint2* ent = reinterpret_cast<uint2*>(fcur + ((FPW + 3) & ~3u));
  uint8_t* bk = reinterpret_cast<uint8_t*>(ent + PB_EC);
  uint32_t* pre = reinterpret_cast<uint32_t*>(stage);  // [PB_SEG + 1] (receive only)
  uint32_t* sb = pre + PB_SEG + 1;                     // [PB_SEG]
  uint32_t* tl = sb + PB_SEG + 3;                      // [NO] nodes with new bits this level
  uint2* gq = p.gq + (size_t)g * p.gq_cap;
  auto node_of = [&](uint32_t li) { return ((((li >> BSF) << GL) + g) << BSF) | (li & BPm); };

  mv_slots_load(a, S, tid, PB_T);
  for (uint32_t i = tid; i < GT_WORDS; i += PB_T) gt[i] = a.gt[i];
  for (uint32_t i = tid; i < NO; i += PB_T) {
    visL[i] = 0;
    visP[i] = 0;
    const uint32_t v = node_of(i);
    bk[i] = v < a.N ? a.bucket[v] : (uint8_t)0;
  }
  for (uint32_t i = tid; i < FPW; i += PB_T) fcur[i] = 0;
  lds_barrier();
  if (tid == 0) {  // level 0: the group's seeds (distinct origins, their own entries) this workgroup owns
    uint32_t n = 0;
    for (uint32_t i = 0; i < p.nseed; ++i) {
      const uint2 sd = p.seeds[i];
      const uint32_t v = sd.x & 0xFFFFFFu, fb = v >> BSF;
      if ((fb & (G - 1)) != g) continue;
      const uint32_t li = ((fb >> GL) << BSF) | (v & BPm);
      visL[li] |= sd.y;
      visP[li] |= sd.y;
      ent[n++] = sd;
    }
    sh[1] = n;
  }
  lds_barrier();
  uint32_t ne = sh[1];
  uint32_t L = 0, ep = 0;
  // GS_PB_TRACE (diagnostics): thread 0 keeps per-level phase times in LDS (u32, 10 ns units)
  // and merges them into the global table (max over workgroups) once, after the BFS
  const bool trc = p.tr != nullptr && tid == 0;
  uint32_t* trl = reinterpret_cast<uint32_t*>(bk + ((NO + 15) & ~15u));  // [PB_TRL][16] (trace builds only)
  constexpr uint32_t PB_TRL = 40;
  if (p.tr) {
    for (uint32_t i = tid; i < PB_TRL * 16; i += PB_T) trl[i] = 0;
    lds_barrier();
  }
  unsigned long long t0 = trc ? wall_clock64() : 0, tm = t0;
  auto tmark = [&](int slot, bool mx) {
    if (!trc || L >= PB_TRL) return;
    const unsigned long long now = wall_clock64();
    if (mx) trl[16 * L + slot] = max(trl[16 * L + slot], (uint32_t)(now - tm));
    else trl[16 * L + slot] = (uint32_t)(now - t0);
    if (slot == 1) trl[16 * L + 15] += (uint32_t)(now - tm);  // (sums over workgroups: expand, receive)
    if (slot == 3) trl[16 * L + 14] += (uint32_t)(now - tm);
    tm = now;
  };
  for (;;) {
    tmark(0, false);
    if (trc && L < PB_TRL) trl[16 * L + 5] = ne;
    // ---------------------------------------------- expand level L ----
    const uint32_t par = L & 1;
    uint32_t* T = p.T[par];
    unsigned long long* area = p.area[par];
    // few entries: one entry per LW lanes, in one chunk (pb_expand_wide)
    constexpr uint32_t LW = ASZP <= 16 ? 16u : 32u;
    const bool wide = a.Sg <= LW && ne <= PB_T / LW;
    const uint32_t step = wide ? PB_T / LW : CH;
    for (uint32_t c0 = 0; c0 < ne; c0 += step) {  // (ne is workgroup-uniform)
      // the chunk's slice: the returned value is first needed after the expansion (its
      // latency overlaps the row loads)
      uint32_t wsl = 0;
      if (tid == 0) wsl = atomicAdd(&p.blk[PB_SLICES + L], 1u);
      for (uint32_t i = tid; i < G; i += PB_T) hist[i] = 0;
      lds_barrier();
      if (c0 == 0) tmark(8, true);
      uint32_t row[ASZP], acc[ASZP], u = 0;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) { row[s] = 0; acc[s] = 0; }
      const uint32_t i = c0 + tid;
      if (wide) {
        const uint32_t e = tid / LW;
        pb_expand_wide<ASZP, LW>(a, e < ne ? ent[e] : make_uint2(0u, 0u), e < ne, S, row, acc, u);
      } else if (tid < CH && i < ne) {
        mv_expand_entry<ASZP>(a, i < PB_EC ? ent[i] : ld_entry(&gq[i - PB_EC]), S, row, acc, u);
      }
      if (trc && c0 == 0) {  // (trace: thread 0's own entry, its loads and stores drained)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        tmark(7, true);
      }
      uint32_t rk[ASZP];
#pragma unroll
      for (int s = 0; s < ASZP; ++s) rk[s] = acc[s] ? atomicAdd(&hist[(row[s] >> BSF) & (G - 1)], 1u) : 0u;
      if (tid == 0) sh[2] = wsl;
      lds_barrier();
      if (c0 == 0) tmark(9, true);
      const uint32_t total = pb_block_scan(hist, G, hist + G);
      const uint32_t w = sh[2];
      if (c0 == 0) tmark(10, true);
      const size_t b64 = (size_t)w * CH * ASZ;
      const bool ok = w < p.rows_cap && b64 + total <= p.area_cap;
      if (!ok && tid == 0) atomicOr(a.err, ERR_MV_CAP | (w < p.rows_cap ? ERR_MVD_AREA : ERR_MVD_ROWS));
      if (w < p.rows_cap) {
        for (uint32_t t = tid; t < G; t += PB_T) st_agent32(&T[(size_t)(1 + t) * p.TS + w], ok ? hist[t] : 0u);
        if (tid == 0) {
          st_agent32(&T[w], ok ? (uint32_t)b64 : 0u);
          st_agent32(&T[(size_t)(1 + G) * p.TS + w], ok ? total : 0u);
        }
      }
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if (acc[s]) {
          const uint32_t wp = row[s], fb = wp >> BSF;
          const uint32_t li = ((fb >> GL) << BSF) | (wp & BPm);
          stage[hist[fb & (G - 1)] + rk[s]] =
              (unsigned long long)u | ((unsigned long long)li << UB) | ((unsigned long long)acc[s] << (UB + LB));
        }
      lds_barrier();
      if (c0 == 0) tmark(11, true);
      if (ok)
        for (uint32_t r = tid; r < total; r += PB_T) st_agent64(&area[b64 + r], stage[r]);
      lds_barrier();  // (stage and hist are reused by the next chunk)
      if (c0 == 0) tmark(12, true);
    }
    tmark(1, true);
    // ---------------------------------------------- barrier ----
    pb_grid_sync(p.blk, ++ep, G, a.err);
    tmark(2, true);
    // ---------------------------------------------- receive level L's records (hop L + 1) ----
    const uint32_t ns = min(ld_agent32(&p.blk[PB_SLICES + L]), p.rows_cap);  // (grid-uniform)
    if (ns == 0) break;
    if (tid == 0) sh[3] = 0;  // touched nodes
    for (uint32_t c0 = 0; c0 < ns; c0 += PB_SEG) {
      const uint32_t gc = min(PB_SEG, ns - c0);
      for (uint32_t i = tid; i < gc; i += PB_T) {
        const uint32_t st = ld_agent32(&T[(size_t)(1 + g) * p.TS + c0 + i]);
        pre[i] = ld_agent32(&T[(size_t)(2 + g) * p.TS + c0 + i]) - st;  // (row 1 + G: the run's total)
        sb[i] = ld_agent32(&T[c0 + i]) + st;
      }
      lds_barrier();
      if (c0 == 0) tmark(13, true);
      const uint32_t ct = pb_block_scan(pre, gc, hist + G);
      if (ct == 0) continue;  // (uniform)
      if (trc && L < PB_TRL) trl[16 * L + 6] += ct;
      if (tid == 0) pre[gc] = ct;
      lds_barrier();
      if (c0 == 0) tmark(13, true);
      constexpr uint32_t AR = 4;  // records per thread per trip: searches and loads issued together
      for (uint32_t r0 = 0; r0 < ct; r0 += PB_T * AR) {
        unsigned long long rec[AR];
#pragma unroll
        for (uint32_t k = 0; k < AR; ++k) {
          const uint32_t r = r0 + k * PB_T + tid;
          uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pre[mid] <= r) lo = mid; else hi = mid;
          }
          rec[k] = r < ct ? ld_agent64(&area[(size_t)sb[lo] + (r - pre[lo])]) : ~0ull;
        }
#pragma unroll
        for (uint32_t k = 0; k < AR; ++k) {
          if (r0 + k * PB_T + tid >= ct) continue;
          uint32_t li = (uint32_t)((rec[k] >> UB) & LBm);
          if (GS_OOB(li, NO, a.err, "pbfs record node")) li = 0;
          const uint32_t m = (uint32_t)(rec[k] >> (UB + LB));
          const uint32_t old = atomicOr(&visL[li], m);
          // first arrivals: the node's first new bits of this level put it on the touched list once
          if ((m & ~old) && !(old & ~visP[li])) tl[atomicAdd(&sh[3], 1u)] = li;
          const uint32_t lf = li >> BSF;
          const uint32_t pp = atomicAdd(&fcur[lf], 1u);
          if (pp < a.pcap)
            a.pool[(size_t)((lf << GL) + g) * a.pcap + pp] = mv_pool_rec(a, (uint32_t)(rec[k] & UBm), li & BPm, L + 1, m);
        }
      }
      lds_barrier();  // (pre / sb are rewritten by the next batch)
    }
    lds_barrier();
    tmark(3, true);
    // ---------------------------------------------- level L + 1 entries ----
    const uint32_t nt = sh[3];
    uint32_t cntp = 0;
    for (uint32_t k = tid; k < nt; k += PB_T) {
      const uint32_t li = tl[k];
      cntp += mv_parts(gt, node_of(li), visL[li] & ~visP[li], bk[li], nullptr, 0);
    }
    const uint32_t incl = wave_incl_scan(cntp);
    if ((tid & 63) == 63) hist[tid >> 6] = incl;
    lds_barrier();
    uint32_t off = 0, tnew = 0;
    for (uint32_t k = 0; k < PB_T / 64; ++k) {
      if (k < (tid >> 6)) off += hist[k];
      tnew += hist[k];
    }
    if (tnew > PB_EC + p.gq_cap) {  // (cannot happen: gq_cap covers every node's parts)
      if (tid == 0) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_Q);
      tnew = PB_EC + p.gq_cap;
    }
    uint32_t pos = off + incl - cntp;
    for (uint32_t k = tid; k < nt; k += PB_T) {
      const uint32_t li = tl[k];
      const uint32_t nw = visL[li] & ~visP[li];
      visP[li] = visL[li];
      pos += mv_parts_to(gt, node_of(li), nw, bk[li], [&](uint32_t j, uint2 x) {
        const uint32_t q = pos + j;
        if (q < PB_EC) ent[q] = x;
        else if (q < PB_EC + p.gq_cap) st_entry(&gq[q - PB_EC], x);
      });
    }
    // entries in LDS; those in the workgroup's global region (sc1) are drained first
    if (tnew > PB_EC) __syncthreads();
    else lds_barrier();
    tmark(4, true);
    ++L;
    ne = tnew;
    if (L >= 254) {  // (grid-uniform) hops are u8: level 254 must be empty
      if (ne && tid == 0) atomicOr(a.err, ERR_DEPTH);
      break;
    }
  }
  if (trc)
    for (uint32_t i = 0; i < PB_TRL * 16; ++i) {
      const uint32_t k = i & 15;
      if (k == 5 || k == 6 || k == 14 || k == 15) atomicAdd(&p.tr[i], (unsigned long long)trl[i]);
      else if (k == 0) { if (g == 0) p.tr[i] = trl[i]; }
      else atomicMax(&p.tr[i], (unsigned long long)trl[i]);
    }
  // the pool fills of this workgroup's fine bins (k_mv_gather reads them)
  for (uint32_t lf = tid; lf < FPW; lf += PB_T) {
    const uint32_t fb = (lf << GL) + g;
    if (fb >= a.fno) continue;
    const uint32_t n = fcur[lf];
    if (n > a.pcap) atomicOr(a.err, ERR_MV_CAP | ERR_MVD_POOL);
    a.pused[fb] = min(n, (uint32_t)a.pcap);
  }
}

static uint32_t ilog2(uint32_t x) {
  uint32_t l = 0;
  while ((1u << (l + 1)) <= x) ++l;
  return l;
}

}  // namespace

// LDS bytes of the persistent BFS workgroup (dynamic part).
static size_t pb_stage_bytes(uint32_t stage_cap, uint32_t NO) {
  const size_t stage = std::max<size_t>((size_t)stage_cap * 8, (2 * (size_t)PB_SEG + 4 + NO) * 4);
  return (stage + 15) & ~(size_t)15;
}
static size_t pb_lds_bytes(uint32_t stage_cap, uint32_t NO, uint32_t G, uint32_t FPW) {
  return PB_HDR + pb_stage_bytes(stage_cap, NO) + 8 * (size_t)NO + 4 * ((size_t)G + 16) + 4 * (size_t)((FPW + 3) & ~3u) +
         8 * (size_t)PB_EC + (((size_t)NO + 15) & ~(size_t)15) + 40 * 16 * 4;  // (+ the GS_PB_TRACE table)
}

// Process-wide count of engines that may launch the persistent BFS: two persistent
// launches on one device (two engines on two streams) could each hold part of the CUs the
// other needs resident, so the persistent path runs only while one such engine exists.
// Across processes the same holds per device: two ranks sharing one GPU (the world-2 tests,
// a rehearsal of a multi-rank launch on one card) would each see one engine of their own.
// So the first registered engine of a process also takes an exclusive, non-blocking lock
// on a file named after the device's PCI bus id; a process that does not get it (another
// process on the card holds it) uses the launched level loop until its engines are gone.
// (Kernels of other processes still share the CUs, but they finish: the persistent
// launch's workgroups that wait at a barrier for the rest only wait longer.)
static std::atomic<int> g_pb_engines{0};
static std::mutex g_pb_mu;
static int g_pb_lock_fd = -1;
static std::atomic<bool> g_pb_locked{false};

static bool pb_lock_device() {
  int dev = 0;
  char bus[64] = {0};
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, dev) != hipSuccess) return false;
  std::string path = "/tmp/gossip_hip_pbfs_";
  for (const char* c = bus; *c; ++c) path += std::isalnum((unsigned char)*c) ? *c : '_';
  path += ".lock";
  const int fd = open(path.c_str(), O_RDONLY | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) return false;
  if (flock(fd, LOCK_EX | LOCK_NB) != 0) {
    close(fd);
    return false;
  }
  g_pb_lock_fd = fd;
  return true;
}

bool pb_setup(Engine& e) {
  e.pb_on = false;
  if (e.bfs_mode != GS_BFS_MULTI || e.part_on) return false;
  if (const char* x = std::getenv("GS_MV_PBFS"); x && x[0] == '0') return false;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  if (cus < 8) return false;
  const uint32_t G = 1u << ilog2((uint32_t)cus), GL = ilog2(G);
  const MvGeom& m = e.mv;
  const uint32_t nbf = (e.N + (1u << m.BSF) - 1) >> m.BSF;
  uint32_t FPW = (nbf + G - 1) >> GL;
  FPW = FPW <= 1 ? 1u : 1u << (ilog2(FPW - 1) + 1);  // power of two
  const uint32_t NO = FPW << m.BSF, LB = ilog2(FPW) + m.BSF;
  if (m.UB + LB + m.GW > 64) return false;
  uint32_t CH = PB_T;
  size_t lds = 0;
  for (;; CH /= 2) {
    lds = pb_lds_bytes(CH * e.ASZ, NO, G, FPW);
    if (lds <= 160 * 1024 || CH <= 256) break;
  }
  if (lds > 160 * 1024) return false;
  e.pb_G = G; e.pb_GL = GL; e.pb_FPW = FPW; e.pb_LB = LB; e.pb_CH = CH; e.pb_lds = lds;
  // slices per level: every workgroup's entries in chunks of CH
  const size_t maxparts = std::min<size_t>(m.GW, 26) + 1;
  e.pb_gq_cap = (uint32_t)std::min<size_t>((size_t)NO * maxparts, 0xFFFFFFF0u);
  e.pb_rows_cap = (uint32_t)std::min<size_t>((m.q_cap + CH - 1) / CH + G + 1, 0xFFFFFFF0u);
  e.pb_area_cap = (size_t)e.pb_rows_cap * CH * e.ASZ;
  if (e.pb_area_cap > 0xFFFFFFF0u) return false;  // (run bases are u32 in the T rows)
  e.pb_on = true;
  return true;
}

void pb_register(Engine& e, bool on) {
  std::lock_guard<std::mutex> lk(g_pb_mu);
  if (on) {
    if (g_pb_engines.fetch_add(1) == 0) g_pb_locked = pb_lock_device();  // (the engine's device is current)
  } else if (g_pb_engines.fetch_sub(1) == 1 && g_pb_lock_fd >= 0) {
    close(g_pb_lock_fd);  // (releases the lock)
    g_pb_lock_fd = -1;
    g_pb_locked = false;
  }
  (void)e;
}

bool pb_usable(const Engine& e) { return e.pb_on && g_pb_engines.load() == 1 && g_pb_locked.load(); }

hipError_t launch_bfs_pers(Engine& e, const MvArgs& a, const MvGroup& gr) {
  hipError_t r = hipSuccess;
  if (e.pb_attr_lds != e.pb_lds) {  // (once per engine)
    GS_ASZP_DISPATCH(e.ASZP, {
      r = hipFuncSetAttribute((const void*)k_mv_pbfs<A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e.pb_lds);
    });
    if (r != hipSuccess) return r;
    e.pb_attr_lds = e.pb_lds;
  }
  PbArgs p;
  p.a = a;
  p.seeds = e.mv_seed + gr.seed0;
  p.nseed = gr.nseed;
  p.G = e.pb_G; p.GL = e.pb_GL; p.FPW = e.pb_FPW; p.LB = e.pb_LB; p.CH = e.pb_CH;
  p.stage_bytes = (uint32_t)pb_stage_bytes(e.pb_CH * e.ASZ, e.pb_FPW << e.mv.BSF);
  p.rows_cap = e.pb_rows_cap; p.TS = e.pb_rows_cap;
  p.T[0] = e.pb_T[0]; p.T[1] = e.pb_T[1];
  p.area[0] = e.pb_area[0]; p.area[1] = e.pb_area[1];
  p.area_cap = e.pb_area_cap;
  p.blk = e.pb_blk;
  p.gq = e.pb_gq; p.gq_cap = e.pb_gq_cap;
  p.tr = nullptr;
  static const int trace_launch = [] {  // GS_PB_TRACE=k: per-level timings of the k-th launch to stderr
    const char* x = std::getenv("GS_PB_TRACE");
    return x ? std::atoi(x) : 0;
  }();
  static unsigned long long* trd = nullptr;
  static unsigned long long trh[640];
  static int launches = 0;
  const bool trace = trace_launch > 0 && ++launches == trace_launch;
  if (trace) {  // (device memory: the kernel's atomics on it stay on the device)
    if (!trd && hipMalloc(&trd, sizeof(trh)) != hipSuccess) return hipErrorOutOfMemory;
    if ((r = hipMemsetAsync(trd, 0, sizeof(trh), e.st))) return r;
    p.tr = trd;
  }
  if ((r = hipMemsetAsync(e.pb_blk, 0, PB_BLK_WORDS * 4, e.st))) return r;
  static const bool twice = std::getenv("GS_PB_TWICE") && std::getenv("GS_PB_TWICE")[0] == '1';  // (diagnostics)
  if (twice) {
    PbArgs q = p;
    q.tr = nullptr;
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_mv_pbfs<A>), dim3(e.pb_G), dim3(PB_T), e.pb_lds, e.st, q));
    if ((r = hipMemsetAsync(e.pb_blk, 0, PB_BLK_WORDS * 4, e.st))) return r;
  }
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL((k_mv_pbfs<A>), dim3(e.pb_G), dim3(PB_T), e.pb_lds, e.st, p));
  if (trace) {  // (diagnostics: waits for the launch; clocks at 100 MHz)
    if ((r = hipMemcpyAsync(trh, trd, sizeof(trh), hipMemcpyDeviceToHost, e.st)) || (r = hipStreamSynchronize(e.st)))
      return r;
    std::fprintf(stderr, "GS_PB_TRACE launch %d: level, start us, max expand / barrier / receive / entries us, entries, "
                 "records | expand: clear, entries+rank, scan+slice, T+stage, area, (thread 0's entry) | receive: T column+scan | "
                 "mean expand, receive\n", launches);
    for (int L = 0; L < 40 && (L == 0 || trh[16 * L + 5] || trh[16 * L + 6]); ++L) {
      const unsigned long long* t = trh + 16 * L;
      std::fprintf(stderr, "  %3d %8.1f %6.1f %6.1f %6.1f %6.1f %8llu %8llu | %5.1f %5.1f %5.1f %5.1f %5.1f (%5.1f) | %5.1f | %5.1f %5.1f\n",
                   L, t[0] / 100.0, t[1] / 100.0, t[2] / 100.0, t[3] / 100.0, t[4] / 100.0, t[5], t[6], t[8] / 100.0,
                   t[9] / 100.0, t[10] / 100.0, t[11] / 100.0, t[12] / 100.0, t[7] / 100.0, t[13] / 100.0,
                   t[15] / 100.0 / e.pb_G, t[14] / 100.0 / e.pb_G);
    }
  }
  return hipGetLastError();
}

size_t pb_blk_words() { return PB_BLK_WORDS; }

}  // namespace gs
