// gs_mv_dev.h -- device pieces shared by the multi-source BFS (gs_bfs_multi.hip) and the
// direction-optimizing BFS over the round's push graph (gs_bfs_hybrid.hip): the kernel
// argument block, the group tables, one frontier entry's expansion (PushActiveSet::get_nodes
// ..take(fanout), gossip.rs:527-541) and its split into per-entry parts.
#pragma once
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

constexpr uint32_t MV_XT = 256;       // expand threads = frontier entries per expand slice (one T row)
constexpr uint32_t MV_XT_L = 1024;    // ... for wide T rows (>= MV_XT_WIDE coarse bins: 10M-node graphs)
constexpr uint32_t MV_XT_WIDE = 512;
constexpr uint32_t MV_AT = 1024;      // apply threads
constexpr uint32_t MV_GT = 512;       // gather threads
constexpr uint32_t MV_SEG = 1024;     // T rows per apply chunk
constexpr uint32_t MV_NOPAIR = 0xFFFFFFFFu;  // expand / apply: the level is the kernel argument d
constexpr uint32_t GT_OWN = 0, GT_NOBS = 25, GT_OBV = 26, GT_OBM = 58, GT_NSEED = 90, GT_SEED = 91, GT_S0 = 92,
                   GT_SG = 93;

struct MvArgs {
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
  const uint32_t* own;    // [N][ORW] own-bucket rows; word ASZP = hl | bucket << 16
  const uint8_t* fcls;    // [N] failure class: smallest i with fail rank < the i-th failure count
  const uint8_t* fk;      // [S] failure class index of the slot's count (0: no failures)
  const uint32_t* origin;
  const uint32_t* mask;   // node-major [N][SP]
  const uint32_t* gt;     // this group's table (GT_STRIDE words)
  uint8_t* hops;
  uint32_t* cnt;
  uint32_t* inb;
  uint8_t* egress;        // node-major [NP][SP] (nodes [vlo, vhi))
  uint32_t* err;
  uint32_t* vis;          // [N] slot masks reached
  uint32_t clear_vis;     // the gather zeroes its bins' vis words (the next BFS needs no memset)
  uint32_t* lvl;          // [256] frontier entries per level
  uint32_t* hlvl;         // host-mapped [256]: expand(d) writes lvl[d] here (the polled loop)
  uint32_t* dpair;        // [258] level of expand/apply pair i (predicted loop): head writes [0], apply(i) [i + 1]
  uint32_t* hprof;        // host-mapped: the tail kernel's level profile (seq, levels, sizes)
  uint32_t* T;            // [rows_cap][TW] rows of the current level
  unsigned long long* area;  // records of the current level
  uint32_t* ctr;          // [0] records used in area (this level)
  unsigned long long* pool;  // [fno][pcap] records of the round per (kept) fine bin (mv_pool_rec)
  uint32_t* pused;        // [fno] records in each fine bin's pool region
  uint32_t* cmeta;        // fused consume (gs_round): the received caches, as in gs_consume_g.hip
  uint32_t* ckey;
  uint8_t* prune_round;
  uint32_t* ingress_acc;
  uint32_t N, SP, ASZ, fanout, capin, s0, Sg, UB, BSC, BSF, nbc, nbf, TW, ORW, any_fail, gcap, gcap_c;
  uint32_t lane_c, wave_c, record;
  unsigned long long* pclk;  // GS_PHASE_PROFILE: gather phase clocks at [11..15] (thread 0 of each workgroup)
  uint32_t gh;  // gather: nodes with more records (all slots) take the wave path
  // nodes with per-pair state [vlo, vhi) (= fine bins [flo, flo + fno)); pair = slot * NP + node - vlo.
  // A node-range partition rank runs the whole BFS but keeps the records, counts and
  // egress of its own nodes only.
  uint32_t vlo, vhi, flo, fno, NP;
  uint32_t MSU;  // node stride of the masks (SP, or 32 in node lines)
  uint32_t XT;   // frontier entries per expand slice (MV_XT or MV_XT_L; mv_geometry)
  uint32_t small;  // levels of at most this many entries run in the one-workgroup kernel
  uint32_t xrows;  // frontier-exchange partition: apply walks this many T rows (one per sender rank), else 0
  uint32_t TS;     // T: entries of one bin slot for consecutive runs are TS apart (mv_t)
  size_t PAIRS, area_cap, rows_cap, q_cap, pcap;
  // direction-optimizing BFS over the round's push graph (gs_bfs_hybrid.hip)
  uint8_t* dist;              // [N][DSP] each slot's BFS distance (0xFF: not reached)
  uint32_t DSP;               // 16 or 32 bytes per node
  uint2* pgo;                 // [N] {first, count} of the node's push-graph in-records in pgr
  uint32_t* F;                // [3][N] the slots each node first reached at level d: buffer d % 3
  unsigned long long* pgr;    // in-records (src | slot mask << 32) by destination, region per coarse bin
  size_t pg_bin_cap;          // records per coarse bin's region of pgr
  uint32_t pg_parts;          // T rows per push-graph slice (1 + the group's lower origin buckets)
  uint32_t pg_slices;         // push-graph slices (XT nodes each)
  uint32_t bu_min;            // bottom-up level: predicted entries at least (host side)
};

// Entry b of expand run (T row) w: b = 0 the run's base in the record area, b = 1 + c its
// start of coarse bin c, b = 1 + nbc its total. Stored bin-major, T[b * TS + w]: an apply
// workgroup reads its bin's starts over every run of the level as one contiguous range
// (row-major it read one scattered word per run: at C5's thousands of runs per level the
// column walk streamed ~1 GB of lines per peak level through L2).
__device__ inline uint32_t& mv_t(const MvArgs& a, uint32_t w, uint32_t b) { return a.T[(size_t)b * a.TS + w]; }

// A pool record: src | node-in-fine-bin << UB | hop << (UB + BSF) | slot mask << (UB + BSF + 8)
// (mv_geometry keeps UB + BSF + 8 + GW <= 64). The hop travels with the record, so the
// gather reads a fine bin's pool as one run whatever the level each record came from.
__device__ inline unsigned long long mv_pool_rec(const MvArgs& a, uint32_t u, uint32_t vf, uint32_t hop, uint32_t m) {
  return (unsigned long long)u | ((unsigned long long)vf << a.UB) | ((unsigned long long)hop << (a.UB + a.BSF)) |
         ((unsigned long long)m << (a.UB + a.BSF + 8));
}

__device__ inline uint32_t mv_xcd_bin(uint32_t i, uint32_t nbins) {
  const uint32_t per = (nbins + 7) / 8;
  return (i & 7u) * per + (i >> 3);
}

// Exclusive scan of LDS h[0..n) in place by the whole workgroup; wsum holds 16 words.
__device__ inline uint32_t mv_block_scan(uint32_t* h, uint32_t n, uint32_t* wsum) {
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

__host__ __device__ inline size_t mv_hist_bytes(uint32_t nbins) { return 4 * (size_t)((nbins + 17 + 1) & ~1u); }

// --------------------------------------------------------------- expand ----
constexpr uint32_t MV_SG4 = 7;  // slot quads per group (GW <= 28)

__host__ __device__ inline uint32_t mv_ohash(uint32_t x) { return (x * 0x9E3779B1u) >> 25; }

// The group's slots as the expand reads them (LDS): origins, failure classes, the slots
// that may take the shared-prefix path (pz: all, or none when the origin hash is
// incomplete, so that every slot takes the per-slot path), the origin -> slot-mask hash of
// the group table, and per failure class c the slots in which a peer of class c failed
// (fm[c] = slots j with 0 < c <= fk[j]; class 255 = fails nowhere, fm[255] = 0).
struct MvSlots {
  uint32_t sorg[32], sfk[32];
  uint2 otab[128];
  uint32_t fm[256];
  uint32_t pz;
};

// (no barrier: the caller's first __syncthreads publishes S)
__device__ inline void mv_slots_load(const MvArgs& a, MvSlots& S, uint32_t tid, uint32_t nth) {
  if (tid < a.Sg) {
    S.sorg[tid] = a.origin[a.s0 + tid];
    S.sfk[tid] = a.fk[a.s0 + tid];
  }
  const uint2* ot = reinterpret_cast<const uint2*>(a.gt + GT_OT);
  for (uint32_t i = tid; i < 128; i += nth) S.otab[i] = ot[i];
  for (uint32_t c = tid; c < 256; c += nth) {
    uint32_t m = 0;
    if (a.any_fail && c != 0)
      for (uint32_t j = 0; j < a.Sg; ++j) {
        const uint32_t f = a.fk[a.s0 + j];
        m |= (uint32_t)(f != 0 && c <= f) << j;
      }
    S.fm[c] = m;
  }
  if (tid == 0) S.pz = a.gt[GT_OTOK] ? 0xFFFFFFFFu : 0u;
}

// The group's slots whose origin is node x.
__device__ inline uint32_t mv_origin_slots(const MvSlots& S, uint32_t x) {
  const uint32_t h0 = mv_ohash(x);
  const uint2 e0 = S.otab[h0], e1 = S.otab[(h0 + 1) & 127u];
  return (e0.x == x ? e0.y : 0u) | (e1.x == x ? e1.y : 0u);
}

// Words of an own-bucket row in the multi-source BFS: the ring, hl | bucket << 16, the
// peers' failure classes (one byte each), padded to 16 bytes.
template <int ASZP>
constexpr int mv_orw() { return ((ASZP + 1 + ASZP / 4) + 3) & ~3; }

// One frontier entry (node u, entry k, slot mask M): the pushed-to ring slots of every
// slot in M (PushActiveSet::get_nodes(..).take(fanout), gossip.rs:527-541: unpruned,
// not the origin, failed peers burn their slot) as per-ring-slot slot masks acc[s], and
// each slot's egress byte.
// Plain slots (no prunes at u) push to the first `fanout` ring positions except their
// own origin: one prefix of the ring for all of them, and a slot whose origin sits in that
// prefix swaps it for position `fanout` (the group's origins are looked up once per
// pushed-to peer in an LDS hash). Failed peers burn their slot (the take(fanout) comes
// before the failed check), so a plain slot's failures only remove pushes from the prefix:
// ring slot s loses the slots fm[class of its peer] (round 6; before, every slot with
// failures ran the per-slot selection -- C4's five fail-nodes slots at every entry). Only
// slots with prune bits at u run the per-slot selection, which a wave executes for the
// union of its lanes' slots. Plain slots' push counts come from bit-sliced counters.
template <int ASZP, bool EG = true>  // EG: write the egress bytes of the entry's slots
__device__ __forceinline__ void mv_expand_entry(const MvArgs& a, uint2 ent, const MvSlots& S, uint32_t (&row)[ASZP],
                                       uint32_t (&acc)[ASZP], uint32_t& u) {
  constexpr int TQ = (mv_orw<ASZP>() - ASZP) / 4;
  u = ent.x & 0xFFFFFFu;
  const uint32_t k = ent.x >> 24, M = ent.y;
  if (GS_OOB(u, a.N, a.err, "multi frontier node")) u = 0;
  const uint32_t nq = (a.Sg + 3) >> 2;
  // the row (with its failure classes) and every slot quad's masks: independent loads
  const uint32_t* orow = a.own + (size_t)u * a.ORW;
  load_row<ASZP>(orow, row);
  uint32_t tail[4 * TQ];
  {
    const uint4* t4 = reinterpret_cast<const uint4*>(orow + ASZP);
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      const uint4 x = t4[q];
      tail[4 * q] = x.x; tail[4 * q + 1] = x.y; tail[4 * q + 2] = x.z; tail[4 * q + 3] = x.w;
    }
  }
  uint4 m4[MV_SG4];
  const uint4* mq = reinterpret_cast<const uint4*>(a.mask + (size_t)u * a.MSU + a.s0);  // (same line as the row)
#pragma unroll
  for (uint32_t q = 0; q < MV_SG4; ++q) m4[q] = (q < nq && ((M >> (4 * q)) & 0xFu)) ? mq[q] : make_uint4(0, 0, 0, 0);
  uint32_t hv = tail[0] & 0xFFFFu;
  uint32_t fc[ASZP];
  if ((tail[0] >> 16) == k) {
#pragma unroll
    for (int s = 0; s < ASZP; ++s) fc[s] = (tail[1 + s / 4] >> (8 * (s % 4))) & 0xFFu;
  } else {  // an origin of lower bucket: entry min(bucket[u], bucket[origin])
    const uint32_t ent_i = u * NB + k;
    hv = a.hl[ent_i];
    load_row<ASZP>(a.peers + (size_t)ent_i * ASZP, row);
#pragma unroll
    for (int s = 0; s < ASZP; ++s) fc[s] = a.any_fail ? a.fcls[row[s]] : 0xFFu;
  }
  const uint32_t head = hv & 0xFF, len = hv >> 8;
  uint32_t plain = 0, pc0 = 0, pc1 = 0, pc2 = 0, pc3 = 0, pc4 = 0;  // (plain slots' push counts, bit-sliced)
  if constexpr (ASZP < 32) {
    uint32_t pmz = 0;  // slots with no prunes at u
#pragma unroll
    for (uint32_t q = 0; q < MV_SG4; ++q)
      pmz |= ((uint32_t)(m4[q].x == 0) | ((uint32_t)(m4[q].y == 0) << 1) | ((uint32_t)(m4[q].z == 0) << 2) |
              ((uint32_t)(m4[q].w == 0) << 3)) << (4 * q);
    plain = M & S.pz & pmz;
    if (plain) {
      const uint32_t SZ = a.ASZ, full = (1u << SZ) - 1u;
      const uint32_t L = min(len, SZ), nf = min(L, a.fanout);
      const uint32_t pre = (1u << nf) - 1u, nxp = L > a.fanout ? 1u << a.fanout : 0u;  // ring positions
      const uint32_t tkn = ((pre << head) | (pre >> (SZ - head))) & full;               // physical slots
      const uint32_t nxt = ((nxp << head) | (nxp >> (SZ - head))) & full;
      // ring slot s pushes to the slots x: failed peers burn their slot (gossip.rs:538-541),
      // and a bit-sliced add counts the pushes per plain slot (<= fanout < 32). (Applied in
      // place per s: a per-slot array here went to scratch at ASZP 20, 3x the expand time.)
      auto take = [&](int s, uint32_t x) {
        if (a.any_fail) x &= ~S.fm[fc[s]];
        acc[s] |= x;
        uint32_t t;
        t = pc0 & x; pc0 ^= x; x = t;
        t = pc1 & x; pc1 ^= x; x = t;
        t = pc2 & x; pc2 ^= x; x = t;
        t = pc3 & x; pc3 ^= x; x = t;
        pc4 ^= x;
      };
      uint32_t rem = 0;  // plain slots whose origin is in the prefix
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        if (!((tkn >> s) & 1u)) continue;
        const uint32_t om = mv_origin_slots(S, row[s]) & plain;
        take(s, plain & ~om);
        rem |= om;
      }
      if (rem) {  // those slots take position `fanout` instead (disjoint from the prefix)
#pragma unroll
        for (int s = 0; s < ASZP; ++s)
          if ((nxt >> s) & 1u) take(s, rem);
      }
    }
  }
  const bool own_u = u - a.vlo < a.vhi - a.vlo;  // egress is kept for owned nodes
  uint8_t* eg = a.egress + (size_t)(u - a.vlo) * a.SP + a.s0;
#pragma unroll
  for (uint32_t q = 0; q < MV_SG4; ++q) {
    if (q >= nq) break;
    const uint32_t mq4 = (M >> (4 * q)) & 0xFu;
    if (!mq4) continue;
    uint32_t egw = 0;
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
      const uint32_t j = 4 * q + t;
      if (!((mq4 >> t) & 1u)) continue;
      if ((plain >> j) & 1u) {
        egw |= (((pc0 >> j) & 1u) | (((pc1 >> j) & 1u) << 1) | (((pc2 >> j) & 1u) << 2) | (((pc3 >> j) & 1u) << 3) |
                (((pc4 >> j) & 1u) << 4)) << (8 * t);
        continue;
      }
      const uint32_t pm = t == 0 ? m4[q].x : t == 1 ? m4[q].y : t == 2 ? m4[q].z : m4[q].w;
      const uint32_t f = S.sfk[j];
      uint32_t tk = taken_slots<ASZP>(row, head, len, a.ASZ, pm, S.sorg[j], a.fanout);
      if (f) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
        for (int s = 0; s < ASZP; ++s)
          if (fc[s] <= f) tk &= ~(1u << s);
      }
#pragma unroll
      for (int s = 0; s < ASZP; ++s) acc[s] |= ((tk >> s) & 1u) << j;
      egw |= (uint32_t)__popc(tk) << (8 * t);
    }
    if (!EG || !own_u) {
    } else if (mq4 == 0xFu) {
      *reinterpret_cast<uint32_t*>(eg + 4 * q) = egw;  // SP and s0 are multiples of 4
    } else {
#pragma unroll
      for (uint32_t t = 0; t < 4; ++t)
        if ((mq4 >> t) & 1u) eg[4 * q + t] = (uint8_t)(egw >> (8 * t));
    }
  }
}

// Node v's new slots as frontier entries, one per distinct entry k: slots whose origin
// bucket is >= bucket[v] share v's own entry, the rest split by origin bucket. Returns
// the entry count; writes them at out[pos..] when out != nullptr.
template <class Put>
__device__ inline uint32_t mv_parts_to(const uint32_t* gt, uint32_t v, uint32_t nw, uint32_t bv, Put put) {
  uint32_t n = 0;
  const uint32_t own = nw & gt[GT_OWN + bv];
  if (own) put(n++, make_uint2(v | (bv << 24), own));
  const uint32_t rest = nw & ~own;
  if (rest) {
    const uint32_t nobs = gt[GT_NOBS];
    for (uint32_t i = 0; i < nobs; ++i) {
      const uint32_t m = rest & gt[GT_OBM + i];
      if (m) put(n++, make_uint2(v | (gt[GT_OBV + i] << 24), m));
    }
  }
  return n;
}

__device__ inline uint32_t mv_parts(const uint32_t* gt, uint32_t v, uint32_t nw, uint32_t bv, uint2* out,
                                    uint32_t pos) {
  return mv_parts_to(gt, v, nw, bv, [&](uint32_t k, uint2 x) {
    if (out) out[pos + k] = x;
  });
}

template <class T>
__device__ inline T mv_ld(T* p) {  // device-scope load: lines updated by atomics elsewhere
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A barrier for LDS only: global stores in flight are not waited for (nothing in the level
// loop reads another thread's global stores; vis is read by atomics only).
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Kernel arguments of slot group g (gs_bfs_multi.hip).
MvArgs mv_args(Engine& e, const MvGroup& gr, uint32_t g);

// The whole BFS of one slot group as one persistent launch (gs_bfs_pers.hip).
hipError_t launch_bfs_pers(Engine& e, const MvArgs& a, const MvGroup& gr);

}  // namespace gs
