// gs_bfs_multi.hip -- Cluster::run_gossip (gossip.rs:494-615) for large clusters as a
// batched multi-source frontier BFS: every slot of a slot group advances at once,
// and a node's active-set row is expanded ONCE per level for all the group's slots
// that reach it at that level.
//
// A slot group is a contiguous range of at most GW slots (bit j = slot s0 + j). The
// visited state is a slot mask per node (vis[N]); a frontier entry is (node u, entry
// k, slot mask M): the slots in M first reached u at this level and all of them push
// from u's entry k = min(bucket[u], bucket[origin]) (push_active_set.rs:38-52). Slots
// that share u and k but not the entry are split into separate entries when u is
// appended. Per BFS level:
//
//   expand (workgroup w owns frontier entries [w*PW, (w+1)*PW)): loads the entry's row
//     (the compact own-bucket table when k = bucket[u]), takes per slot the first
//     `fanout` unpruned non-origin ring slots (failed peers burn a slot, gossip.rs:
//     527-541) and ORs the slot's bit into a per-ring-slot mask; every pushed-to peer w
//     becomes ONE record (src u, w, slots) however many slots pushed there. Records
//     are ranked per destination bin (2^BS nodes) with LDS atomics, staged sorted by
//     bin and written as one contiguous run; T row [base, bin starts..., total].
//   apply (one workgroup per bin, bins dealt to XCDs in contiguous ranges): ORs the
//     level's records into an LDS copy of the bin's vis masks; new bits are first
//     arrivals at hop d+1 (gossip.rs:594-600); new nodes are appended to the next
//     frontier, one entry per distinct entry k.
//   gather (after the last level, one workgroup per bin): the bin's records of every
//     level as an LDS CSR by destination; per (slot, node): in-degree, the inbound
//     records hop << 24 | src (gossip.rs:601-607) written as rows inb[c][pair]
//     coalesced over nodes, and the hop (1 + the smallest pusher level; 0 at the
//     origin, unreached = 0xFF).
//
// Results equal k_bfs_level's: hops, in-degrees, inbound record sets, egress.
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

namespace {

constexpr uint32_t MV_XT = 256;       // expand threads
constexpr uint32_t MV_AT = 256;       // apply threads
constexpr uint32_t MV_GT = 512;       // gather threads
constexpr uint32_t MV_SEG = 1024;     // T rows per apply / gather chunk
constexpr uint32_t GT_OWN = 0, GT_NOBS = 25, GT_OBV = 26, GT_OBM = 58, GT_NSEED = 90, GT_SEED = 91, GT_S0 = 92,
                   GT_SG = 93;

struct MvArgs {
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
  const uint32_t* own;    // [N][ORW] own-bucket rows; word ASZP = hl | bucket << 16
  const uint32_t* frank;
  const uint32_t* origin;
  const uint32_t* nfail;
  const uint32_t* mask;
  const uint32_t* gt;     // this group's table (GT_WORDS words)
  uint8_t* hops;
  uint32_t* cnt;
  uint32_t* inb;
  uint8_t* egress;
  uint32_t* err;
  uint32_t* vis;          // [N] slot masks reached
  uint32_t* lvl;          // [256] frontier entries per level
  uint32_t* tb;           // [257] first T row of level d
  uint32_t* T;            // [rows][TW]
  unsigned long long* area;
  uint32_t* ctr;          // [0] records used in area
  uint32_t N, ASZ, fanout, capin, s0, Sg, UB, BS, nbins, TW, PW, ORW, any_fail, gcap;
  size_t PAIRS, area_cap, rows_cap, q_cap;
};

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
template <int ASZP, int XPT>
__global__ __launch_bounds__(MV_XT) void k_mv_expand(MvArgs a, uint32_t d, const uint2* __restrict__ qcur) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t sorg[32], snf[32], sbase;
  const uint32_t qn = a.lvl[d];
  const uint32_t tb = a.tb[d];
  constexpr uint32_t PW = MV_XT * XPT;
  const uint32_t G = (qn + PW - 1) / PW;
  if (blockIdx.x == 0 && threadIdx.x == 0) a.tb[d + 1] = tb + G;  // read by apply(d+1) and the gather
  if (qn == 0) return;
  if ((size_t)tb + G > a.rows_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.err, ERR_MV_CAP);
    return;
  }
  const uint32_t tid = threadIdx.x, nb = a.nbins, BS = a.BS, UB = a.UB, BPm = (1u << BS) - 1;
  if (tid < a.Sg) {
    sorg[tid] = a.origin[a.s0 + tid];
    snf[tid] = a.nfail[a.s0 + tid];
  }
  uint32_t* hist = reinterpret_cast<uint32_t*>(smem);  // [nb] + scan words
  unsigned long long* stage = reinterpret_cast<unsigned long long*>(smem + mv_hist_bytes(nb));  // [PW * ASZP]
  __syncthreads();
  for (uint32_t w = blockIdx.x; w < G; w += gridDim.x) {
    for (uint32_t i = tid; i < nb; i += MV_XT) hist[i] = 0;
    __syncthreads();
    uint32_t row[XPT][ASZP], acc[XPT][ASZP], uu[XPT];
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      const uint32_t i = w * PW + j * MV_XT + tid;
      uu[j] = 0;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) { row[j][s] = 0; acc[j][s] = 0; }
      if (i >= qn) continue;
      const uint2 ent = qcur[i];
      uint32_t u = ent.x & 0xFFFFFFu;
      const uint32_t k = ent.x >> 24, M = ent.y;
      if (GS_OOB(u, a.N, a.err, "multi frontier node")) continue;
      uu[j] = u;
      const uint32_t* orow = a.own + (size_t)u * a.ORW;
      load_row<ASZP>(orow, row[j]);
      const uint32_t meta = orow[ASZP];
      uint32_t hv = meta & 0xFFFFu;
      if ((meta >> 16) != k) {  // an origin of lower bucket: entry min(bucket[u], bucket[origin])
        const uint32_t ent_i = u * NB + k;
        hv = a.hl[ent_i];
        load_row<ASZP>(a.peers + (size_t)ent_i * ASZP, row[j]);
      }
      const uint32_t head = hv & 0xFF, len = hv >> 8;
      uint32_t fr[ASZP];
      if (a.any_fail) {
#pragma unroll
        for (int s = 0; s < ASZP; ++s) fr[s] = a.frank[row[j][s]];
      }
      // slot masks four at a time: the loads issue back to back
      for (uint32_t mm = M; mm;) {
        uint32_t jj[4], pm[4];
        int nq = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          jj[t] = 0;
          pm[t] = 0;
          if (mm) {
            jj[t] = __ffs(mm) - 1;
            mm &= mm - 1;
            pm[t] = a.mask[(size_t)(a.s0 + jj[t]) * a.N + u];
            nq = t + 1;
          }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t >= nq) break;
          uint32_t tk = taken_slots<ASZP>(row[j], head, len, a.ASZ, pm[t], sorg[jj[t]], a.fanout);
          const uint32_t nf = snf[jj[t]];
          if (nf) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
            for (int s = 0; s < ASZP; ++s)
              if (((tk >> s) & 1u) && fr[s] < nf) tk &= ~(1u << s);
          }
          a.egress[(size_t)(a.s0 + jj[t]) * a.N + u] = (uint8_t)__popc(tk);
#pragma unroll
          for (int s = 0; s < ASZP; ++s) acc[j][s] |= ((tk >> s) & 1u) << jj[t];
        }
      }
    }
    // every LDS atomic after every load: each record's rank within its bin
    uint32_t rk[XPT][ASZP];
#pragma unroll
    for (int j = 0; j < XPT; ++j)
#pragma unroll
      for (int s = 0; s < ASZP; ++s) rk[j][s] = acc[j][s] ? atomicAdd(&hist[row[j][s] >> BS], 1u) : 0u;
    __syncthreads();
    uint32_t total = mv_block_scan(hist, nb, hist + nb);
    if (tid == 0) {
      uint32_t base = atomicAdd(a.ctr, total);
      if ((size_t)base + total > a.area_cap) {
        atomicOr(a.err, ERR_MV_CAP);
        base = 0xFFFFFFFFu;
      }
      sbase = base;
    }
    __syncthreads();
    const uint32_t base = sbase;
    const bool ok = base != 0xFFFFFFFFu;
    uint32_t* Tr = a.T + (size_t)(tb + w) * a.TW;
    for (uint32_t b = tid; b < nb; b += MV_XT) Tr[1 + b] = ok ? hist[b] : 0u;
    if (tid == 0) {
      Tr[0] = ok ? base : 0u;
      Tr[1 + nb] = ok ? total : 0u;
    }
#pragma unroll
    for (int j = 0; j < XPT; ++j)
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if (acc[j][s]) {
          const uint32_t wp = row[j][s];
          stage[hist[wp >> BS] + rk[j][s]] = (unsigned long long)uu[j] | ((unsigned long long)(wp & BPm) << UB) |
                                             ((unsigned long long)acc[j][s] << (UB + BS));
        }
    __syncthreads();
    if (ok)
      for (uint32_t i = tid; i < total; i += MV_XT) a.area[base + i] = stage[i];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- apply ----
__host__ __device__ inline size_t mv_apply_lds_bytes(uint32_t BS) {
  return 4 * (2 * (size_t)MV_SEG + 1 + 2 * ((size_t)1 << BS) + 32 + GT_WORDS);
}

// Node v's new slots as frontier entries, one per distinct entry k: slots whose origin
// bucket is >= bucket[v] share v's own entry, the rest split by origin bucket. Returns
// the entry count; writes them at out[pos..] when out != nullptr.
__device__ inline uint32_t mv_parts(const uint32_t* gt, uint32_t v, uint32_t nw, uint32_t bv, uint2* out,
                                    uint32_t pos) {
  uint32_t n = 0;
  const uint32_t own = nw & gt[GT_OWN + bv];
  if (own) {
    if (out) out[pos] = make_uint2(v | (bv << 24), own);
    ++n;
  }
  const uint32_t rest = nw & ~own;
  if (rest) {
    const uint32_t nobs = gt[GT_NOBS];
    for (uint32_t i = 0; i < nobs; ++i) {
      const uint32_t m = rest & gt[GT_OBM + i];
      if (!m) continue;
      if (out) out[pos + n] = make_uint2(v | (gt[GT_OBV + i] << 24), m);
      ++n;
    }
  }
  return n;
}

__global__ __launch_bounds__(MV_AT) void k_mv_apply(MvArgs a, uint32_t d, uint2* __restrict__ qnxt) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t qn = a.lvl[d];
  if (qn == 0) return;
  const uint32_t b = mv_xcd_bin(blockIdx.x, a.nbins);
  if (b >= a.nbins) return;
  const uint32_t tid = threadIdx.x, BS = a.BS, UB = a.UB, BP = 1u << BS, BPm = BP - 1;
  const uint32_t G = (qn + a.PW - 1) / a.PW, tb = a.tb[d];
  const uint32_t v0 = b << BS, nv = min(BP, a.N - v0);
  uint32_t* pre = reinterpret_cast<uint32_t*>(smem);  // [MV_SEG + 1]
  uint32_t* sb = pre + MV_SEG + 1;                    // [MV_SEG]
  uint32_t* visL = sb + MV_SEG;                       // [BP]
  uint32_t* vis0 = visL + BP;                         // [BP]
  uint32_t* ctl = vis0 + BP;                          // [32]
  uint32_t* gt = ctl + 32;                            // [GT_WORDS]
  for (uint32_t i = tid; i < GT_WORDS; i += MV_AT) gt[i] = a.gt[i];
  for (uint32_t i = tid; i < nv; i += MV_AT) {
    const uint32_t m = a.vis[v0 + i];
    visL[i] = m;
    vis0[i] = m;
  }
  __syncthreads();
  for (uint32_t c0 = 0; c0 < G; c0 += MV_SEG) {
    const uint32_t gc = min(MV_SEG, G - c0);
    for (uint32_t i = tid; i < gc; i += MV_AT) {
      const uint32_t* Tr = a.T + (size_t)(tb + c0 + i) * a.TW;
      const uint32_t st = Tr[1 + b];
      pre[i] = Tr[2 + b] - st;  // bin starts are exclusive; Tr[1 + nbins] is the run's total
      sb[i] = Tr[0] + st;
    }
    __syncthreads();
    const uint32_t ct = mv_block_scan(pre, gc, ctl);
    if (tid == 0) pre[gc] = ct;
    __syncthreads();
    for (uint32_t r = tid; r < ct; r += MV_AT) {
      uint32_t lo = 0, hi = gc;  // largest i with pre[i] <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= r) lo = mid; else hi = mid;
      }
      const unsigned long long rec = a.area[sb[lo] + (r - pre[lo])];
      uint32_t vl = (uint32_t)(rec >> UB) & BPm;
      if (GS_OOB(vl, nv, a.err, "multi record node")) vl = 0;
      atomicOr(&visL[vl], (uint32_t)(rec >> (UB + BS)));
    }
    __syncthreads();
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
  if (tnew == 0) return;
  if (tid == 0) {
    const uint32_t base = atomicAdd(&a.lvl[d + 1], tnew);
    ctl[1] = base;
    if ((size_t)base + tnew > a.q_cap) { atomicOr(a.err, ERR_MV_CAP); ctl[1] = 0xFFFFFFFFu; }
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
}

// --------------------------------------------------------------- gather ----


__host__ __device__ inline size_t mv_gather_fixed_bytes(uint32_t BS) {
  return 4 * (2 * ((size_t)1 << BS) + 2 + 3 * (size_t)MV_SEG + 1 + 32 + 32);
}

// Walks the bin's records of levels [0, nlev) (T rows in level order); f(level, rec).
template <class F>
__device__ inline void mv_walk(const MvArgs& a, uint32_t b, uint32_t nlev, uint32_t* pre, uint32_t* sb, uint32_t* lv,
                               uint32_t* ctl, F&& f) {
  const uint32_t tid = threadIdx.x, TH = blockDim.x;
  const uint32_t R = a.tb[nlev];
  for (uint32_t c0 = 0; c0 < R; c0 += MV_SEG) {
    const uint32_t gc = min(MV_SEG, R - c0);
    for (uint32_t i = tid; i < gc; i += TH) {
      const uint32_t r = c0 + i;
      const uint32_t* Tr = a.T + (size_t)r * a.TW;
      const uint32_t st = Tr[1 + b];
      pre[i] = Tr[2 + b] - st;
      sb[i] = Tr[0] + st;
      uint32_t lo = 0, hi = nlev;  // level of row r: largest d with tb[d] <= r
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.tb[mid] <= r) lo = mid; else hi = mid;
      }
      lv[i] = lo;
    }
    __syncthreads();
    const uint32_t ct = mv_block_scan(pre, gc, ctl);
    if (tid == 0) pre[gc] = ct;
    __syncthreads();
    for (uint32_t r = tid; r < ct; r += TH) {
      uint32_t lo = 0, hi = gc;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= r) lo = mid; else hi = mid;
      }
      f(lv[lo], a.area[sb[lo] + (r - pre[lo])]);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(MV_GT) void k_mv_gather(MvArgs a, uint32_t nlev) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t b = mv_xcd_bin(blockIdx.x, a.nbins);
  if (b >= a.nbins) return;
  const uint32_t tid = threadIdx.x, BS = a.BS, UB = a.UB, BP = 1u << BS, BPm = BP - 1, Sg = a.Sg;
  const uint32_t v0 = b << BS, nv = min(BP, a.N - v0);
  const unsigned long long um = (1ull << UB) - 1;
  uint32_t* cn = reinterpret_cast<uint32_t*>(smem);  // [BP + 1] records per node -> CSR starts
  uint32_t* cur = cn + BP + 1;                       // [BP + 1] placement cursors
  uint32_t* pre = cur + BP + 1;                      // [MV_SEG + 1]
  uint32_t* sb = pre + MV_SEG + 1;                   // [MV_SEG]
  uint32_t* lv = sb + MV_SEG;                        // [MV_SEG]
  uint32_t* ctl = lv + MV_SEG;                       // [32]
  uint32_t* sorg = ctl + 32;                         // [32]
  uint32_t* keys = sorg + 32;                        // [gcap] hop << 24 | src
  uint32_t* msk = keys + a.gcap;                     // [gcap] slot masks
  for (uint32_t i = tid; i <= BP; i += MV_GT) cn[i] = 0;
  if (tid < Sg) sorg[tid] = a.origin[a.s0 + tid];
  __syncthreads();
  // 1. records per destination node
  mv_walk(a, b, nlev, pre, sb, lv, ctl, [&](uint32_t, unsigned long long rec) {
    atomicAdd(&cn[(uint32_t)(rec >> UB) & BPm], 1u);
  });
  const uint32_t Etot = mv_block_scan(cn, BP, ctl);
  if (tid == 0) cn[BP] = Etot;
  __syncthreads();
  // 2. node ranges whose records fit the LDS CSR (one range unless the bin is heavy)
  bool over = false;
  for (uint32_t lo = 0; lo < nv;) {
    uint32_t hi = lo;
    if (tid == 0) {
      uint32_t h = lo;
      while (h < nv && cn[h + 1] - cn[lo] <= a.gcap) ++h;
      if (h == lo) { atomicOr(a.err, ERR_MV_CAP); h = nv; }  // one node beyond the LDS CSR
      ctl[16] = h;
    }
    __syncthreads();
    hi = ctl[16];
    const uint32_t base = cn[lo];
    for (uint32_t i = lo + tid; i < hi; i += MV_GT) cur[i] = cn[i] - base;
    __syncthreads();
    mv_walk(a, b, nlev, pre, sb, lv, ctl, [&](uint32_t d, unsigned long long rec) {
      const uint32_t vl = (uint32_t)(rec >> UB) & BPm;
      if (vl < lo || vl >= hi) return;
      const uint32_t p = atomicAdd(&cur[vl], 1u);
      if (p >= a.gcap) return;
      keys[p] = ((d + 1) << 24) | (uint32_t)(rec & um);
      msk[p] = (uint32_t)(rec >> (UB + BS));
    });
    // 3. per (slot, node): in-degree, inbound rows, hop; coalesced over nodes
    for (uint32_t i = lo + tid; i < hi; i += MV_GT) {
      const uint32_t v = v0 + i, r0 = cn[i] - base, r1 = min(cn[i + 1] - base, a.gcap);
      for (uint32_t j = 0; j < Sg; ++j) {
        const size_t p = (size_t)(a.s0 + j) * a.N + v;
        uint32_t c = 0, mh = 0xFFu;
        for (uint32_t r = r0; r < r1; ++r) {
          if (!((msk[r] >> j) & 1u)) continue;
          const uint32_t key = keys[r];
          if (c < a.capin) a.inb[(size_t)c * a.PAIRS + p] = key;
          mh = min(mh, key >> 24);
          ++c;
        }
        over |= c > a.capin;
        a.cnt[p] = c;
        a.hops[p] = (uint8_t)(v == sorg[j] ? 0u : (c ? mh : 0xFFu));
      }
    }
    __syncthreads();
    lo = hi;
  }
  if (over) atomicOr(a.err, ERR_INBOUND);
}

__global__ void k_mv_seed(MvArgs a, const uint2* __restrict__ seeds, uint32_t nseed, uint2* __restrict__ q0) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nseed) {
    const uint2 s = seeds[i];
    q0[i] = s;
    a.vis[s.x & 0xFFFFFFu] = s.y;  // seed nodes are distinct origins
  }
  if (i == 0) {
    a.lvl[0] = nseed;
    a.tb[0] = 0;
    a.ctr[0] = 0;
  }
}

}  // namespace

// ------------------------------------------------------------------ host ----
static uint32_t ceil_log2(size_t x) {
  uint32_t l = 0;
  while (((size_t)1 << l) < x) ++l;
  return l;
}

void mv_geometry(uint32_t N, uint32_t S, uint32_t ASZ, uint32_t ASZP, MvGeom& g) {
  g.UB = std::max(1u, ceil_log2(N));
  g.BS = std::min(13u, std::max(6u, g.UB > 10 ? g.UB - 10 : 0u));
  g.nbins = (N + (1u << g.BS) - 1) >> g.BS;
  g.GW = std::min(32u, 64u - g.UB - g.BS);
  g.XPT = ASZP <= 16 ? 2 : 1;
  g.PW = MV_XT * g.XPT;
  g.TW = g.nbins + 2;
  const size_t sg = std::min<size_t>(S, g.GW);
  g.q_cap = (size_t)N * std::min<size_t>(sg, 26) + 64;
  const size_t hard = (size_t)N * sg * ASZ;  // every (slot, node) reached once, <= ASZ records each
  g.area_cap = std::min(hard, std::max<size_t>((size_t)N * ASZ * 4, (size_t)1 << 29));
  g.area_cap = std::min<size_t>(g.area_cap, 0xFFFFFFF0u);
  const size_t rows_hard = (size_t)N * sg / g.PW + 260;
  g.rows_cap = std::min(rows_hard, std::max<size_t>((size_t)N * 4 / g.PW + 260, ((size_t)1 << 30) / (4 * g.TW)));
  const size_t lds_total = 160 * 1024;
  g.gcap = (uint32_t)((lds_total - mv_gather_fixed_bytes(g.BS)) / 8);
}

bool mv_supported(const MvGeom& g, uint32_t ASZP) {
  return mv_hist_bytes(g.nbins) + (size_t)g.PW * ASZP * 8 <= 160 * 1024 && mv_apply_lds_bytes(g.BS) <= 160 * 1024;
}

// Host-side slot groups (contiguous ranges of <= GW slots) and their tables.
void mv_build_groups(Engine& e, const std::vector<uint32_t>& origins, const std::vector<uint8_t>& obkt,
                     const std::vector<uint8_t>& bucket, std::vector<uint32_t>& gtab, std::vector<uint2>& seeds) {
  const uint32_t GW = e.mv.GW;
  const uint32_t ng = (e.S + GW - 1) / GW;
  gtab.assign((size_t)ng * GT_WORDS, 0);
  seeds.clear();
  e.mv_groups.clear();
  for (uint32_t g = 0; g < ng; ++g) {
    const uint32_t s0 = g * GW, sg = std::min(GW, e.S - s0);
    uint32_t* t = gtab.data() + (size_t)g * GT_WORDS;
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

static MvArgs mv_args(Engine& e, const MvGroup& gr, uint32_t g) {
  MvArgs a;
  a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.own = e.own; a.frank = e.frank; a.origin = e.origin;
  a.nfail = e.nfail; a.mask = e.mask; a.gt = e.mv_gtab + (size_t)g * GT_WORDS;
  a.hops = e.hops; a.cnt = e.cnt; a.inb = e.inb; a.egress = e.egress; a.err = e.err;
  a.vis = e.mv_vis; a.lvl = e.lvl; a.tb = e.mv_tb; a.T = e.mv_T; a.area = e.mv_area; a.ctr = e.mv_ctr;
  a.N = e.N; a.ASZ = e.ASZ; a.fanout = e.fanout; a.capin = e.capin; a.s0 = gr.s0; a.Sg = gr.sg;
  a.UB = e.mv.UB; a.BS = e.mv.BS; a.nbins = e.mv.nbins; a.TW = e.mv.TW; a.PW = e.mv.PW; a.ORW = e.ASZP + 4;
  a.any_fail = 0;
  for (uint32_t j = 0; j < gr.sg; ++j) a.any_fail |= e.h_nfail_any[gr.s0 + j] ? 1u : 0u;
  a.gcap = e.mv.gcap;
  a.PAIRS = e.PAIRS; a.area_cap = e.mv.area_cap; a.rows_cap = e.mv.rows_cap; a.q_cap = e.mv.q_cap;
  return a;
}

hipError_t launch_bfs_multi(Engine& e, bool /*record*/) {
  hipError_t r;
  const size_t lds_x = mv_hist_bytes(e.mv.nbins) + (size_t)e.mv.PW * e.ASZP * 8;
  const size_t lds_a = mv_apply_lds_bytes(e.mv.BS);
  const size_t lds_g = 160 * 1024;
  if (!e.mv_attr_set) {
    GS_ASZP_DISPATCH(e.ASZP, {
      if (e.mv.XPT == 2)
        r = hipFuncSetAttribute((const void*)k_mv_expand<A, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_x);
      else
        r = hipFuncSetAttribute((const void*)k_mv_expand<A, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_x);
    });
    if (r != hipSuccess) return r;
    if ((r = hipFuncSetAttribute((const void*)k_mv_apply, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a)))
      return r;
    if ((r = hipFuncSetAttribute((const void*)k_mv_gather, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_g)))
      return r;
    for (int i = 0; i < 4; ++i)
      if ((r = hipEventCreateWithFlags(&e.mv_ev[i], hipEventDisableTiming)) != hipSuccess) return r;
    e.mv_attr_set = true;
  }
  const uint32_t bgrid = ((e.mv.nbins + 7) / 8) * 8;
  const uint32_t xgrid = 512;
  volatile uint32_t* poll = e.h_err + 8;  // pinned
  for (uint32_t g = 0; g < (uint32_t)e.mv_groups.size(); ++g) {
    const MvGroup& gr = e.mv_groups[g];
    MvArgs a = mv_args(e, gr, g);
    if ((r = hipMemsetAsync(e.mv_vis, 0, (size_t)e.N * 4, e.st)) != hipSuccess) return r;
    if ((r = hipMemsetAsync(e.lvl, 0, 256 * 4, e.st)) != hipSuccess) return r;
    hipLaunchKernelGGL(k_mv_seed, dim3((gr.nseed + 255) / 256), dim3(256), 0, e.st, a, e.mv_seed + gr.seed0, gr.nseed,
                       e.mv_q[0]);
    uint32_t nlev = 0;
    for (uint32_t d = 0; d < 254; ++d) {
      GS_ASZP_DISPATCH(e.ASZP, {
        if (e.mv.XPT == 2)
          hipLaunchKernelGGL((k_mv_expand<A, 2>), dim3(xgrid), dim3(MV_XT), lds_x, e.st, a, d, e.mv_q[d & 1]);
        else
          hipLaunchKernelGGL((k_mv_expand<A, 1>), dim3(xgrid), dim3(MV_XT), lds_x, e.st, a, d, e.mv_q[d & 1]);
      });
      hipLaunchKernelGGL(k_mv_apply, dim3(bgrid), dim3(MV_AT), lds_a, e.st, a, d, e.mv_q[(d + 1) & 1]);
      // the next frontier's size, polled three levels late so the GPU never idles on the host
      if ((r = hipMemcpyAsync((void*)(poll + (d & 3)), e.lvl + d + 1, 4, hipMemcpyDeviceToHost, e.st))) return r;
      if ((r = hipEventRecord(e.mv_ev[d & 3], e.st))) return r;
      if (d >= 3) {
        if ((r = hipEventSynchronize(e.mv_ev[(d - 3) & 3]))) return r;
        if (poll[(d - 3) & 3] == 0) { nlev = d + 1; break; }
      }
    }
    if (!nlev) return hipErrorNotSupported;  // frontier still non-empty after 254 levels
    hipLaunchKernelGGL(k_mv_gather, dim3(bgrid), dim3(MV_GT), lds_g, e.st, a, nlev);
  }
  return hipGetLastError();
}

}  // namespace gs
