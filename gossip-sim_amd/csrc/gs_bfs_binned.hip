// gs_bfs_binned.hip -- Cluster::run_gossip (gossip.rs:494-615) for large clusters:
// level-synchronous BFS over every slot at once, propagation-blocked.
//
// The level kernel k_bfs_level updates a pair's in-degree with a global atomic
// per push. On gfx950 global atomics execute at the memory side; scattered ones
// (64 lanes, 64 rows) run ~17x below coalesced ones, so at 1M nodes that one
// atomic per push is the whole cost of the BFS. Here each level is two kernels
// and no push touches a global atomic:
//
//   expand (grid G): workgroup w owns a contiguous slice of the frontier. Pass 1
//     computes every frontier pair's push mask (the first `fanout` unpruned,
//     non-origin peers of its active-set entry; failed peers burn a slot) and
//     counts its pushes per destination bin (2^BS consecutive pairs) in LDS;
//     an exclusive scan turns the counts into the workgroup's per-bin segment
//     starts, published as T[b][w]. Pass 2 writes each push record
//     (destination pair, source node) into its bin segment of the workgroup's
//     area.
//   apply (one workgroup per bin): walks the bin's segments of every expand
//     workgroup. The bin's in-degree counters for THIS level live in LDS (u16),
//     so a record's arrival index is an LDS atomic; the record lands in inbound
//     slot cnt[q] + index; a pair's first arrival sets its hop and joins the
//     next frontier (collected in LDS, appended with one reservation). Finally
//     the bin's touched counters are added to cnt[] -- the bin owns its pairs,
//     so plain read-modify-writes suffice.
//
// Results are identical to k_bfs_level: hops, in-degree, the inbound record
// SETS per pair (consume sorts them by (hop, src)), egress, frontier sizes.
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

constexpr uint32_t BIN_THREADS = 256;

struct BinArgs {
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
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
  uint32_t* pm;     // push mask per frontier position (pass 1 -> pass 2)
  uint2* area;      // push records (pair, src) per expand workgroup
  uint32_t* T;      // [nbins + 1][G] segment starts (row nbins = workgroup totals)
  uint32_t N, ASZ, fanout, capin, G, BS, nbins, qmin;
  size_t PAIRS;
  int record;
};

__device__ inline void slice_of(uint32_t qn, uint32_t G, uint32_t w, uint32_t& lo, uint32_t& hi) {
  const uint32_t per = (qn + G - 1) / G;
  lo = min(qn, w * per);
  hi = min(qn, lo + per);
}

// the pushes of frontier pair p (gossip.rs:511-541): ring slots taken this round
template <int ASZP>
__device__ inline uint32_t pair_pushes(const BinArgs& a, uint32_t p, uint32_t (&row)[ASZP], uint32_t& o,
                                       uint32_t& u) {
  o = p / a.N;
  u = p - o * a.N;
  const uint32_t org = a.origin[o], nf = a.nfail[o];
  const uint32_t b = min((uint32_t)a.bucket[u], (uint32_t)a.obkt[o]);
  const uint32_t ent = u * NB + b;
  const uint32_t hv = a.hl[ent];
  load_row<ASZP>(a.peers + (size_t)ent * ASZP, row);
  uint32_t pushm = taken_slots<ASZP>(row, hv & 0xFF, hv >> 8, a.ASZ, a.mask[p], org, a.fanout);
  if (nf) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
    for (int s = 0; s < ASZP; ++s)
      if (((pushm >> s) & 1u) && a.frank[row[s]] < nf) pushm &= ~(1u << s);
  }
  return pushm;
}

constexpr uint32_t APPLY_THREADS = 256;
// Levels with fewer frontier pairs than this run k_bfs_level (a global atomic per
// push is cheap at that size; the binned pair of kernels has a fixed cost).
// (GS_FLAG_BINNED_ALL_LEVELS: 0, every level binned -- lets small tests cover the kernels.)
constexpr uint32_t BIN_MIN_FRONTIER = 1u << 17;

// Exclusive scan of LDS counts h[0..n) in place (whole workgroup of THREADS); returns the total.
template <uint32_t THREADS = BIN_THREADS>
__device__ inline uint32_t block_excl_scan(uint32_t* h, uint32_t n, uint32_t* wsum) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t per = (n + THREADS - 1) / THREADS;
  const uint32_t lo = min(n, tid * per), hi = min(n, lo + per);
  uint32_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += h[i];
  const uint32_t incl = wave_incl_scan(s);
  if (lane == 63) wsum[wid] = incl;
  __syncthreads();
  uint32_t wb = 0, tot = 0;
  for (uint32_t k = 0; k < THREADS / 64; ++k) {
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

template <int ASZP>
__global__ __launch_bounds__(BIN_THREADS) void k_bin_expand(BinArgs a, uint32_t d, const uint32_t* __restrict__ qcur) {
  extern __shared__ uint32_t hist[];  // [nbins] + 4 wave sums
  const uint32_t qn = a.lvl[d];
  if (qn < a.qmin || qn == 0) return;
  uint32_t lo, hi;
  slice_of(qn, a.G, blockIdx.x, lo, hi);
  if (lo >= hi) return;  // apply derives the same slices and skips this workgroup
  const uint32_t tid = threadIdx.x, w = blockIdx.x;
  const uint32_t nb = a.nbins, BS = a.BS;
  for (uint32_t i = tid; i < nb; i += BIN_THREADS) hist[i] = 0;
  __syncthreads();
  // pass 1: push masks, per-bin counts
  for (uint32_t i = lo + tid; i < hi; i += BIN_THREADS) {
    const uint32_t p = qcur[i];
    uint32_t row[ASZP], o, u;
    const uint32_t pushm = pair_pushes<ASZP>(a, p, row, o, u);
    a.pm[i] = pushm;
    const uint32_t eg = __popc(pushm);
    a.egress[p] = (uint8_t)eg;
    if (a.record && eg) a.egress_acc[p] += eg;
    const uint32_t qb = o * a.N;
#pragma unroll
    for (int s = 0; s < ASZP; ++s)
      if ((pushm >> s) & 1u) atomicAdd(&hist[(qb + row[s]) >> BS], 1u);
  }
  __syncthreads();
  const uint32_t total = block_excl_scan(hist, nb, hist + nb);
  for (uint32_t b = tid; b < nb; b += BIN_THREADS) a.T[(size_t)b * a.G + w] = hist[b];
  if (tid == 0) a.T[(size_t)nb * a.G + w] = total;
  __syncthreads();  // every segment start is published before pass 2 advances them
  // pass 2: records into the bin segments of this workgroup's area
  uint2* area = a.area + (size_t)lo * min(a.fanout, a.ASZ);
  for (uint32_t i = lo + tid; i < hi; i += BIN_THREADS) {
    const uint32_t p = qcur[i];
    const uint32_t pushm = a.pm[i];
    const uint32_t o = p / a.N, u = p - o * a.N;
    const uint32_t b = min((uint32_t)a.bucket[u], (uint32_t)a.obkt[o]);
    uint32_t row[ASZP];
    load_row<ASZP>(a.peers + (size_t)(u * NB + b) * ASZP, row);
    const uint32_t qb = o * a.N;
#pragma unroll
    for (int s = 0; s < ASZP; ++s)
      if ((pushm >> s) & 1u) {
        const uint32_t q = qb + row[s];
        const uint32_t pos = atomicAdd(&hist[q >> BS], 1u);
        area[pos] = make_uint2(q, u);
      }
  }
}

// LDS of the apply kernel: segment prefix [G + 1], segment starts [G], the bin's
// counters [BP] (u32 in-degrees when staged, else packed u16 arrival indices),
// first arrivals u16 [BP], control words.
__host__ __device__ inline size_t bin_apply_lds_words(uint32_t G, uint32_t BS) {
  return 2 * (size_t)G + 1 + ((size_t)1 << BS) + ((size_t)1 << BS) / 2 + 24;
}

__global__ __launch_bounds__(APPLY_THREADS) void k_bin_apply(BinArgs a, uint32_t d, uint32_t* __restrict__ qnxt) {
  extern __shared__ uint32_t smem[];
  const uint32_t qn = a.lvl[d];
  if (qn < a.qmin || qn == 0) return;
  const uint32_t tid = threadIdx.x, G = a.G;
  const uint32_t b = blockIdx.x, BP = 1u << a.BS;
  uint32_t* pre = smem;                                          // [G + 1]
  uint32_t* sb = pre + G + 1;                                    // [G]
  uint32_t* cw = sb + G;                                         // [BP]
  uint16_t* fl = reinterpret_cast<uint16_t*>(cw + BP);           // [BP]
  uint32_t* ctl = cw + BP + BP / 2;                              // [0] first arrivals, [1] base, [2] overflow, [4..19] scan
  // 1. this bin's segment in every expand workgroup's area
  for (uint32_t w = tid; w < G; w += APPLY_THREADS) {
    uint32_t lo, hi, sz = 0, st = 0;
    slice_of(qn, G, w, lo, hi);
    if (lo < hi) {
      st = a.T[(size_t)b * G + w];
      sz = a.T[(size_t)(b + 1) * G + w] - st;
    }
    pre[w] = sz;
    sb[w] = st;
  }
  if (tid < 3) ctl[tid] = 0;
  __syncthreads();
  const uint32_t total = block_excl_scan<APPLY_THREADS>(pre, G, ctl + 4);
  if (tid == 0) pre[G] = total;
  const uint32_t q0 = b << a.BS;
  const uint32_t qend = (uint32_t)min((size_t)q0 + BP, a.PAIRS);
  // 2. counters: a busy bin stages its in-degrees (one coalesced read and write);
  //    a quiet one keeps per-level arrival indices and reads cnt[] per record
  const bool staged = total >= BP / 4;
  if (staged) {
    for (uint32_t i = tid; i < BP; i += APPLY_THREADS) cw[i] = q0 + i < qend ? a.cnt[q0 + i] : 0u;
  } else {
    for (uint32_t i = tid; i < BP / 2; i += APPLY_THREADS) cw[i] = 0;
  }
  __syncthreads();
  const uint32_t fc = min(a.fanout, a.ASZ);
  const uint32_t hop = d + 1;
  bool overflow = false;
  // 3. one thread per record
  for (uint32_t r = tid; r < total; r += APPLY_THREADS) {
    uint32_t lo = 0, hi = G;  // largest w with pre[w] <= r (a non-empty segment)
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= r) lo = mid; else hi = mid;
    }
    const uint32_t w = lo;
    uint32_t wlo, whi;
    slice_of(qn, G, w, wlo, whi);
    const uint2 rec = a.area[(size_t)wlo * fc + sb[w] + (r - pre[w])];
    const uint32_t q = rec.x, ql = q - q0;
    uint32_t slot;
    if (staged) {
      slot = atomicAdd(&cw[ql], 1u);
    } else {
      const uint32_t sh = (ql & 1u) << 4;
      const uint32_t k = (atomicAdd(&cw[ql >> 1], 1u << sh) >> sh) & 0xFFFFu;
      slot = a.cnt[q] + k;
    }
    if (slot < a.capin) a.inb[(size_t)slot * a.PAIRS + q] = (hop << 24) | rec.y;
    else overflow = true;
    if (slot == 0) {  // first arrival: hop = dist[src] + 1 (gossip.rs:594-600)
      a.hops[q] = (uint8_t)hop;
      fl[atomicAdd(&ctl[0], 1u)] = (uint16_t)ql;
    }
  }
  if (overflow) ctl[2] = 1;
  __syncthreads();
  const uint32_t nf = ctl[0];
  if (tid == 0 && nf) ctl[1] = atomicAdd(&a.lvl[d + 1], nf);
  if (tid == 0 && ctl[2]) atomicOr(a.err, ERR_INBOUND);
  // 4. the bin's in-degrees after this level
  if (staged) {
    for (uint32_t i = tid; q0 + i < qend; i += APPLY_THREADS) a.cnt[q0 + i] = cw[i];
  } else {
    for (uint32_t ql = 2 * tid; q0 + ql < qend; ql += 2 * APPLY_THREADS) {
      const uint32_t c2 = cw[ql >> 1];
      if (!c2) continue;
      if (c2 & 0xFFFFu) a.cnt[q0 + ql] += c2 & 0xFFFFu;
      if ((c2 >> 16) && q0 + ql + 1 < qend) a.cnt[q0 + ql + 1] += c2 >> 16;
    }
  }
  __syncthreads();
  // 5. first arrivals join the next frontier
  const uint32_t base = ctl[1];
  for (uint32_t i = tid; i < nf; i += APPLY_THREADS) qnxt[base + i] = q0 + fl[i];
}

__global__ void k_bin_seed(BinArgs a, const uint32_t* __restrict__ origin, uint32_t S, uint32_t* q0) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= S) return;
  const size_t p = (size_t)o * a.N + origin[o];
  a.hops[p] = 0;
  q0[o] = (uint32_t)p;
  if (o == 0) a.lvl[0] = S;
}


hipError_t launch_bfs_binned(Engine& e, bool record) {
  BinArgs a;
  a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.frank = e.frank; a.origin = e.origin; a.obkt = e.obkt;
  a.nfail = e.nfail; a.mask = e.mask; a.hops = e.hops; a.cnt = e.cnt; a.inb = e.inb; a.egress = e.egress;
  a.egress_acc = e.egress_acc; a.lvl = e.lvl; a.err = e.err; a.pm = e.bin_pm; a.area = e.bin_area;
  a.T = e.bin_T; a.N = e.N; a.ASZ = e.ASZ; a.fanout = e.fanout; a.capin = e.capin; a.G = e.bin_G;
  a.BS = e.bin_BS; a.nbins = e.bin_nb; a.PAIRS = e.PAIRS; a.record = record ? 1 : 0;
  a.qmin = (e.prm.flags & GS_FLAG_BINNED_ALL_LEVELS) ? 0u : BIN_MIN_FRONTIER;
  hipError_t r;
  if ((r = hipMemsetAsync(e.hops, 0xFF, e.PAIRS, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.cnt, 0, e.PAIRS * 4, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.lvl, 0, 256 * 4, e.st)) != hipSuccess) return r;
  hipLaunchKernelGGL(k_bin_seed, dim3((e.S + 255) / 256), dim3(256), 0, e.st, a, e.origin, e.S, e.q[0]);
  const size_t lds_x = ((size_t)e.bin_nb + 4) * 4;
  const size_t lds_a = bin_apply_lds_words(e.bin_G, e.bin_BS) * 4;
  r = hipFuncSetAttribute((const void*)k_bin_apply, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a);
  if (r != hipSuccess) return r;
  for (uint32_t d = 0; d < 254; ++d) {
    if (a.qmin && (r = launch_bfs_level_step(e, record, d, 0, a.qmin)) != hipSuccess) return r;
    GS_ASZP_DISPATCH(e.ASZP, {
      r = hipFuncSetAttribute((const void*)k_bin_expand<A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_x);
      if (r != hipSuccess) return r;
      hipLaunchKernelGGL(k_bin_expand<A>, dim3(e.bin_G), dim3(BIN_THREADS), lds_x, e.st, a, d, e.q[d & 1]);
    });
    hipLaunchKernelGGL(k_bin_apply, dim3(e.bin_nb), dim3(APPLY_THREADS), lds_a, e.st, a, d, e.q[(d + 1) & 1]);
    if ((d & 3) == 3) {  // poll the frontier size every 4 levels
      uint32_t* h = e.h_err + 1;
      if ((r = hipMemcpyAsync(h, e.lvl + d + 1, 4, hipMemcpyDeviceToHost, e.st)) != hipSuccess) return r;
      if ((r = hipStreamSynchronize(e.st)) != hipSuccess) return r;
      if (*h == 0) return hipGetLastError();
    }
  }
  return hipErrorNotSupported;  // frontier still non-empty after 254 levels: hop counts no longer fit u8
}

}  // namespace gs
