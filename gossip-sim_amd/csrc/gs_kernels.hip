// gs_kernels.hip -- gfx950 kernels of the push-propagation engine.
//
// Kernel map (reference function each one restates):
//   k_prefix_weights   rotation weights (push_active_set.rs:97-111) as prefix sums
//   k_init_entries     PushActiveSet::rotate on empty entries (push_active_set.rs:73-114,153-187)
//   k_rotate_*         Cluster::chance_to_rotate -> Node::rotate_active_set (gossip.rs:739-754,815-842)
//   k_bfs_wg           Cluster::run_gossip (gossip.rs:494-615), one workgroup per slot, LDS frontier
//   k_bfs_level        Cluster::run_gossip, level-synchronous over all slots (large N)
//   k_consume_prune    consume_messages + ReceivedCache::record/prune + send_prunes +
//                      prune_connections (gossip.rs:618-737, received_cache.rs:27-131)
//   k_stats_*          the measured-round statistics inserts (gossip_main.rs:480-563)
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

static inline uint32_t grid_for(size_t n, uint32_t block, uint32_t cap = 1u << 20) {
  size_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (uint32_t)g;
}

// -------------------------------------------------------------- weights ----
__global__ __launch_bounds__(1024) void k_prefix_weights(const uint8_t* __restrict__ bucket, uint64_t* __restrict__ P,
                                                        uint32_t N) {
  const int k = blockIdx.x;
  uint64_t* Pk = P + (size_t)k * (N + 1);
  const uint32_t T = blockDim.x, t = threadIdx.x;
  const uint32_t chunk = (N + T - 1) / T;
  const uint32_t lo = min(N, t * chunk), hi = min(N, lo + chunk);
  uint64_t s = 0;
  for (uint32_t i = lo; i < hi; ++i) s += weight(k, bucket[i]);
  __shared__ uint64_t part[1024];
  part[t] = s;
  __syncthreads();
  for (uint32_t off = 1; off < T; off <<= 1) {
    uint64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = part[t] - s;
  if (t == 0) Pk[0] = 0;
  for (uint32_t i = lo; i < hi; ++i) {
    run += weight(k, bucket[i]);
    Pk[i + 1] = run;
  }
}

// The index table of each entry k's prefix sums (prefix_search_ix): IX[k][j] = the
// smallest c with P[c + 1] > floor(total * j / 2^L), j = 0 .. 2^L.
__global__ void k_build_ix(const uint64_t* __restrict__ P, uint32_t N, uint32_t* __restrict__ IX) {
  const uint32_t L = ix_log(N), m = ix_count(N);
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < (uint32_t)NB * m; g += gridDim.x * blockDim.x) {
    const uint32_t k = g / m, j = g - k * m;
    const uint64_t* Pk = P + (size_t)k * (N + 1);
    const uint64_t x = (Pk[N] * (uint64_t)j) >> L;
    IX[g] = prefix_search(Pk, N, x);
  }
}

hipError_t launch_prefix_weights(Engine& e) {
  hipLaunchKernelGGL(k_prefix_weights, dim3(NB), dim3(1024), 0, e.st, e.bucket, e.P, e.N);
  hipLaunchKernelGGL(k_build_ix, dim3(grid_for((size_t)NB * ix_count(e.N), 256, 4096)), dim3(256), 0, e.st, e.P, e.N,
                     e.IX);
  return hipGetLastError();
}

// ------------------------------------------------------------ init (R6) ----
// One thread per entry (u, k). From an empty entry the reference appends fresh
// shuffle draws until len > size, then drops the oldest: the entry keeps draws
// 2..size+1 (or every candidate when N - 1 <= size).
template <int ASZP>
__global__ __launch_bounds__(256) void k_init_entries(const uint8_t* __restrict__ bucket,
                                                     const uint64_t* __restrict__ P, const uint32_t* __restrict__ IX,
                                                     uint32_t* __restrict__ peers,
                                                     uint16_t* __restrict__ hl, uint32_t N, uint32_t size,
                                                     uint64_t seed) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= N * NB) return;
  const uint32_t u = gid / NB, k = gid % NB;
  const uint64_t* Pk = P + (size_t)k * (N + 1);
  const uint32_t L = ix_log(N);
  const uint32_t* IXk = IX + (size_t)k * ix_count(N);
  constexpr int R = ASZP + 2;
  uint32_t rem[R];
  uint64_t remw[R];
  int nr = 0;
  const uint64_t wself = weight(k, bucket[u]);
  rem_insert(rem, remw, nr, u, wself);
  const uint64_t total = Pk[N];
  uint64_t left = total - wself;
  const uint32_t ncand = N - 1;
  const uint32_t T = min(ncand, size + 1);
  const bool drop = ncand >= size + 1;
  Philox s(seed, P_INIT, u, k);
  uint32_t* row = peers + (size_t)gid * ASZP;
  uint32_t filled = 0;
  for (uint32_t t = 0; t < T; ++t) {
    const uint64_t v = sample_below(left, s);
    const uint32_t c = shuffle_pick(Pk, IXk, L, total, v, rem, remw, nr);
    const uint64_t wc = weight(k, bucket[c]);
    left -= wc;
    rem_insert(rem, remw, nr, c, wc);
    if (!(t == 0 && drop)) row[filled++] = c;
  }
  hl[gid] = (uint16_t)(filled << 8);
}

hipError_t launch_init_entries(Engine& e) {
  const uint32_t total = e.N * NB;
  e.rows2_stale = true;
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_init_entries<A>, dim3(grid_for(total, 256)), dim3(256), 0, e.st,
                                              e.bucket, e.P, e.IX, e.peers, e.hl, e.N, e.ASZ, e.prm.seed));
  hipError_t r = hipGetLastError();
  return r != hipSuccess ? r : launch_own_rows(e, nullptr, nullptr);
}

// ------------------------------------------------------------ fail (R15) ----
__global__ void k_fail_keys(uint32_t N, uint64_t seed, uint64_t* keys, uint32_t* ids) {
  const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= N) return;
  Philox s(seed, P_FAIL, v, 0);
  keys[v] = s.next();
  ids[v] = v;
}
hipError_t launch_fail_keys(Engine& e, uint64_t* keys, uint32_t* ids) {
  hipLaunchKernelGGL(k_fail_keys, dim3(grid_for(e.N, 256)), dim3(256), 0, e.st, e.N, e.prm.seed, keys, ids);
  return hipGetLastError();
}
__global__ void k_scatter_rank(uint32_t N, const uint32_t* sorted_ids, uint32_t* rank) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N) rank[sorted_ids[i]] = i;
}
hipError_t launch_scatter_rank(Engine& e, const uint32_t* sorted_ids, uint32_t* rank_out) {
  hipLaunchKernelGGL(k_scatter_rank, dim3(grid_for(e.N, 256)), dim3(256), 0, e.st, e.N, sorted_ids, rank_out);
  return hipGetLastError();
}

__global__ void k_clear_slot_masks(size_t mso, size_t msu, uint32_t S, uint32_t node, uint32_t bucket_k,
                                   const uint8_t* __restrict__ bucket, const uint8_t* __restrict__ obkt,
                                   uint32_t bits, uint32_t* mask) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= S) return;
  const uint32_t b = min((uint32_t)bucket[node], (uint32_t)obkt[o]);
  if (b == bucket_k) mask[o * mso + node * msu] &= ~bits;
}
hipError_t launch_clear_slot_masks(Engine& e, uint32_t node, uint32_t bucket_k, uint32_t bits) {
  hipLaunchKernelGGL(k_clear_slot_masks, dim3(grid_for(e.S, 256)), dim3(256), 0, e.st, e.mso, e.msu, e.S, node,
                     bucket_k, e.bucket, e.obkt, bits, e.mask);
  return hipGetLastError();
}

// ---------------------------------------------------------- rotation (R14) ----
// Each block decides a contiguous node range and appends its rotating nodes with ONE
// global atomic (rotation is per node and order-free: rot_list order does not matter).
__global__ __launch_bounds__(1024) void k_rotate_decide(uint32_t N, uint64_t seed, uint32_t round, double p,
                                                       uint32_t* rot_list, uint32_t* rot_count,
                                                       uint32_t* rot_count_other) {
  __shared__ uint32_t lcount, lbase;
  __shared__ uint32_t lids[2048];
  if (blockIdx.x == 0 && threadIdx.x == 0) *rot_count_other = 0;  // the next rotation's counter
  const uint32_t per = (N + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = min(N, blockIdx.x * per), hi = min(N, lo + per);
  for (uint32_t c0 = lo; c0 < hi; c0 += 2048) {  // chunks of at most 2048 nodes fit the LDS list
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    for (uint32_t u = c0 + threadIdx.x; u < min(hi, c0 + 2048); u += blockDim.x) {
      Philox s(seed, P_DECIDE, u, round);
      if (unit_f64(s.next()) < p) lids[atomicAdd(&lcount, 1u)] = u;
    }
    __syncthreads();
    const uint32_t n = lcount;
    if (threadIdx.x == 0 && n) lbase = atomicAdd(rot_count, n);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) rot_list[lbase + i] = lids[i];
    __syncthreads();
  }
}

template <int ASZP>
__global__ __launch_bounds__(256) void k_rotate_entries(const uint8_t* __restrict__ bucket,
                                                       const uint64_t* __restrict__ P, const uint32_t* __restrict__ IX,
                                                       uint32_t* __restrict__ peers,
                                                       uint16_t* __restrict__ hl, const uint32_t* __restrict__ rot_list,
                                                       const uint32_t* __restrict__ rot_count,
                                                       uint32_t* __restrict__ rot_changed, uint32_t N, uint32_t size,
                                                       uint64_t seed, uint32_t round) {
  const uint32_t total = *rot_count * NB;
  for (uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x; gid < total; gid += gridDim.x * blockDim.x)
    rotate_entry<ASZP>(bucket, P, IX, peers, hl, rot_list, rot_changed, N, size, seed, round, gid);
}

// Small clusters (N <= RS_MAX): decide and rotate in ONE workgroup, one launch instead of two
// (a dependent launch costs several us against ~5 us of work at C2's 3,000 nodes).
constexpr uint32_t RS_MAX = 16384;
template <int ASZP>
__global__ __launch_bounds__(1024) void k_rotate_small(const uint8_t* __restrict__ bucket,
                                                      const uint64_t* __restrict__ P, const uint32_t* __restrict__ IX,
                                                      uint32_t* __restrict__ peers, uint16_t* __restrict__ hl,
                                                      uint32_t* __restrict__ rot_list, uint32_t* __restrict__ rot_count,
                                                      uint32_t* __restrict__ rot_count_other,
                                                      uint32_t* __restrict__ rot_changed, uint32_t N, uint32_t size,
                                                      uint64_t seed, uint32_t round, double p) {
  __shared__ uint32_t lcount, base0;
  if (threadIdx.x == 0) {
    *rot_count_other = 0;  // the next rotation's counter
    lcount = 0;
    base0 = *rot_count;    // (zero unless a repeated round index appends)
  }
  __syncthreads();
  for (uint32_t u = threadIdx.x; u < N; u += blockDim.x) {  // DECIDE (gossip.rs:739-754), order-free
    Philox s(seed, P_DECIDE, u, round);
    if (unit_f64(s.next()) < p) rot_list[base0 + atomicAdd(&lcount, 1u)] = u;
  }
  __syncthreads();
  const uint32_t n = base0 + lcount;
  if (threadIdx.x == 0) *rot_count = n;
  __threadfence_block();  // (this workgroup's rot_list stores before its entries read them)
  for (uint32_t gid = threadIdx.x; gid < n * NB; gid += blockDim.x)
    rotate_entry<ASZP>(bucket, P, IX, peers, hl, rot_list, rot_changed, N, size, seed, round, gid);
}

// Larger clusters: decide, rotate and refresh the own rows in ONE launch instead of three
// (k_rotate_decide, k_rotate_entries, k_own_rows: ~12 us of dependent launches per round at
// C3's 100k nodes). Each 256-thread block takes RF_NODES consecutive nodes (two per
// thread), lists its rotating nodes in LDS, appends them to rot_list with one atomic,
// rotates their entries (one (node, entry) per thread: p x NB ~ 0.33 entries per node, so
// ~170 per block) and then rewrites their own rows -- everything a block touches is its own
// nodes' rows, so no grid-wide ordering is needed.
constexpr uint32_t RF_THREADS = 256;
constexpr uint32_t RF_NODES = 512;
template <int ASZP>
__global__ __launch_bounds__(RF_THREADS) void k_rotate_fused(const uint8_t* __restrict__ bucket,
                                                            const uint64_t* __restrict__ P, const uint32_t* __restrict__ IX,
                                                            uint32_t* __restrict__ peers, uint16_t* __restrict__ hl,
                                                            uint32_t* __restrict__ rot_list, uint32_t* __restrict__ rot_count,
                                                            uint32_t* __restrict__ rot_count_other,
                                                            uint32_t* __restrict__ rot_changed, uint32_t N, uint32_t size,
                                                            uint64_t seed, uint32_t round, double p, uint32_t ORW,
                                                            const uint8_t* __restrict__ fcls, uint32_t* __restrict__ own) {
  __shared__ uint32_t lids[RF_NODES], lcount, lbase;
  if (blockIdx.x == 0 && threadIdx.x == 0) *rot_count_other = 0;  // the next rotation's counter
  if (threadIdx.x == 0) lcount = 0;
  __syncthreads();
  const uint32_t lo = blockIdx.x * RF_NODES, hi = min(N, lo + RF_NODES);
  for (uint32_t u = lo + threadIdx.x; u < hi; u += RF_THREADS) {  // DECIDE (gossip.rs:739-754), order-free
    Philox s(seed, P_DECIDE, u, round);
    if (unit_f64(s.next()) < p) lids[atomicAdd(&lcount, 1u)] = u;
  }
  __syncthreads();
  const uint32_t n = lcount;
  if (n == 0) return;  // (block-uniform)
  if (threadIdx.x == 0) lbase = atomicAdd(rot_count, n);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += RF_THREADS) rot_list[lbase + i] = lids[i];
  for (uint32_t gid = threadIdx.x; gid < n * NB; gid += RF_THREADS)  // (rotate_entry reads the LDS list)
    rotate_entry<ASZP>(bucket, P, IX, peers, hl, lids, rot_changed, N, size, seed, round, gid);
  if (!own) return;
  __syncthreads();  // (the block's entry rows and ring heads are written before its own rows read them)
  for (uint32_t i = threadIdx.x; i < n; i += RF_THREADS) own_row<ASZP>(bucket, peers, hl, ORW, fcls, own, lids[i]);
}

// A replaced peer gets a fresh filter: clear its ring slot's prune bit for every
// slot whose origin uses that entry.
__global__ void k_rotate_clear(size_t mso, size_t msu, uint32_t S, const uint8_t* __restrict__ bucket,
                               const uint8_t* __restrict__ obkt, const uint32_t* __restrict__ rot_list,
                               const uint32_t* __restrict__ rot_count, const uint32_t* __restrict__ rot_changed,
                               uint32_t* __restrict__ mask) {
  const uint32_t total = *rot_count * S;
  for (uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x; gid < total; gid += gridDim.x * blockDim.x) {
    const uint32_t i = gid / S, o = gid - i * S;
    const uint32_t u = rot_list[i];
    const uint32_t b = min((uint32_t)bucket[u], (uint32_t)obkt[o]);
    const uint32_t m = rot_changed[u * NB + b];
    if (m) mask[o * mso + u * msu] &= ~m;
  }
}

hipError_t launch_rotate_clear(Engine& e) {
  hipLaunchKernelGGL(k_rotate_clear, dim3(grid_for((size_t)e.N * e.S, 256, 2048)), dim3(256), 0, e.st, e.mso, e.msu, e.S,
                     e.bucket, e.obkt, e.rot_list, e.rot_count + e.rot_parity, e.rot_changed, e.mask);
  return hipGetLastError();
}

hipError_t launch_rotate(Engine& e, uint32_t round, bool defer_clear) {
  // GS_ROT_SPLIT=1: the three-launch rotation (decide, entries, own rows) for N > RS_MAX
  static const bool rot_split = std::getenv("GS_ROT_SPLIT") && std::getenv("GS_ROT_SPLIT")[0] == '1';
  const uint32_t par = round & 1u;
  uint32_t* cnt = e.rot_count + par;
  e.rows2_stale = true;  // (the rows change in place: a later ahead rotation copies them whole first)
  if (e.rot_cnt_dirty || (e.rot_have_prev && par == e.rot_parity)) {  // not pre-zeroed (rounds not
                                                                      // consecutive, or after an ahead rotation)
    e.rot_cnt_dirty = false;
    hipError_t r = hipMemsetAsync(cnt, 0, sizeof(uint32_t), e.st);
    if (r != hipSuccess) return r;
  }
  if (e.N <= RS_MAX) {
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_rotate_small<A>, dim3(1), dim3(1024), 0, e.st, e.bucket, e.P, e.IX,
                                                e.peers, e.hl, e.rot_list, cnt, e.rot_count + (par ^ 1u),
                                                e.rot_changed, e.N, e.ASZ, e.prm.seed, round,
                                                e.prm.rotation_probability));
  } else if (!rot_split) {
    const uint32_t grid = (e.N + RF_NODES - 1) / RF_NODES;
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_rotate_fused<A>, dim3(grid), dim3(RF_THREADS), 0, e.st, e.bucket,
                                                e.P, e.IX, e.peers, e.hl, e.rot_list, cnt, e.rot_count + (par ^ 1u),
                                                e.rot_changed, e.N, e.ASZ, e.prm.seed, round,
                                                e.prm.rotation_probability, e.ORW, e.mv_fcls, e.own));
  } else {
    hipLaunchKernelGGL(k_rotate_decide, dim3(grid_for(e.N, 4096, 256)), dim3(1024), 0, e.st, e.N, e.prm.seed, round,
                       e.prm.rotation_probability, e.rot_list, cnt, e.rot_count + (par ^ 1u));
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_rotate_entries<A>, dim3(grid_for((size_t)e.N * NB, 256, 2048)),
                                                dim3(256), 0, e.st, e.bucket, e.P, e.IX, e.peers, e.hl, e.rot_list,
                                                cnt, e.rot_changed, e.N, e.ASZ, e.prm.seed, round));
  }
  if (e.N <= RS_MAX || rot_split) {  // (the fused kernel refreshed its nodes' own rows itself)
    hipError_t ro = launch_own_rows(e, e.rot_list, cnt);
    if (ro != hipSuccess) return ro;
  }
  e.rot_parity = par;
  e.rot_have_prev = true;
  e.rot_clear_pending = true;
  if (defer_clear) return hipGetLastError();
  e.rot_clear_pending = false;
  return launch_rotate_clear(e);
}

// ------------------------------------------------------------- BFS (R8) ----
struct BfsArgs {
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
  uint32_t* lvl;
  uint32_t* err;
  // measured-round accumulation (record != 0)
  uint32_t* egress_acc;
  const uint64_t* stake;
  const uint32_t* srank;
  uint32_t* strand;
  uint32_t* bm;
  uint32_t* rs_u32;
  uint64_t* rs_ssum;
  uint32_t* rs_hist;
  uint32_t W;
  int record;
  uint32_t N, S, ASZ, fanout, capin;
  size_t PAIRS;
};


// Expands one frontier node u of slot o at level d (Cluster::run_gossip body,
// gossip.rs:511-609), in three phases so that no memory round trip waits on
// another: (1) every in-degree atomic of the node's pushes is issued back to
// back; (2) their results are used: the (hop, src) record, first-visit hop;
// (3) the newly visited peers are appended to the next frontier with ONE
// wave-aggregated reservation. `valid` lanes expand; the rest only join the
// wave collectives. CNT/HOPS index by peer (LDS tables, or global + base).
template <int ASZP, class QT, bool LDS_TAIL>
__device__ inline uint32_t expand_node(const BfsArgs& a, bool valid, uint32_t u, uint32_t ob, uint32_t org,
                                       uint32_t nf, uint32_t pmask, size_t base, uint32_t d, uint32_t* cntp,
                                       uint8_t* hopsp, QT* nxt, uint32_t* tail, size_t qoff, bool& overflow) {
  uint32_t row[ASZP];
  uint32_t pushm = 0;
  if (valid && GS_OOB(u, a.N, a.err, "expand u")) valid = false;
  if (valid) {
    const uint32_t b = min((uint32_t)a.bucket[u], ob);
    const uint32_t ent = u * NB + b;
    const uint32_t hv = a.hl[ent];
    load_row<ASZP>(a.peers + (size_t)ent * ASZP, row);
    pushm = taken_slots<ASZP>(row, hv & 0xFF, hv >> 8, a.ASZ, pmask, org, a.fanout);
#ifdef GS_DEBUG_BOUNDS
    for (int s = 0; s < ASZP; ++s)
      if (((pushm >> s) & 1u) && GS_OOB(row[s], a.N, a.err, "expand peer")) pushm &= ~(1u << s);
#endif
    if (nf) {  // failed peers burn their fanout slot (gossip.rs:538-541)
#pragma unroll
      for (int s = 0; s < ASZP; ++s)
        if (((pushm >> s) & 1u) && a.frank[row[s]] < nf) pushm &= ~(1u << s);
    }
  } else {
#pragma unroll
    for (int s = 0; s < ASZP; ++s) row[s] = 0;
  }
  uint32_t old[ASZP];
#pragma unroll
  for (int s = 0; s < ASZP; ++s) old[s] = ((pushm >> s) & 1u) ? atomicAdd(&cntp[row[s]], 1u) : 1u;
  asm volatile("" ::: "memory");
  const uint32_t rec = ((d + 1) << 24) | u;
  uint32_t newm = 0;
#pragma unroll
  for (int s = 0; s < ASZP; ++s) {
    if (!((pushm >> s) & 1u)) continue;
    if (old[s] < a.capin) a.inb[(size_t)old[s] * a.PAIRS + base + row[s]] = rec;
    else overflow = true;
    if (old[s] == 0) {
      newm |= 1u << s;
      hopsp[row[s]] = (uint8_t)(d + 1);
    }
  }
  const uint32_t k = __popc(newm);
  uint32_t idx;
  if (LDS_TAIL) {  // LDS counter: one per-lane atomic is a single round trip
    idx = k ? atomicAdd(tail, k) : 0;
  } else {         // global counter: one atomic per wave after a wave prefix sum
    const uint32_t incl = wave_incl_scan(k);
    const uint32_t total = (uint32_t)__shfl((int)incl, 63);
    uint32_t qb = 0;
    if (lane_id() == 0 && total) qb = atomicAdd(tail, total);
    idx = (uint32_t)__shfl((int)qb, 0) + incl - k;
  }
#pragma unroll
  for (int s = 0; s < ASZP; ++s)
    if ((newm >> s) & 1u) {
      if (GS_OOB(idx, LDS_TAIL ? a.N : a.PAIRS, a.err, "queue idx")) continue;
      nxt[idx++] = (QT)(qoff + row[s]);
    }
  return __popc(pushm);
}

// Workgroup-per-slot BFS: hop table, in-degree counters, egress and both
// frontier queues live in LDS (10 bytes per node), so the level loop needs
// workgroup barriers only. First visit = the in-degree atomic returning 0.
template <int ASZP>
__global__ __launch_bounds__(256) void k_bfs_wg(BfsArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t N = a.N;
  // [0] frontier size, [1] next size, [2] err, [4..6] visited/pushes/stranded, [8..9] stranded stake (u64)
  uint32_t* ctrl = reinterpret_cast<uint32_t*>(smem);
  unsigned long long* ssum_l = reinterpret_cast<unsigned long long*>(ctrl + 8);
  uint32_t* hist_l = ctrl + 16;
  uint32_t* cnt_l = hist_l + 256;
  uint8_t* hops_l = reinterpret_cast<uint8_t*>(cnt_l + N);
  uint8_t* eg_l = hops_l + ((N + 3) & ~3u);
  uint16_t* q0 = reinterpret_cast<uint16_t*>(eg_l + ((N + 3) & ~3u));
  uint16_t* q1 = q0 + ((N + 1) & ~1u);
  const uint32_t tid = threadIdx.x, bd = blockDim.x;
  for (uint32_t o = blockIdx.x; o < a.S; o += gridDim.x) {
    const uint32_t org = a.origin[o];
    const uint32_t ob = a.obkt[o];
    const uint32_t nf = a.nfail[o];
    const size_t base = (size_t)o * N;
    for (uint32_t v = tid; v < N; v += bd) { cnt_l[v] = 0; hops_l[v] = 0xFF; eg_l[v] = 0; }
    for (uint32_t i = tid; i < 256; i += bd) hist_l[i] = 0;
    __syncthreads();
    if (tid == 0) {
      ctrl[0] = 1; ctrl[1] = 0; ctrl[2] = 0; ctrl[4] = 0; ctrl[5] = 0; ctrl[6] = 0; *ssum_l = 0;
      hops_l[org] = 0; q0[0] = (uint16_t)org;
    }
    __syncthreads();
    uint16_t* cur = q0;
    uint16_t* nxt = q1;
    bool overflow = false;
    for (uint32_t d = 0;; ++d) {
      const uint32_t qn = ctrl[0];
      if (qn == 0) break;
      if (d + 1 >= 255) { if (tid == 0) atomicOr(a.err, ERR_DEPTH); break; }
      for (uint32_t i0 = 0; i0 < qn; i0 += bd) {  // uniform trip count: whole waves stay active
        const bool valid = i0 + tid < qn;
        const uint32_t u = valid ? cur[i0 + tid] : 0;
        const uint32_t pm = valid ? a.mask[base + u] : 0;
        const uint32_t pushes =
            expand_node<ASZP, uint16_t, true>(a, valid, u, ob, org, nf, pm, base, d, cnt_l, hops_l, nxt, &ctrl[1], 0,
                                        overflow);
        if (valid) eg_l[u] = (uint8_t)pushes;
      }
      __syncthreads();
      if (tid == 0) { ctrl[0] = ctrl[1]; ctrl[1] = 0; }
      uint16_t* t = cur; cur = nxt; nxt = t;
      __syncthreads();
    }
    if (overflow) ctrl[2] = 1;
    uint32_t vis = 0, pushes = 0, sc = 0;
    uint64_t ss = 0;
    for (uint32_t v = tid; v < N; v += bd) {
      const uint32_t h = hops_l[v], c = cnt_l[v], eg = eg_l[v];
      a.hops[base + v] = (uint8_t)h;
      a.cnt[base + v] = c;
      a.egress[base + v] = (uint8_t)eg;
      if (a.record) {  // the measured-round statistics, fused (gossip_main.rs:480-514)
        pushes += c;
        if (eg) a.egress_acc[base + v] += eg;
        if (h != 0xFF) {
          ++vis;
          atomicAdd(&hist_l[h], 1u);
        } else if (!(nf && a.frank[v] < nf)) {
          a.strand[base + v] += 1;
          ++sc;
          ss += a.stake[v];
          const uint32_t r = a.srank[v];
          atomicOr(&a.bm[(size_t)o * a.W + (r >> 5)], 1u << (r & 31));
        }
      }
    }
    if (a.record) {
      atomicAdd(&ctrl[4], vis);
      atomicAdd(&ctrl[5], pushes);
      atomicAdd(&ctrl[6], sc);
      if (ss) atomicAdd(ssum_l, (unsigned long long)ss);
    }
    __syncthreads();
    if (a.record) {
      for (uint32_t i = tid; i < 256; i += bd) a.rs_hist[o * 256 + i] = hist_l[i];
      if (tid == 0) {
        a.rs_u32[o * 4 + 0] = ctrl[4];
        a.rs_u32[o * 4 + 1] = ctrl[5];
        a.rs_u32[o * 4 + 2] = ctrl[6];
        a.rs_ssum[o] = *ssum_l;
      }
    }
    if (tid == 0 && ctrl[2]) atomicOr(a.err, ERR_INBOUND);
    __syncthreads();
  }
}

__global__ void k_bfs_seed(BfsArgs a, uint32_t* q0) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= a.S) return;
  const size_t p = (size_t)o * a.N + a.origin[o];
  a.hops[p] = 0;
  q0[o] = (uint32_t)p;
  if (o == 0) a.lvl[0] = a.S;
}

// Level-synchronous BFS over every slot at once (frontier of pair indices).
template <int ASZP>
__global__ __launch_bounds__(256) void k_bfs_level(BfsArgs a, uint32_t d, const uint32_t* __restrict__ qcur,
                                                  uint32_t* __restrict__ qnxt, uint32_t qmin, uint32_t qmax) {
  const uint32_t qn = a.lvl[d];
  if (qn < qmin || qn >= qmax) return;  // hybrid with the binned BFS: this level is the other kernel's
  const uint32_t N = a.N;
  bool overflow = false;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < qn; i0 += gridDim.x * blockDim.x) {
    const uint32_t i = i0 + threadIdx.x;
    const bool valid = i < qn;
    uint32_t p = valid ? qcur[i] : 0;
    if (valid && GS_OOB(p, a.PAIRS, a.err, "level frontier pair")) p = 0;
    const uint32_t o = p / N;
    const uint32_t u = p - o * N;
    const size_t base = (size_t)o * N;
    const uint32_t org = a.origin[o];
    const uint32_t nf = a.nfail[o];
    const uint32_t pm = valid ? a.mask[p] : 0;
    const uint32_t pushes = expand_node<ASZP, uint32_t, false>(a, valid, u, a.obkt[o], org, nf, pm, base, d,
                                                        a.cnt + base, a.hops + base, qnxt, &a.lvl[d + 1], base,
                                                        overflow);
    if (valid) {
      a.egress[p] = (uint8_t)pushes;
      if (a.record) a.egress_acc[p] += pushes;
    }
  }
  if (overflow) atomicOr(a.err, ERR_INBOUND);
}

static BfsArgs bfs_args(Engine& e);

// One level of k_bfs_level, run only when qmin <= frontier size < qmax (the binned
// BFS takes small levels this way: one atomic per push is cheap when there are few).
hipError_t launch_bfs_level_step(Engine& e, bool record, uint32_t d, uint32_t qmin, uint32_t qmax) {
  BfsArgs a = bfs_args(e);
  a.record = record ? 1 : 0;
  const uint32_t grid = (uint32_t)std::min<size_t>((qmax == 0xFFFFFFFFu ? e.PAIRS : qmax) / 256 + 1, 2048);
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_bfs_level<A>, dim3(grid), dim3(256), 0, e.st, a, d, e.q[d & 1],
                                              e.q[(d + 1) & 1], qmin, qmax));
  return hipGetLastError();
}

static BfsArgs bfs_args(Engine& e) {
  BfsArgs a;
  a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.frank = e.frank; a.origin = e.origin; a.obkt = e.obkt;
  a.nfail = e.nfail; a.mask = e.mask; a.hops = e.hops; a.cnt = e.cnt; a.inb = e.inb; a.egress = e.egress;
  a.lvl = e.lvl; a.err = e.err; a.N = e.N; a.S = e.S; a.ASZ = e.ASZ; a.fanout = e.fanout; a.capin = e.capin;
  a.PAIRS = e.PAIRS;
  a.egress_acc = e.egress_acc; a.stake = e.stake; a.srank = e.srank; a.strand = e.strand; a.bm = e.bm;
  a.rs_u32 = e.rs_u32; a.rs_ssum = e.rs_ssum; a.rs_hist = e.rs_hist; a.W = e.bm_words; a.record = 0;
  return a;
}

size_t bfs_wg_lds_bytes(uint32_t N) {
  return 64 + 1024 + 4 * (size_t)N + 2 * (size_t)((N + 3) & ~3u) + 2 * 2 * (size_t)((N + 1) & ~1u);
}

hipError_t launch_bfs(Engine& e, bool record) {
  BfsArgs a = bfs_args(e);
  a.record = record ? 1 : 0;
  hipError_t r;
  if (e.bfs_mode == GS_BFS_WORKGROUP) {
    const size_t lds = bfs_wg_lds_bytes(e.N);
    const uint32_t grid = e.S < 4096 ? e.S : 4096;
    GS_ASZP_DISPATCH(e.ASZP, {
      r = hipFuncSetAttribute((const void*)k_bfs_wg<A>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (r != hipSuccess) return r;
      hipLaunchKernelGGL(k_bfs_wg<A>, dim3(grid), dim3(256), lds, e.st, a);
    });
    return hipGetLastError();
  }
  if (e.bfs_mode == GS_BFS_BINNED) return launch_bfs_binned(e, record);
  if (e.bfs_mode == GS_BFS_MULTI) return launch_bfs_multi(e, record);
  if (e.bfs_mode == GS_BFS_HYBRID) return launch_bfs_hybrid(e, record);
  if ((r = hipMemsetAsync(e.hops, 0xFF, e.PAIRS, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.cnt, 0, e.PAIRS * 4, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.lvl, 0, 256 * 4, e.st)) != hipSuccess) return r;
  hipLaunchKernelGGL(k_bfs_seed, dim3(grid_for(e.S, 256)), dim3(256), 0, e.st, a, e.q[0]);
  const uint32_t grid = grid_for(e.PAIRS, 256, 2048);
  for (uint32_t d = 0; d < 254; ++d) {
    GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_bfs_level<A>, dim3(grid), dim3(256), 0, e.st, a, d, e.q[d & 1],
                                                e.q[(d + 1) & 1], 0u, 0xFFFFFFFFu));
    if ((d & 3) == 3) {  // poll the frontier size every 4 levels
      uint32_t* h = e.h_err + 1;
      if ((r = hipMemcpyAsync(h, e.lvl + d + 1, 4, hipMemcpyDeviceToHost, e.st)) != hipSuccess) return r;
      if ((r = hipStreamSynchronize(e.st)) != hipSuccess) return r;
      if (*h == 0) return hipGetLastError();
    }
  }
  return hipErrorNotSupported;  // frontier still non-empty after 254 levels: hop counts no longer fit u8
}

// --------------------------------------------- consume / prune (R9-R13) ----
struct CpArgs {
  const uint64_t* stake;
  const uint8_t* bucket;
  const uint32_t* peers;
  const uint16_t* hl;
  const uint32_t* origin;
  const uint8_t* obkt;
  const uint32_t* min_ingress;
  const double* thr;
  const uint32_t* cnt;
  const uint32_t* inb;
  uint32_t* cmeta;
  uint32_t* ckey;  // [CACHE_CAP][PAIRS] slot words (ck_make)
  uint8_t* prune_round;
  uint32_t* slot_prunes;
  uint32_t* mask;
  uint32_t* ingress_acc;
  uint32_t* prune_acc;
  uint32_t* err;
  uint32_t N, S, ASZ, ASZP, capin;
  int record;
  size_t PAIRS;
  size_t mso, msu;  // prune-mask strides of (slot, node)
};


// prune_connections -> PushActiveSet::prune(prunee u, pruner v, [origin]) for one
// prunee (gossip.rs:701-737, push_active_set.rs:56-71,143-151): set the prune bit
// of v's ring slot in u's entry for this origin, if v is still there.
__device__ inline void apply_prune(const CpArgs& a, uint32_t o, uint32_t ob, uint32_t u, uint32_t v) {
  if (GS_OOB(u, a.N, a.err, "apply_prune u")) return;
  const uint32_t b = min((uint32_t)a.bucket[u], ob);
  const uint32_t ent = u * NB + b;
  const uint32_t hv = a.hl[ent];
  const uint32_t head = hv & 0xFF, L = hv >> 8;
  const uint32_t* row = a.peers + (size_t)ent * a.ASZP;
  for (uint32_t j = 0; j < L; ++j) {
    uint32_t slot = head + j;
    if (slot >= a.ASZ) slot -= a.ASZ;
    if (row[slot] == v) {
      atomicOr(&a.mask[o * a.mso + u * a.msu], 1u << slot);
      return;
    }
  }
}

// Generic per-pair path (any in-degree / cache length): state read and written in place.
template <bool CONSUME, bool PRUNE, bool APPLY>
__device__ inline void cp_generic(const CpArgs& a, size_t p, uint32_t o, uint32_t v, bool& cache_overflow) {
  const size_t PAIRS = a.PAIRS;
  uint32_t meta = a.cmeta[p];
  uint32_t len = meta & 0xFF, up = (meta >> 8) & 0xFF;
  uint32_t c = 0;
  if (CONSUME) {
    // consume_messages (gossip.rs:618-653): inbound sorted by (hop, base58 id) =
    // ascending record value; ReceivedCache::record with num_dups = rank.
    c = a.cnt[p];
    if (c > a.capin) c = a.capin;
    uint32_t prev = 0;
    for (uint32_t k = 0; k < c; ++k) {
      uint32_t best = 0xFFFFFFFFu;
      for (uint32_t j = 0; j < c; ++j) {
        const uint32_t r = a.inb[(size_t)j * PAIRS + p];
        if ((k == 0 || r > prev) && r < best) best = r;
      }
      prev = best;
      const uint32_t src = best & 0xFFFFFFu;
      if (k == 0) up = up < 255 ? up + 1 : 255;
      int found = -1;
      for (uint32_t i = 0; i < len; ++i)
        if (ck_id(a.ckey[(size_t)i * PAIRS + p]) == src) { found = (int)i; break; }
      if (k < 2) {
        if (found >= 0) {
          uint32_t& w = a.ckey[(size_t)found * PAIRS + p];
          w = ck_bump(w);
        } else if (len < CACHE_CAP) {
          a.ckey[(size_t)len * PAIRS + p] = ck_make(src, 1u);
          ++len;
        } else {
          cache_overflow = true;
        }
      } else if (found < 0 && len < CACHE_LIMIT) {
        a.ckey[(size_t)len * PAIRS + p] = ck_make(src, 0u);
        ++len;
      }
    }
    meta = len | (up << 8) | (meta & 0xFF0000u);
    if (a.record && c) a.ingress_acc[p] += c;
  }
  uint32_t plen = (meta >> 16) & 0xFF;
  if (PRUNE) {
    // send_prunes -> ReceivedCache::prune (received_cache.rs:38-63,100-131).
    uint32_t npr = 0;
    plen = 0;
    if (up >= MIN_NUM_UPSERTS) {
      const uint32_t org = a.origin[o];
      const uint64_t sv = a.stake[v], so = a.stake[org];
      const uint64_t mis = min_ingress_stake(sv < so ? sv : so, a.thr[o]);
      const uint32_t mi = a.min_ingress[o];
      for (uint32_t i = 0; i < len; ++i) {
        const uint32_t wi = a.ckey[(size_t)i * PAIRS + p];
        const uint32_t ki = ck_id(wi), si = ck_score(wi);
        const uint64_t sti = a.stake[ki];
        uint32_t pos = 0;
        uint64_t cum = 0;
        for (uint32_t j = 0; j < len; ++j) {
          if (j == i) continue;
          const uint32_t wj = a.ckey[(size_t)j * PAIRS + p];
          const uint32_t kj = ck_id(wj), sj = ck_score(wj);
          const uint64_t stj = a.stake[kj];
          // sort by Reverse((score, stake)); ties by ascending id (canonical order)
          const bool before = sj > si || (sj == si && (stj > sti || (stj == sti && kj < ki)));
          if (before) { ++pos; cum = sat_add(cum, stj); }
        }
        if (pos >= mi && cum >= mis && ki != org) {
          a.ckey[(size_t)i * PAIRS + p] = ck_make(ki, si | PRUNED_FLAG);
          ++npr;
        }
      }
      plen = len;  // std::mem::take: the entry resets, the pruned keys stay readable
      len = 0;
      up = 0;
    }
    a.prune_round[p] = (uint8_t)(npr < 255 ? npr : 255);
    if (npr) {
      atomicAdd(&a.slot_prunes[o], npr);
      if (a.record) a.prune_acc[p] += npr;
    }
    meta = len | (up << 8) | (plen << 16);
  }
  if (APPLY && plen) {
    const uint32_t org = a.origin[o], ob = a.obkt[o];
    for (uint32_t i = 0; i < plen; ++i) {
      const uint32_t w = a.ckey[(size_t)i * PAIRS + p];
      if (!ck_pruned(w)) continue;
      const uint32_t u = ck_id(w);
      if (u != org) apply_prune(a, o, ob, u, v);
    }
  }
  a.cmeta[p] = meta;
}

// Step-wise forms (gs_consume_messages / gs_send_prunes / gs_prune_connections).
template <bool CONSUME, bool PRUNE, bool APPLY>
__global__ __launch_bounds__(256) void k_consume_prune(CpArgs a) {
  bool cache_overflow = false;
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < a.PAIRS; p += (size_t)gridDim.x * blockDim.x) {
    const uint32_t o = (uint32_t)(p / a.N);
    const uint32_t v = (uint32_t)(p - (size_t)o * a.N);
    cp_generic<CONSUME, PRUNE, APPLY>(a, p, o, v, cache_overflow);
  }
  if (cache_overflow) atomicOr(a.err, ERR_CACHE);
}

hipError_t launch_consume_prune(Engine& e, bool consume, bool prune, bool apply, bool record) {
  CpArgs a;
  a.stake = e.stake; a.bucket = e.bucket; a.peers = e.peers; a.hl = e.hl; a.origin = e.origin; a.obkt = e.obkt;
  a.min_ingress = e.min_ingress; a.thr = e.thr; a.cnt = e.cnt; a.inb = e.inb; a.cmeta = e.cmeta; a.ckey = e.ckey;
  a.prune_round = e.prune_round; a.slot_prunes = e.slot_prunes; a.mask = e.mask; a.err = e.err;
  a.ingress_acc = e.ingress_acc; a.prune_acc = e.prune_acc; a.record = record ? 1 : 0;
  a.N = e.N; a.S = e.S; a.ASZ = e.ASZ; a.ASZP = e.ASZP; a.capin = e.capin; a.PAIRS = e.PAIRS;
  a.mso = e.mso; a.msu = e.msu;
  const uint32_t grid = grid_for(e.PAIRS, 256, 8192);
  hipError_t r;
  if (consume && prune && apply) return launch_consume_prune_g(e, record, true, true);  // gs_consume_g.hip
  if (prune && (r = hipMemsetAsync(e.slot_prunes, 0, e.S * 4, e.st)) != hipSuccess) return r;
#define GS_CP(C, P, A) hipLaunchKernelGGL((k_consume_prune<C, P, A>), dim3(grid), dim3(256), 0, e.st, a)
  if (consume && !prune && !apply) GS_CP(true, false, false);
  else if (!consume && prune && !apply) GS_CP(false, true, false);
  else if (!consume && !prune && apply) GS_CP(false, false, true);
  else return hipErrorInvalidValue;
#undef GS_CP
  return hipGetLastError();
}

// ------------------------------------------------------ stats (R16-R22) ----
struct StatsArgs {
  const uint64_t* stake;
  const uint32_t* frank;
  const uint32_t* srank;
  const uint32_t* by_srank;
  const uint32_t* nfail;
  const uint8_t* hops;
  const uint32_t* cnt;
  const uint8_t* egress;
  const uint8_t* prune_round;
  const uint32_t* slot_prunes;
  uint32_t* egress_acc;
  uint32_t* ingress_acc;
  uint32_t* prune_acc;
  uint32_t* strand;
  uint32_t* rs_u32;
  uint64_t* rs_ssum;
  uint32_t* rs_hist;
  uint64_t* hist_acc;
  uint32_t* bm;
  uint32_t* bm_cnt;  // [S][64] set bits per chunk of each slot's bitmap (k_bm_count)
  gs_round_summary* sum;
  uint32_t N, S, W;
  uint32_t lo, hi;  // nodes of this pass (a node-range partition passes its own range)
  uint32_t NP, vlo; // pair p = slot * NP + (node - vlo); egress at slot * eso + (node - vlo) * esu
  size_t eso, esu;  // egress strides of (slot, node)
};

// FULL: the step-wise gs_record_round (reads the per-round counters of every pair);
// LITE: after a fused round whose kernels already accumulated egress/ingress/prunes
// (EG: the BFS left egress to this pass: the multi-source BFS).
// Grid (slots, node blocks); a block takes SP_UN x 256 nodes per trip, their loads issued
// together: a thread's trip is a chain of dependent loads (hop, then egress and the
// accumulators), and one node per trip left the pass bound by loads in flight (C5: 16 x
// 10M pairs in ~0.7 ms).
constexpr uint32_t SP_UN = 4;
template <bool FULL, bool EG = false>
__global__ __launch_bounds__(256) void k_stats_pass(StatsArgs a) {
  const uint32_t o = blockIdx.x, bx = blockIdx.y, gxn = gridDim.y;
  const size_t base = (size_t)o * a.NP - a.vlo;
  const uint32_t nf = a.nfail[o];
  __shared__ uint32_t h[256];
  __shared__ uint32_t acc[3];
  __shared__ unsigned long long ssum_s;
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  if (threadIdx.x < 3) acc[threadIdx.x] = 0;
  if (threadIdx.x == 0) ssum_s = 0;
  __syncthreads();
  uint32_t vis = 0, pushes = 0, sc = 0;
  uint64_t ss = 0;
  constexpr uint32_t OUT = 0x1FFu;  // not a node of this pass
  for (uint32_t vb = a.lo + bx * (SP_UN * 256); vb < a.hi; vb += gxn * (SP_UN * 256)) {
    uint32_t hh[SP_UN], cc[SP_UN], eg[SP_UN];
#pragma unroll
    for (uint32_t k = 0; k < SP_UN; ++k) {
      const uint32_t v = vb + k * 256 + threadIdx.x;
      const bool in = v < a.hi;
      const size_t p = base + v;
      hh[k] = in ? a.hops[p] : OUT;
      cc[k] = in ? a.cnt[p] : 0u;
      eg[k] = (in && (FULL || EG)) ? a.egress[o * a.eso + (v - a.vlo) * a.esu] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < SP_UN; ++k) {
      if (hh[k] == OUT) continue;
      const uint32_t v = vb + k * 256 + threadIdx.x;
      const size_t p = base + v;
      const uint32_t c = cc[k];
      pushes += c;
      if (FULL) {
        a.ingress_acc[p] += c;
        a.prune_acc[p] += a.prune_round[p];
      }
      if (hh[k] != 0xFF) {
        ++vis;
        atomicAdd(&h[hh[k]], 1u);
        if (FULL || EG) a.egress_acc[p] += eg[k];
      } else if (!(nf && a.frank[v] < nf)) {
        a.strand[p] += 1;
        ++sc;
        ss += a.stake[v];
        const uint32_t r = a.srank[v];
        atomicOr(&a.bm[(size_t)o * a.W + (r >> 5)], 1u << (r & 31));
      }
    }
  }
  atomicAdd(&acc[0], vis);
  atomicAdd(&acc[1], pushes);
  atomicAdd(&acc[2], sc);
  if (ss) atomicAdd(&ssum_s, (unsigned long long)ss);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x)
    if (h[i]) atomicAdd(&a.rs_hist[o * 256 + i], h[i]);
  if (threadIdx.x < 3 && acc[threadIdx.x]) atomicAdd(&a.rs_u32[o * 4 + threadIdx.x], acc[threadIdx.x]);
  if (threadIdx.x == 0 && ssum_s) atomicAdd((unsigned long long*)&a.rs_ssum[o], ssum_s);
}

// The k[0..3]-th set bits (0-based) of a slot's stranded bitmap, found by the whole
// block with ONE prefix pass over the bitmap's per-thread popcounts.
__device__ void block_kth_bits(const uint32_t* __restrict__ bm, uint32_t W, const uint32_t (&k)[4], uint32_t* scratch,
                               uint32_t* out) {
  const uint32_t T = blockDim.x, t = threadIdx.x;
  const uint32_t chunk = (W + T - 1) / T;
  const uint32_t lo = min(W, t * chunk), hi = min(W, lo + chunk);
  uint32_t c = 0;
  for (uint32_t i = lo; i < hi; i += 8) {  // 8 loads in flight per wait (a slot's bitmap is N / 32 words)
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = i + j < hi ? bm[i + j] : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) c += __popc(x[j]);
  }
  const uint32_t incl = wave_incl_scan(c);
  if ((t & 63) == 63) scratch[t >> 6] = incl;
  __syncthreads();
  uint32_t before = incl - c;
  for (uint32_t w = 0; w < (t >> 6); ++w) before += scratch[w];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!(k[j] >= before && k[j] < before + c)) continue;
    uint32_t need = k[j] - before;
    for (uint32_t i = lo; i < hi; ++i) {
      uint32_t w = bm[i];
      const uint32_t pc = __popc(w);
      if (need < pc) {
        for (uint32_t q = 0; q < need; ++q) w &= w - 1;
        out[j] = i * 32 + (__ffs(w) - 1);
        break;
      }
      need -= pc;
    }
  }
  __syncthreads();
}

// Set bits of each 1/64 of every slot's stranded bitmap (grid 64 x S): the finalize then
// scans only the chunks holding its order statistics instead of one block walking the
// whole bitmap twice (N / 32 words per slot: 312 K at 10M nodes).
constexpr uint32_t BM_CHUNKS = 64;
__global__ __launch_bounds__(256) void k_bm_count(const uint32_t* __restrict__ bm, uint32_t W, uint32_t* bm_cnt) {
  const uint32_t o = blockIdx.y, b = blockIdx.x;
  const uint32_t cw = (W + BM_CHUNKS - 1) / BM_CHUNKS;
  const uint32_t lo = min(W, b * cw), hi = min(W, lo + cw);
  const uint32_t* x = bm + (size_t)o * W;
  uint32_t c = 0;
  for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) c += __popc(x[i]);
  for (int off = 32; off > 0; off >>= 1) c += (uint32_t)__shfl_xor((int)c, off);
  __shared__ uint32_t ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bm_cnt[o * BM_CHUNKS + b] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(1024) void k_stats_finalize(StatsArgs a, uint32_t rec_slot) {
  const uint32_t o = blockIdx.x;
  __shared__ uint32_t hb[256];
  __shared__ uint32_t scratch[16];
  __shared__ uint32_t kth[4];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    hb[i] = a.rs_hist[o * 256 + i];
    a.hist_acc[o * 256 + i] += hb[i];
    a.rs_hist[o * 256 + i] = 0;
  }
  __syncthreads();
  gs_round_summary s = {};
  s.visited = a.rs_u32[o * 4 + 0];
  s.pushes = a.rs_u32[o * 4 + 1];
  s.stranded = a.rs_u32[o * 4 + 2];
  s.prunes = a.slot_prunes[o];
  s.stranded_stake_sum = a.rs_ssum[o];
  // HopsStat over reached non-origin nodes (hops 1..254), by wave 0: four bins per lane,
  // a wave scan of the counts, min/max from ballots, the medians from the scan
  __shared__ uint32_t hs[6];  // count, min, max, med lo, med hi, (pad)
  __shared__ unsigned long long hsum_s;
  if (threadIdx.x < 64) {
    const uint32_t l = threadIdx.x;
    uint32_t h[4], c = 0;
    uint64_t sm = 0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t i = 4 * l + t;
      h[t] = (i >= 1 && i < 255) ? hb[i] : 0u;
      c += h[t];
      sm += (uint64_t)i * h[t];
    }
    const uint32_t incl = wave_incl_scan(c);
    const uint32_t total = (uint32_t)__shfl((int)incl, 63);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)sm, off), hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(sm >> 32), off);
      sm += ((uint64_t)hi32 << 32) | lo32;
    }
    const uint64_t nz = __ballot(c > 0);
    if (l == 0) { hs[0] = total; hsum_s = sm; }
    if (total) {
      const uint32_t before = incl - c;
      if (l == (uint32_t)(__ffsll((long long)nz) - 1))
        for (int t = 0; t < 4; ++t)
          if (h[t]) { hs[1] = 4 * l + t; break; }
      if (l == 63u - (uint32_t)__clzll((long long)nz))
        for (int t = 3; t >= 0; --t)
          if (h[t]) { hs[2] = 4 * l + t; break; }
      const uint32_t ks[2] = {total % 2 ? total / 2 : total / 2 - 1, total / 2};
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (ks[q] >= before && ks[q] < incl) {
          uint32_t run = before;
          for (int t = 0; t < 4; ++t) {
            if (ks[q] < run + h[t]) { hs[3 + q] = 4 * l + t; break; }
            run += h[t];
          }
        }
      }
    }
  }
  __syncthreads();
  const uint32_t count = hs[0];
  s.hop_count = count;
  s.hop_sum = hsum_s;
  if (count) {
    s.hop_min = hs[1];
    s.hop_max = hs[2];
    s.hop_med_lo = hs[3];
    s.hop_med_hi = hs[4];
  }
  const uint32_t* bmo = a.bm + (size_t)o * a.W;
  const uint32_t sc = s.stranded;
  if (sc) {
    const uint32_t klo = sc % 2 ? sc / 2 : sc / 2 - 1, khi = sc / 2;
    const uint32_t ks[4] = {0u, sc - 1, klo, khi};
    // the chunk of each order statistic (wave 0, one chunk per lane), then a block scan of
    // that chunk only
    __shared__ uint32_t kc[4], kr[4], ktmp[4];
    if (threadIdx.x < 64) {
      const uint32_t l = threadIdx.x;
      const uint32_t c = a.bm_cnt[o * BM_CHUNKS + l];
      const uint32_t incl = wave_incl_scan(c), before = incl - c;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ks[j] >= before && ks[j] < incl) { kc[j] = l; kr[j] = ks[j] - before; }
    }
    __syncthreads();
    const uint32_t cw = (a.W + BM_CHUNKS - 1) / BM_CHUNKS;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = min(a.W, kc[j] * cw), n = min(a.W, lo + cw) - lo;
      const uint32_t kj[4] = {kr[j], 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
      block_kth_bits(bmo + lo, n, kj, scratch, ktmp);  // (ends with a barrier)
      if (threadIdx.x == 0) kth[j] = lo * 32 + ktmp[0];
      __syncthreads();
    }
    s.stranded_stake_min = a.stake[a.by_srank[kth[0]]];
    s.stranded_stake_max = a.stake[a.by_srank[kth[1]]];
    s.stranded_med_lo = a.stake[a.by_srank[kth[2]]];
    s.stranded_med_hi = a.stake[a.by_srank[kth[3]]];
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < a.W; i += blockDim.x) a.bm[(size_t)o * a.W + i] = 0;
  if (threadIdx.x == 0) {
    a.sum[(size_t)rec_slot * a.S + o] = s;
    a.rs_u32[o * 4 + 0] = 0;
    a.rs_u32[o * 4 + 1] = 0;
    a.rs_u32[o * 4 + 2] = 0;
    a.rs_ssum[o] = 0;
  }
}

// mode 0: full pass; 1: hop-only pass (fused level-synchronous round); 2: finalize only
// (the workgroup BFS already reduced the round, or a partition summed its partials);
// 3: the full pass only; 4: hop pass that also accumulates egress (multi-source BFS
// round); 5: mode 4's pass only (a partition rank's partials).
hipError_t launch_stats(Engine& e, uint32_t rec_slot, int mode) {
  StatsArgs a;
  a.stake = e.stake; a.frank = e.frank; a.srank = e.srank; a.by_srank = e.by_srank; a.nfail = e.nfail;
  a.hops = e.hops; a.cnt = e.cnt; a.egress = e.egress; a.prune_round = e.prune_round; a.slot_prunes = e.slot_prunes;
  a.egress_acc = e.egress_acc; a.ingress_acc = e.ingress_acc; a.prune_acc = e.prune_acc; a.strand = e.strand;
  a.rs_u32 = e.rs_u32; a.rs_ssum = e.rs_ssum; a.rs_hist = e.rs_hist; a.hist_acc = e.hist_acc; a.bm = e.bm;
  a.sum = e.sum; a.N = e.N; a.S = e.S; a.W = e.bm_words; a.eso = e.eso; a.esu = e.esu; a.bm_cnt = e.bm_cnt;
  a.lo = e.vlo;
  a.hi = e.vlo + e.NP;
  a.NP = e.NP; a.vlo = e.vlo;
  uint32_t gx = grid_for(e.NP, 256 * SP_UN, std::max<uint32_t>(64, 2048 / std::max<uint32_t>(e.S, 1)));
  if (mode == 0 || mode == 3) hipLaunchKernelGGL(k_stats_pass<true>, dim3(e.S, gx), dim3(256), 0, e.st, a);
  else if (mode == 1) hipLaunchKernelGGL(k_stats_pass<false>, dim3(e.S, gx), dim3(256), 0, e.st, a);
  else if (mode == 4 || mode == 5) hipLaunchKernelGGL((k_stats_pass<false, true>), dim3(e.S, gx), dim3(256), 0, e.st, a);
  if (mode != 3 && mode != 5)  // the pass only (a partition sums the partials over ranks first)
  {
    hipLaunchKernelGGL(k_bm_count, dim3(BM_CHUNKS, e.S), dim3(256), 0, e.st, e.bm, e.bm_words, e.bm_cnt);
    hipLaunchKernelGGL(k_stats_finalize, dim3(e.S), dim3(1024), 0, e.st, a, rec_slot);
  }
  return hipGetLastError();
}

// ------------------------------------------------------------ readback ----
template <class T>
__global__ void k_gather_strided(const T* __restrict__ src, size_t stride, uint32_t n, T* __restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[(size_t)i * stride];
}
hipError_t launch_gather_strided_u32(Engine& e, const uint32_t* src, size_t stride, uint32_t n, uint32_t* dst) {
  hipLaunchKernelGGL(k_gather_strided<uint32_t>, dim3(grid_for(n, 256)), dim3(256), 0, e.st, src, stride, n, dst);
  return hipGetLastError();
}

}  // namespace gs
