// gs_partition.hip -- node-range partition of one simulation batch over K ranks
// (per-origin state larger than one GPU).
//
// Rank r owns node ids [lo, hi) (contiguous, starting on a 1,024-node bin). Replicated
// on every rank: stakes, active-set rows, prune masks and failed flags -- every rank
// applies the same rotations (Philox), the same failures and the same prune bits.
// Partitioned: every per-(slot, node) array -- hop counts, in-degrees, received caches,
// round counters, accumulators, stranded counts -- exists for owned nodes only
// (S x (hi - lo) pairs), and so do the BFS's per-destination record pools.
//
// A round: each rank runs the whole multi-source BFS (Cluster::run_gossip,
// gossip.rs:494-615) over its replicated rows and masks -- no exchange per level --
// keeping only the records of pushes to its own nodes; gathers and consumes them
// (gossip.rs:618-653) and runs send_prunes for its own pruners (gossip.rs:657-699).
// prune_connections (gossip.rs:701-737) sets bits in the PRUNEE's replicated mask row:
// each rank stages its prunes as records (slot * N + prunee, ring-slot bits), the
// ranks all-gather them and every rank ORs every record into its masks -- or, when the
// records outgrow the preallocated buffer or the dense form is smaller (a prune wave),
// as dense bit words [N][S] that the ranks SUM-all-reduce (bit-disjoint, so SUM = OR). Recorded
// statistics are partial sums over owned nodes (counts, hop bins, the stranded bitmap
// over stake rank), summed over ranks before the per-slot summary is finalized. The
// exchanges are the caller's (RCCL on device buffers, or host buffers): see
// include/gossip_hip.h gs_part_*.
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

namespace {

// Stats partials of one slot: visited, pushes, stranded, prunes, stranded stake sum,
// 256 hop bins, the stranded bitmap (W words), as u64 words.
__global__ void k_part_stats_pack(uint32_t S, uint32_t W, const uint32_t* rs_u32, const uint64_t* rs_ssum,
                                  const uint32_t* rs_hist, const uint32_t* bm, const uint32_t* slot_prunes,
                                  uint64_t* out) {
  const uint32_t R = 5 + 256 + W;
  const size_t total = (size_t)S * R;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t o = (uint32_t)(i / R), k = (uint32_t)(i - (size_t)o * R);
    uint64_t x;
    if (k < 3) x = rs_u32[o * 4 + k];
    else if (k == 3) x = slot_prunes[o];
    else if (k == 4) x = rs_ssum[o];
    else if (k < 261) x = rs_hist[o * 256 + (k - 5)];
    else x = bm[(size_t)o * W + (k - 261)];
    out[i] = x;
  }
}

__global__ void k_part_stats_unpack(uint32_t S, uint32_t W, const uint64_t* in, uint32_t* rs_u32, uint64_t* rs_ssum,
                                    uint32_t* rs_hist, uint32_t* bm, uint32_t* slot_prunes) {
  const uint32_t R = 5 + 256 + W;
  const size_t total = (size_t)S * R;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t o = (uint32_t)(i / R), k = (uint32_t)(i - (size_t)o * R);
    const uint64_t x = in[i];
    if (k < 3) rs_u32[o * 4 + k] = (uint32_t)x;
    else if (k == 3) slot_prunes[o] = (uint32_t)x;
    else if (k == 4) rs_ssum[o] = x;
    else if (k < 261) rs_hist[o * 256 + (k - 5)] = (uint32_t)x;
    else bm[(size_t)o * W + (k - 261)] = (uint32_t)x;
  }
}

// PushActiveSet::prune of every rank's prunes (push_active_set.rs:56-71): the record's
// ring-slot bits OR-ed into the prunee's mask word of the slot. Bits are idempotent, so
// a rank re-applying its own records changes nothing.
__global__ void k_part_prunes_apply(uint32_t* mask, size_t mso, size_t msu, uint32_t N, uint32_t S,
                                    const uint2* __restrict__ rec, size_t n, uint32_t* err) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint2 r = rec[i];
    const uint32_t o = r.x / N, u = r.x - o * N;
    if (o >= S) {  // a record from another engine geometry: refuse rather than write out of range
      atomicOr(err, ERR_BOUNDS);
      continue;
    }
    atomicOr(&mask[o * mso + u * msu], r.y);
  }
}

// The prune records of this rank's round, regenerated from the received caches: a pair
// that pruned this round (prune_round > 0) holds its prunees flagged in cache rows
// [0, pruned-len) (ReceivedCache::prune, received_cache.rs:100-131, as k_cg_prune left
// them); each prunee u's ring slots holding the pruner v in u's entry for the slot's
// origin become one record (slot * N + u, bits) -- the bits PushActiveSet::prune sets
// (push_active_set.rs:56-71). Records beyond cap are counted, not written.
template <int ASZP>
__global__ __launch_bounds__(256) void k_part_emit(const uint8_t* __restrict__ prune_round,
                                                   const uint32_t* __restrict__ cmeta, const uint32_t* __restrict__ ckey,
                                                   const uint8_t* __restrict__ bucket, const uint8_t* __restrict__ obkt,
                                                   const uint32_t* __restrict__ peers, const uint16_t* __restrict__ hl,
                                                   uint32_t N, uint32_t NP, uint32_t vlo, uint32_t ASZ, size_t PAIRS,
                                                   uint2* __restrict__ rec, size_t cap, uint32_t* __restrict__ count) {
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < PAIRS; q += (size_t)gridDim.x * blockDim.x) {
    if (!prune_round[q]) continue;
    const uint32_t o = (uint32_t)(q / NP), v = vlo + (uint32_t)(q - (size_t)o * NP);
    const uint32_t plen = (cmeta[q] >> 16) & 0xFFu, ob = obkt[o];
    for (uint32_t i = 0; i < plen; ++i) {
      const uint32_t w = ckey[(size_t)i * PAIRS + q];
      if (!ck_pruned(w)) continue;
      const uint32_t u = ck_id(w);
      const uint32_t ent = u * NB + min((uint32_t)bucket[u], ob);
      const uint32_t hv = hl[ent], head = hv & 0xFF, L = hv >> 8;
      uint32_t row[ASZP];
      load_row<ASZP>(peers + (size_t)ent * ASZP, row);
      uint32_t hit = 0;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        const uint32_t pos = (uint32_t)s >= head ? (uint32_t)s - head : (uint32_t)s + ASZ - head;
        hit |= (uint32_t)((uint32_t)s < ASZ && pos < L && row[s] == v) << s;
      }
      if (!hit) continue;
      const uint32_t k = atomicAdd(count, 1u);
      if (k < cap) rec[k] = make_uint2(o * N + u, hit);
    }
  }
}

// The same prunes as dense words: dense[u * S + o] |= the ring-slot bits of prunee u's
// entry for slot o (the caller zeroed dense). Every (slot, prunee) word gets bits from
// pruners of one rank only per ring slot -- a ring slot holds one pruner, and a pruner is
// owned by one rank -- so the ranks' words are bit-disjoint and their SUM is their OR.
template <int ASZP>
__global__ __launch_bounds__(256) void k_part_emit_dense(const uint8_t* __restrict__ prune_round,
                                                         const uint32_t* __restrict__ cmeta,
                                                         const uint32_t* __restrict__ ckey,
                                                         const uint8_t* __restrict__ bucket,
                                                         const uint8_t* __restrict__ obkt,
                                                         const uint32_t* __restrict__ peers,
                                                         const uint16_t* __restrict__ hl, uint32_t S, uint32_t NP,
                                                         uint32_t vlo, uint32_t ASZ, size_t PAIRS,
                                                         uint32_t* __restrict__ dense) {
  for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < PAIRS; q += (size_t)gridDim.x * blockDim.x) {
    if (!prune_round[q]) continue;
    const uint32_t o = (uint32_t)(q / NP), v = vlo + (uint32_t)(q - (size_t)o * NP);
    const uint32_t plen = (cmeta[q] >> 16) & 0xFFu, ob = obkt[o];
    for (uint32_t i = 0; i < plen; ++i) {
      const uint32_t w = ckey[(size_t)i * PAIRS + q];
      if (!ck_pruned(w)) continue;
      const uint32_t u = ck_id(w);
      const uint32_t ent = u * NB + min((uint32_t)bucket[u], ob);
      const uint32_t hv = hl[ent], head = hv & 0xFF, L = hv >> 8;
      uint32_t row[ASZP];
      load_row<ASZP>(peers + (size_t)ent * ASZP, row);
      uint32_t hit = 0;
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        const uint32_t pos = (uint32_t)s >= head ? (uint32_t)s - head : (uint32_t)s + ASZ - head;
        hit |= (uint32_t)((uint32_t)s < ASZ && pos < L && row[s] == v) << s;
      }
      if (hit) atomicOr(&dense[(size_t)u * S + o], hit);
    }
  }
}

// prune_connections from the summed dense words: mask |= word (push_active_set.rs:56-71).
__global__ void k_part_dense_apply(uint32_t* mask, size_t mso, size_t msu, uint32_t S, size_t words,
                                   const uint32_t* __restrict__ dense) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t x = dense[i];
    if (!x) continue;
    const size_t u = i / S, o = i - u * S;
    mask[o * mso + u * msu] |= x;  // (one thread per word: no atomic needed)
  }
}

uint32_t grid_of(size_t n, uint32_t cap = 4096) {
  const size_t g = (n + 255) / 256;
  return (uint32_t)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

size_t part_stats_words(const Engine& e) { return (size_t)e.S * (5 + 256 + e.bm_words); }

hipError_t launch_part_stats_pack(Engine& e) {
  hipLaunchKernelGGL(k_part_stats_pack, dim3(grid_of(part_stats_words(e))), dim3(256), 0, e.st, e.S, e.bm_words,
                     e.rs_u32, e.rs_ssum, e.rs_hist, e.bm, e.slot_prunes, e.part_stats);
  return hipGetLastError();
}

hipError_t launch_part_stats_unpack(Engine& e) {
  hipLaunchKernelGGL(k_part_stats_unpack, dim3(grid_of(part_stats_words(e))), dim3(256), 0, e.st, e.S, e.bm_words,
                     e.part_stats, e.rs_u32, e.rs_ssum, e.rs_hist, e.bm, e.slot_prunes);
  return hipGetLastError();
}

hipError_t launch_part_emit(Engine& e) {
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_part_emit<A>, dim3(grid_of(e.PAIRS, 8192)), dim3(256), 0, e.st,
                                              e.prune_round, e.cmeta, e.ckey, e.bucket, e.obkt, e.peers, e.hl, e.N,
                                              e.NP, e.vlo, e.ASZ, e.PAIRS, e.part_rec, e.part_rec_cap, e.part_cnt));
  return hipGetLastError();
}

hipError_t launch_part_emit_dense(Engine& e, uint32_t* dense) {
  hipError_t r = hipMemsetAsync(dense, 0, (size_t)e.S * e.N * 4, e.st);
  if (r != hipSuccess) return r;
  GS_ASZP_DISPATCH(e.ASZP, hipLaunchKernelGGL(k_part_emit_dense<A>, dim3(grid_of(e.PAIRS, 8192)), dim3(256), 0, e.st,
                                              e.prune_round, e.cmeta, e.ckey, e.bucket, e.obkt, e.peers, e.hl, e.S,
                                              e.NP, e.vlo, e.ASZ, e.PAIRS, dense));
  return hipGetLastError();
}

hipError_t launch_part_dense_apply(Engine& e, const uint32_t* dense) {
  const size_t words = (size_t)e.S * e.N;
  hipLaunchKernelGGL(k_part_dense_apply, dim3(grid_of(words, 8192)), dim3(256), 0, e.st, e.mask, e.mso, e.msu, e.S,
                     words, dense);
  return hipGetLastError();
}

hipError_t launch_part_prunes_apply(Engine& e, const uint2* rec, size_t n) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_part_prunes_apply, dim3(grid_of(n)), dim3(256), 0, e.st, e.mask, e.mso, e.msu, e.N, e.S, rec,
                     n, e.err);
  return hipGetLastError();
}

}  // namespace gs
