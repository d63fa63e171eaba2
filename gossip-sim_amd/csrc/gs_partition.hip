// gs_partition.hip -- node-range partition of one simulation batch over K ranks
// (per-origin state larger than one GPU).
//
// Rank r owns node ids [r*C, min((r+1)*C, N)). Active sets, prune masks and failed
// flags are replicated: every rank applies the same rotation (Philox), the same failures
// and the same (exchanged) prune bits. Per BFS level (Cluster::run_gossip,
// gossip.rs:494-615) every rank expands the WHOLE frontier -- rows and masks are local
// copies -- but keeps only the pushes whose destination it owns: in-degree, inbound
// record, first-visit hop and the next-level frontier bit. The frontier of the next level
// is the all-gather of the ranks' bitsets [K][S][Wr]. consume / send_prunes run on owned
// destinations; the prune bits they set (prune_connections, gossip.rs:701-737) go to a
// per-round delta whose sum over ranks is an OR -- a bit belongs to one pruner, owned by
// one rank -- and is OR-ed into every rank's masks. Statistics are partial sums over owned
// nodes (counts, hop bins, the stranded bitmap over stake rank), summed over ranks before
// the per-slot summary is finalized. The exchanges are the caller's (RCCL on device
// buffers, or host buffers): see include/gossip_hip.h gs_part_*.
#include "gs_device.h"
#include "gs_internal.h"

namespace gs {

namespace {

// Level 0: the origins, known to every rank.
__global__ void k_part_seed(uint32_t* fr_all, const uint32_t* __restrict__ origin, uint32_t S, uint32_t Wr,
                            uint32_t C, uint32_t N, uint32_t lo, uint32_t hi, uint8_t* hops) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= S) return;
  const uint32_t u = origin[o], r = u / C, off = u - r * C;
  atomicOr(&fr_all[((size_t)r * S + o) * Wr + (off >> 5)], 1u << (off & 31));
  if (u >= lo && u < hi) hops[(size_t)o * N + u] = 0;
}

// Global frontier bitsets -> queue of pairs (o * N + u); one atomic per wave.
__global__ __launch_bounds__(256) void k_part_compact(const uint32_t* __restrict__ fr_all, uint32_t K, uint32_t S,
                                                      uint32_t Wr, uint32_t C, uint32_t N, uint32_t* q,
                                                      uint32_t* qcount) {
  const size_t total = (size_t)K * S * Wr;
  for (size_t i0 = (size_t)blockIdx.x * blockDim.x; i0 < total; i0 += (size_t)gridDim.x * blockDim.x) {
    const size_t i = i0 + threadIdx.x;
    const uint32_t w = i < total ? fr_all[i] : 0u;
    const uint32_t k = __popc(w);
    const uint32_t incl = wave_incl_scan(k);
    const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
    if (!tot) continue;
    uint32_t b = 0;
    if (lane_id() == 63) b = atomicAdd(qcount, tot);
    b = (uint32_t)__shfl((int)b, 63) + incl - k;
    if (!w) continue;
    const uint32_t wi = (uint32_t)(i % Wr), ro = (uint32_t)(i / Wr);
    const uint32_t o = ro % S, r = ro / S;
    uint32_t m = w;
    while (m) {
      const uint32_t bit = __ffs(m) - 1;
      m &= m - 1;
      const uint32_t u = r * C + wi * 32 + bit;
      q[b++] = o * N + u;
    }
  }
}

// One BFS level over the whole frontier, keeping owned destinations.
template <int ASZP>
__global__ __launch_bounds__(256) void k_part_expand(
    const uint32_t* __restrict__ q, const uint32_t* __restrict__ qcount, uint32_t d, const uint8_t* __restrict__ bucket,
    const uint32_t* __restrict__ peers, const uint16_t* __restrict__ hl, const uint32_t* __restrict__ frank,
    const uint32_t* __restrict__ origin, const uint8_t* __restrict__ obkt, const uint32_t* __restrict__ nfail,
    const uint32_t* __restrict__ mask, uint8_t* hops, uint32_t* cnt, uint32_t* inb, uint8_t* egress,
    uint32_t* fr_own, uint32_t* newcount, uint32_t* err, uint32_t N, uint32_t ASZ, uint32_t fanout, uint32_t capin,
    size_t PAIRS, uint32_t lo, uint32_t hi, uint32_t Wr) {
  const uint32_t qn = *qcount;
  bool overflow = false;
  for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < qn; i0 += gridDim.x * blockDim.x) {
    const uint32_t i = i0 + threadIdx.x;
    const bool valid = i < qn;
    const uint32_t p = valid ? q[i] : 0u;
    const uint32_t o = p / N, u = p - o * N;
    uint32_t fresh = 0;
    if (valid) {
      const uint32_t org = origin[o], nf = nfail[o];
      const uint32_t ent = u * NB + min((uint32_t)bucket[u], (uint32_t)obkt[o]);
      const uint32_t hv = hl[ent];
      uint32_t row[ASZP];
      load_row<ASZP>(peers + (size_t)ent * ASZP, row);
      // PushActiveSet::get_nodes(..).take(fanout), failed peers burn their slot (gossip.rs:527-541)
      uint32_t pushm = taken_slots<ASZP>(row, hv & 0xFF, hv >> 8, ASZ, mask[p], org, fanout);
      if (nf) {
#pragma unroll
        for (int s = 0; s < ASZP; ++s)
          if (((pushm >> s) & 1u) && frank[row[s]] < nf) pushm &= ~(1u << s);
      }
      if (u >= lo && u < hi) egress[p] = (uint8_t)__popc(pushm);
      const size_t base = (size_t)o * N;
      const uint32_t rec = ((d + 1) << 24) | u;
      uint32_t old[ASZP];
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        const bool mine = ((pushm >> s) & 1u) && row[s] >= lo && row[s] < hi;
        old[s] = mine ? atomicAdd(&cnt[base + row[s]], 1u) : 0xFFFFFFFFu;
      }
#pragma unroll
      for (int s = 0; s < ASZP; ++s) {
        if (old[s] == 0xFFFFFFFFu) continue;
        const uint32_t w = row[s];
        if (old[s] < capin) inb[(size_t)old[s] * PAIRS + base + w] = rec;
        else overflow = true;
        if (old[s] == 0) {  // first arrival: dist = dist[src] + 1 (gossip.rs:594-600)
          hops[base + w] = (uint8_t)(d + 1);
          const uint32_t off = w - lo;
          atomicOr(&fr_own[(size_t)o * Wr + (off >> 5)], 1u << (off & 31));
          ++fresh;
        }
      }
    }
    const uint32_t incl = wave_incl_scan(fresh);
    if (lane_id() == 63 && incl) atomicAdd(newcount, incl);
  }
  if (overflow) atomicOr(err, ERR_INBOUND);
}

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

__global__ void k_part_delta_apply(uint32_t* mask, const uint32_t* __restrict__ delta, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (delta[i]) mask[i] |= delta[i];
}

uint32_t grid_of(size_t n, uint32_t cap = 4096) {
  const size_t g = (n + 255) / 256;
  return (uint32_t)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

size_t part_stats_words(const Engine& e) { return (size_t)e.S * (5 + 256 + e.bm_words); }

hipError_t launch_part_begin(Engine& e) {
  hipError_t r;
  if ((r = hipMemsetAsync(e.hops, 0xFF, e.PAIRS, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.cnt, 0, e.PAIRS * 4, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.egress, 0, e.PAIRS, e.st)) != hipSuccess) return r;
  if ((r = hipMemsetAsync(e.part_fr_all, 0, (size_t)e.part_K * e.S * e.part_Wr * 4, e.st)) != hipSuccess) return r;
  hipLaunchKernelGGL(k_part_seed, dim3(grid_of(e.S)), dim3(256), 0, e.st, e.part_fr_all, e.origin, e.S, e.part_Wr,
                     e.part_C, e.N, e.part_lo, e.part_hi, e.hops);
  return hipGetLastError();
}

hipError_t launch_part_level(Engine& e, uint32_t d) {
  hipError_t r;
  if ((r = hipMemsetAsync(e.part_cnt, 0, 8, e.st)) != hipSuccess) return r;
  hipLaunchKernelGGL(k_part_compact, dim3(grid_of((size_t)e.part_K * e.S * e.part_Wr)), dim3(256), 0, e.st,
                     e.part_fr_all, e.part_K, e.S, e.part_Wr, e.part_C, e.N, e.q[0], e.part_cnt);
  if ((r = hipMemsetAsync(e.part_fr_own, 0, (size_t)e.S * e.part_Wr * 4, e.st)) != hipSuccess) return r;
  GS_ASZP_DISPATCH(e.ASZP,
                   hipLaunchKernelGGL(k_part_expand<A>, dim3(grid_of(e.PAIRS, 2048)), dim3(256), 0, e.st, e.q[0],
                                      e.part_cnt, d, e.bucket, e.peers, e.hl, e.frank, e.origin, e.obkt, e.nfail,
                                      e.mask, e.hops, e.cnt, e.inb, e.egress, e.part_fr_own, e.part_cnt + 1, e.err,
                                      e.N, e.ASZ, e.fanout, e.capin, e.PAIRS, e.part_lo, e.part_hi, e.part_Wr));
  return hipGetLastError();
}

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

hipError_t launch_part_delta_apply(Engine& e) {
  hipLaunchKernelGGL(k_part_delta_apply, dim3(grid_of(e.PAIRS)), dim3(256), 0, e.st, e.mask, e.part_delta, e.PAIRS);
  return hipGetLastError();
}

}  // namespace gs
