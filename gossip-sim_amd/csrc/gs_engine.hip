// gs_engine.hip -- engine lifetime, the C ABI of include/gossip_hip.h and readbacks.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>

#include "gs_device.h"
#include "gs_internal.h"

using namespace gs;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPC(expr)                                                                              \
  do {                                                                                          \
    hipError_t _r = (expr);                                                                     \
    if (_r != hipSuccess)                                                                       \
      return fail(GS_EHIP, std::string(#expr) + ": " + hipGetErrorString(_r));                  \
  } while (0)

hipEvent_t Engine::ev_take() {
  hipEvent_t x = nullptr;
  if (!ev_pool.empty()) {
    x = ev_pool.back();
    ev_pool.pop_back();
  } else {
    // timing only (read after a stream sync): no system-scope fence -- its L2 write-back
    // idled the GPU ~10 us at every recorded family boundary
    hipEventCreateWithFlags(&x, hipEventDisableSystemFence);
  }
  return x;
}
// GS_PROFILE_ONLY=fam1,fam2 at gs_create: this engine times only these families (an event
// record at a family boundary idles the GPU for a few us; bench.py's headline reads only the
// round kernel's)
static bool family_timed(const Engine& e, const char* fam) {
  return e.prof_only.empty() || e.prof_only.find("," + std::string(fam) + ",") != std::string::npos;
}

void Engine::tbegin(const char* fam, hipEvent_t* a) {
  *a = nullptr;
  if (!(prm.flags & GS_FLAG_PROFILE) || !family_timed(*this, fam)) return;
  *a = ev_take();
  hipEventRecord(*a, st);
  (void)fam;
}
void Engine::tend(const char* fam, hipEvent_t a) {
  if (!a) return;
  hipEvent_t b = ev_take();
  hipEventRecord(b, st);
  timers[fam].ev.push_back({a, b});
}

template <class T>
static int dalloc(Engine& e, T** p, size_t count, int fill = 0) {
  size_t bytes = count * sizeof(T);
  if (bytes == 0) bytes = 16;
  void* ptr = nullptr;
  hipError_t r = hipMalloc(&ptr, bytes);
  if (r != hipSuccess) return fail(GS_ENOMEM, "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(r));
  e.allocs.push_back(ptr);
  e.dev_bytes += bytes;
  r = hipMemsetAsync(ptr, fill, bytes, e.st);
  if (r != hipSuccess) return fail(GS_EHIP, std::string("hipMemsetAsync: ") + hipGetErrorString(r));
  *p = (T*)ptr;
  return GS_OK;
}
#define ALLOC(ptr, count, fill)                   \
  do {                                            \
    int _s = dalloc(*e, &(ptr), (count), (fill)); \
    if (_s) { destroy_engine(e); return _s; }     \
  } while (0)

static int flush_rot_clear(Engine* e);
static int ensure_rot_ahead(Engine* e);

template <class T>
static void dfree(Engine& e, T*& p, size_t count) {
  if (!p) return;
  auto it = std::find(e.allocs.begin(), e.allocs.end(), (void*)p);
  if (it != e.allocs.end()) e.allocs.erase(it);
  hipFree((void*)p);
  e.dev_bytes -= std::max<size_t>(16, count * sizeof(T));
  p = nullptr;
}

// GS_BFS_HYBRID: the push graph's T rows, level-record area and in-record regions for
// `parts` entries per node (1 + the distinct lower origin buckets of a group; set_slots
// grows them when a slot set needs more).
static int hb_alloc(Engine* e, uint32_t parts) {
  if (e->hb_pgr && parts <= e->hb_parts) return GS_OK;
  const uint32_t old_parts = e->hb_parts;
  hb_geometry(*e, parts);
  const size_t area = e->mv.area_cap, pgr = (size_t)e->mv.nbc * e->hb_bin_cap, T = e->mv.rows_cap * e->mv.TW;
  hb_geometry(*e, old_parts ? old_parts : 1);  // (unchanged until the new sizes are accepted)
  if ((double)area > (double)0xFFFFFFF0u || (double)pgr > (double)0xFFFFFFF0u)
    return fail(GS_ERANGE, "hybrid BFS: the push graph (nodes x active-set size x " + std::to_string(parts) +
                               " entries per node) exceeds 2^32 records");
  HIPC(hipStreamSynchronize(e->st));
  dfree(*e, e->mv_T, e->mv.rows_cap * e->mv.TW);
  dfree(*e, e->mv_area, e->mv.area_cap);
  dfree(*e, e->hb_pgr, (size_t)e->mv.nbc * e->hb_bin_cap);
  hb_geometry(*e, parts);
  int st = dalloc(*e, &e->mv_T, T, 0);
  if (!st) st = dalloc(*e, &e->mv_area, area, 0);
  if (!st) st = dalloc(*e, &e->hb_pgr, pgr, 0);
  if (st) e->slots_set = false;  // (no BFS runs on the missing buffers)
  return st;
}

static void destroy_engine(Engine* e) {
  if (!e) return;
  if (e->st) hipStreamSynchronize(e->st);
  for (void* p : e->allocs) hipFree(p);
  if (e->h_err) hipHostFree(e->h_err);
  if (e->part_in) hipFree(e->part_in);
  if (e->x_recv) hipFree(e->x_recv);
  if (e->x_pin) hipHostFree(e->x_pin);
  if (e->mv_hlvl) hipHostFree(e->mv_hlvl);
  if (e->mv_prof) hipHostFree(e->mv_prof);
  if (e->pb_registered) pb_register(*e, false);
  for (auto& kv : e->timers)
    for (auto& pr : kv.second.ev) { hipEventDestroy(pr.first); hipEventDestroy(pr.second); }
  for (hipEvent_t x : e->ev_pool) hipEventDestroy(x);
  if (e->st) hipStreamDestroy(e->st);
  delete e;
}

// Sorts (key, id) pairs on the device (stable, so ties stay in id order) and
// returns the sorted ids in out_ids.
// Device scratch freed on every exit path.
struct DevScratch {
  std::vector<void*> p;
  template <class T>
  bool get(T** out, size_t bytes) {
    void* x = nullptr;
    if (hipMalloc(&x, bytes ? bytes : 16) != hipSuccess) return false;
    p.push_back(x);
    *out = (T*)x;
    return true;
  }
  ~DevScratch() {
    for (void* x : p) hipFree(x);
  }
};

static int sort_ids_by_key(Engine& e, const uint64_t* keys_in, uint32_t* out_ids) {
  DevScratch sc;
  uint64_t *kin = nullptr, *kout = nullptr;
  uint32_t* vin = nullptr;
  void* tmp = nullptr;
  if (!sc.get(&kin, e.N * 8ull) || !sc.get(&kout, e.N * 8ull) || !sc.get(&vin, e.N * 4ull))
    return fail(GS_ENOMEM, "sort alloc");
  HIPC(hipMemcpyAsync(kin, keys_in, e.N * 8ull, hipMemcpyDeviceToDevice, e.st));
  std::vector<uint32_t> ids(e.N);
  for (uint32_t i = 0; i < e.N; ++i) ids[i] = i;
  HIPC(hipMemcpyAsync(vin, ids.data(), e.N * 4ull, hipMemcpyHostToDevice, e.st));
  size_t tmp_bytes = 0;
  HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, kin, kout, vin, out_ids, (int)e.N, 0, 64, e.st));
  if (!sc.get(&tmp, tmp_bytes)) return fail(GS_ENOMEM, "sort temp alloc");
  HIPC(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, out_ids, (int)e.N, 0, 64, e.st));
  HIPC(hipStreamSynchronize(e.st));  // the scratch is freed on return
  return GS_OK;
}

static int check_err(Engine* e) {
  HIPC(hipMemcpyAsync(e->h_err, e->err, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  const uint32_t f = e->h_err[0];
  if (f & ERR_SYNC) {  // (first: a barrier that timed out leaves every later result suspect)
    e->broken = true;  // its barrier epochs are out of step: every later call is refused
    return fail(GS_EHIP, "multi-source BFS: a grid barrier of the persistent BFS timed out (workgroups not "
                         "co-resident?); the engine is unusable -- destroy it and rerun with GS_MV_PBFS=0");
  }
  if (f & ERR_INBOUND)
    return fail(GS_ERANGE, "inbound capacity exceeded: a node received more than " + std::to_string(e->capin) +
                               " pushes in one round; recreate the engine with a larger inbound_capacity");
  if (f & ERR_CACHE) return fail(GS_ERANGE, "received-cache capacity (96 keys) exceeded");
  if (f & ERR_DEPTH) return fail(GS_ERANGE, "BFS depth exceeds 254 hops (hop counts are u8)");
  if (f & ERR_MV_CAP) {
    std::string what;
    if (f & ERR_MVD_ROWS) what += " level rows";
    if (f & ERR_MVD_AREA) what += " level records";
    if (f & ERR_MVD_POOL) what += " record pool";
    if (f & ERR_MVD_Q) what += " frontier queue";
    if (f & ERR_MVD_CSR) what += " gather CSR (one node's records)";
    return fail(GS_ERANGE, "multi-source BFS: capacity exceeded:" + what + " (recreate with GS_BFS_LEVEL)");
  }
  if (f & ERR_BOUNDS) return fail(GS_ERANGE, "debug bounds check failed (see GS_OOB lines on stdout)");
  return GS_OK;
}

extern "C" {

const char* gs_last_error(void) { return g_err.c_str(); }

int gs_device_count(int* n) {
  if (!n) return fail(GS_EINVAL, "null argument");
  *n = 0;
  if (hipGetDeviceCount(n) != hipSuccess) *n = 0;
  return GS_OK;
}

// Prune records a partition rank stages per round: past S * N / (2K) records per rank the
// dense words (S * N u32, all-reduced) are the smaller exchange anyway.
static size_t part_record_cap(size_t N, size_t S, uint32_t K) {
  if (const char* x = std::getenv("GS_PART_RECORD_CAP"))  // (tests: the record exchange through a prune wave)
    return std::max<size_t>(1, std::strtoull(x, nullptr, 10));
  return std::max<size_t>(1u << 16, (S * N) / (2 * (size_t)K));
}

// K == 0: an engine over all nodes; K >= 1: rank `rank` of a node-range partition over K
// ranks (K == 1: one rank owning every node, the exchange calls still available).
static int create_engine(const gs_params* prm, const uint64_t* stakes, uint32_t n, uint32_t n_slots, uint32_t rank,
                         uint32_t K, gs_engine** out) {
  const bool part = K >= 1;
  if (!part) K = 1;
  if (!prm || !stakes || !out) return fail(GS_EINVAL, "null argument");
  *out = nullptr;
  if (n < 2 || n > GS_MAX_NODES) return fail(GS_EINVAL, "n_nodes must be in [2, 2^24-1]");
  if (n_slots < 1) return fail(GS_EINVAL, "n_slots must be >= 1");
  if (prm->active_set_size < 1 || prm->active_set_size > GS_MAX_ACTIVE_SET_SIZE)
    return fail(GS_EINVAL, "active_set_size must be in [1, 32]");
  if (prm->push_fanout < 1) return fail(GS_EINVAL, "push_fanout must be >= 1");
  if (!(prm->rotation_probability >= 0.0 && prm->rotation_probability <= 1.0))
    return fail(GS_EINVAL, "rotation_probability must be in [0, 1]");
  if ((uint64_t)n * n_slots >= (1ull << 32)) return fail(GS_EINVAL, "n_nodes * n_slots must be < 2^32");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(GS_EHIP, "no HIP device visible (the engine has no CPU fallback)");
  if (prm->device < 0 || prm->device >= ndev) return fail(GS_EINVAL, "device ordinal out of range");
  HIPC(hipSetDevice(prm->device));

  Engine* e = new (std::nothrow) Engine();
  if (!e) return fail(GS_ENOMEM, "host allocation");
  e->prm = *prm;
  if (const char* x = std::getenv("GS_PROFILE_ONLY")) e->prof_only = "," + std::string(x) + ",";
  e->N = n;
  e->S = n_slots;
  e->NP = n;
  e->vlo = 0;
  e->PAIRS = (size_t)n * n_slots;
  e->ASZ = prm->active_set_size;
  e->ASZP = (e->ASZ + 3) & ~3u;
  e->fanout = prm->push_fanout;
  e->fcap = std::min(e->fanout, e->ASZ);
  e->capin = prm->inbound_capacity ? prm->inbound_capacity : 64;
  if (hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking) != hipSuccess) {
    destroy_engine(e);
    return fail(GS_EHIP, "hipStreamCreate");
  }
  if (hipHostMalloc(&e->h_err, 64) != hipSuccess) { destroy_engine(e); return fail(GS_ENOMEM, "pinned alloc"); }
  std::memset(e->h_err, 0, 64);

  uint32_t mode = prm->bfs_mode;
  const size_t lds = bfs_wg_lds_bytes(n);
  const size_t pairs = (size_t)n * n_slots;
  bin_geometry(n, pairs, e->fcap, e->bin, !(prm->flags & GS_FLAG_WIDE_RECORDS));
  const bool bin_ok = pairs <= (1ull << 28) && bin_supported(e->bin, e->fcap);
  mv_geometry(n, n_slots, e->ASZ, e->ASZP, e->mv);
  // (expand slice w writes its records at w * XT * ASZ and a T row holds that place as a u32:
  // the whole area must stay below 2^32 records -- ~16M nodes x 20-slot groups x a wide
  // active set would not)
  const bool mv_area_ok = (double)e->mv.rows_cap * e->mv.XT * e->ASZ <= (double)0xFFFFFFF0u;
  const bool mv_ok = mv_supported(e->mv, e->ASZP) && mv_area_ok;
  if (part) {  // a partition rank runs the multi-source BFS over its replicated tables
    if (mode != GS_BFS_AUTO && mode != GS_BFS_MULTI) {
      destroy_engine(e);
      return fail(GS_EINVAL, "a node-range partition runs bfs_mode GS_BFS_MULTI (or AUTO)");
    }
    mode = GS_BFS_MULTI;
    // whole 1,024-node bins per rank; a frontier-exchange rank owns whole coarse bins too (its
    // level records go to one owner per bin)
    e->part_x = (prm->flags & GS_FLAG_FRONTIER_EXCHANGE) != 0;
    const uint32_t unit = e->part_x ? std::max<uint32_t>(1024, 1u << e->mv.BSC) : 1024u;
    const uint32_t C = (uint32_t)((((size_t)n + K - 1) / K + unit - 1) / unit * unit);
    const uint32_t lo = (uint32_t)std::min<uint64_t>(n, (uint64_t)rank * C), hi = std::min(n, lo + C);
    if (lo >= hi) {
      destroy_engine(e);
      return fail(GS_EINVAL, "node-range partition: rank owns no nodes (ranges are multiples of 1,024 ids)");
    }
    e->part_on = true;
    e->part_C = C;
    e->part_K = K;
    e->part_rank = rank;
    e->part_lo = lo;
    e->part_hi = hi;
    e->NP = hi - lo;
    e->vlo = lo;
    e->PAIRS = (size_t)e->NP * n_slots;
  }
  // AUTO, measured: MULTI 2.6 vs BINNED 3.6 ms per C4 round (13 slots); at 10M nodes MULTI wins
  // from 2 slots (4.86 vs 5.26 ms); round 5, with expand grids sized from the level profile, at
  // one slot too (C3's one-slot 100k engines: 0.371 vs 0.450 ms per round of both)
  if (mode == GS_BFS_AUTO)
    mode = (n <= 8192 && n_slots >= 64) ? GS_BFS_WORKGROUP
           : mv_ok                      ? GS_BFS_MULTI
           : bin_ok                     ? GS_BFS_BINNED
                                        : GS_BFS_LEVEL;
  if (mode == GS_BFS_BINNED && !bin_ok) {
    destroy_engine(e);
    return fail(GS_EINVAL, "binned BFS: n_nodes * n_slots too large for its bin tables (use GS_BFS_LEVEL)");
  }
  if (mode == GS_BFS_MULTI && !mv_ok) {
    destroy_engine(e);
    return fail(GS_EINVAL, mv_area_ok ? "multi-source BFS: bin geometry exceeds LDS (use GS_BFS_LEVEL)"
                                      : "multi-source BFS: a level's record area (frontier capacity x expand slice x "
                                        "active-set size) exceeds 2^32 records (use GS_BFS_HYBRID or GS_BFS_LEVEL)");
  }
  if (mode == GS_BFS_WORKGROUP && (n > 65535 || lds > 160 * 1024)) {
    destroy_engine(e);
    return fail(GS_EINVAL, "workgroup BFS needs the per-slot state (9 B/node) to fit in 160 KiB of LDS");
  }
  if (mode == GS_BFS_HYBRID && !mv_ok) {
    destroy_engine(e);
    return fail(GS_EINVAL, "hybrid BFS: bin geometry exceeds LDS (use GS_BFS_LEVEL)");
  }
  if (mode != GS_BFS_WORKGROUP && mode != GS_BFS_LEVEL && mode != GS_BFS_BINNED && mode != GS_BFS_MULTI &&
      mode != GS_BFS_HYBRID) {
    destroy_engine(e);
    return fail(GS_EINVAL, "bfs_mode");
  }
  e->bfs_mode = mode;
  if (e->part_x) {  // a frontier-exchange rank's queues and level area hold its own nodes' entries only
    MvGeom& g = e->mv;
    g.q_cap = (size_t)e->NP * std::min<size_t>(std::min<size_t>(n_slots, g.GW), 26) + 64;
    g.rows_cap = (g.q_cap + g.XT - 1) / g.XT + 1;
    g.area_cap = g.rows_cap * g.XT * e->ASZ;
  }
  const bool mvl = mv_layout(*e);
  e->inb_valid = !mvl;  // multi / hybrid: no inbound rows until a BFS writes them
  if (mode == GS_BFS_HYBRID) {  // no pool records: slot groups limited by the level records only
    MvGeom& g = e->mv;
    g.GW = std::min(28u, (64u - g.UB - g.BSC) & ~3u);
    g.q_cap = (size_t)n * std::min<size_t>(std::min<size_t>(n_slots, g.GW), 26) + 64;
    e->hb_dsp = std::min<uint32_t>(n_slots, g.GW) <= 16 ? 16u : 32u;
    hb_geometry(*e, 1);
  }
  // one-kernel round (gs_round): per-slot state in LDS, at most 160 KiB per workgroup
  e->fused = mode == GS_BFS_WORKGROUP && !(prm->flags & GS_FLAG_SPLIT_ROUND) &&
             round_wg_lds_bytes(n, e->fcap, e->ASZP) <= 160 * 1024;
  // rotation ahead of the fused round (one-workgroup rotation sizes; GS_ROT_AHEAD=0: off)
  e->rot_ahead_ok = e->fused && n <= 16384 && round_wg_lds_bytes(n, e->fcap, e->ASZP) >= 4 * ((size_t)n + 1) &&
                    !(std::getenv("GS_ROT_AHEAD") && std::getenv("GS_ROT_AHEAD")[0] == '0');

  const size_t N = n, S = n_slots, PAIRS = e->PAIRS, NP = e->NP;
  e->SP = (uint32_t)((S + 3) & ~(size_t)3);
  if (mvl) {  // node-major masks / egress: a node's slots share one line
    e->mso = 1; e->msu = e->SP; e->eso = 1; e->esu = e->SP; e->mask_words = N * e->SP;
    // node lines: when a node's own-entry row and its masks fit 128 B, both live in one
    // line of the row table (stride 32 words, masks at the row's end): an expansion
    // reads one HBM line per entry instead of two half-used ones
    const uint32_t row_words = ((e->ASZP + 1 + e->ASZP / 4) + 3) & ~3u;
    const char* nl = std::getenv("GS_MV_NO_LINE");
    if (row_words + e->SP <= 32 && !(nl && nl[0] == '1')) {
      e->mv_line = true;
      e->msu = 32;
    }
  } else {
    e->mso = N; e->msu = 1; e->eso = N; e->esu = 1; e->mask_words = PAIRS;
  }
  ALLOC(e->stake, N, 0);
  ALLOC(e->bucket, N, 0);
  ALLOC(e->P, (size_t)NB * (N + 1), 0);
  ALLOC(e->IX, (size_t)NB * ix_count(n), 0);
  ALLOC(e->peers, N * NB * e->ASZP, 0);
  ALLOC(e->hl, N * NB, 0);
  ALLOC(e->frank, N, 0);
  ALLOC(e->srank, N, 0);
  ALLOC(e->by_srank, N, 0);
  ALLOC(e->prank, N, 0);
  ALLOC(e->by_prank, N, 0);
  ALLOC(e->pstake, N, 0);
  ALLOC(e->pinfo, N, 0);
  ALLOC(e->rinfo, N, 0);
  ALLOC(e->origin, S, 0);
  ALLOC(e->obkt, S, 0);
  ALLOC(e->min_ingress, S, 0);
  ALLOC(e->thr, S, 0);
  ALLOC(e->nfail, S, 0);
  ALLOC(e->slot_prunes, S, 0);
  if (!e->mv_line) ALLOC(e->mask, e->mask_words, 0);  // (node lines: inside the row table below)
  size_t b0 = e->dev_bytes;  // per-(slot, node) state from here (a partition rank: its own nodes)
  ALLOC(e->hops, PAIRS, 0xFF);
  ALLOC(e->cnt, PAIRS, 0);
  if (!mvl) ALLOC(e->inb, (size_t)e->capin * PAIRS, 0);  // multi / hybrid: on first use (ensure_inb)
  ALLOC(e->cmeta, PAIRS, 0);
  ALLOC(e->ckey, (size_t)CACHE_CAP * PAIRS, 0);
  ALLOC(e->egress, std::max(PAIRS, NP * e->esu), 0);
  ALLOC(e->prune_round, PAIRS, 0);
  ALLOC(e->egress_acc, PAIRS, 0);
  ALLOC(e->ingress_acc, PAIRS, 0);
  ALLOC(e->prune_acc, PAIRS, 0);
  ALLOC(e->strand, PAIRS, 0);
  e->pair_bytes += e->dev_bytes - b0;
  if (mode == GS_BFS_LEVEL || mode == GS_BFS_BINNED) {
    ALLOC(e->q[0], PAIRS, 0);
    ALLOC(e->q[1], PAIRS, 0);
  }
  if (mode == GS_BFS_BINNED) {  // ~4096 bins of 2^BS consecutive pairs (L2-sized apply working set)
    e->ORW = e->ASZP + 4;
    ALLOC(e->own, N * e->ORW, 0);
    ALLOC(e->bin_area, PAIRS * e->fcap, 0);
    ALLOC(e->bin_T, e->bin.T_words, 0);
    // pool: one region of 2^BS * capin records per bin (u32 records when narrow)
    ALLOC(e->bin_pool, ((size_t)e->bin.nbins << e->bin.BS) * e->capin / (e->bin.narrow ? 2 : 1), 0);
    ALLOC(e->bin_Lt, (size_t)256 * e->bin.nbins, 0);
    ALLOC(e->bin_binoff, e->bin.nbins, 0);
    ALLOC(e->bin_vis, (size_t)e->bin.nbins << (e->bin.BS - 5), 0);  // whole bins (applies read a bin's words)
  }
  if (mode == GS_BFS_BINNED || mvl) {  // host-mapped level sizes the level loops poll
    if (hipHostMalloc(&e->mv_hlvl, 272 * 4, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&e->mv_hlvl_dev, e->mv_hlvl, 0) != hipSuccess) {
      destroy_engine(e);
      return fail(GS_ENOMEM, "host-mapped frontier counters");
    }
    e->mv_hstate_dev = e->mv_hlvl_dev + 256;
    // the predicted level loops: per-pair levels, and one level profile per slot group
    ALLOC(e->mv_dpair, 258, 0);
    const size_t ng = mvl ? (S + e->mv.GW - 1) / e->mv.GW : 1;
    if (hipHostMalloc(&e->mv_prof, ng * MV_PROF_WORDS * 4, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&e->mv_prof_dev, e->mv_prof, 0) != hipSuccess) {
      destroy_engine(e);
      return fail(GS_ENOMEM, "host-mapped level profiles");
    }
    std::memset(e->mv_prof, 0, ng * MV_PROF_WORDS * 4);
    e->mv_pred.assign(ng, {});
    e->mv_prof_seen.assign(ng, 0);
  }
  if (mvl) {
    const MvGeom& g = e->mv;
    if (const char* dg = std::getenv("GS_MV_DIAG"); dg && dg[0] == '1') e->mv_diag = true;
    if (const char* fu = std::getenv("GS_MV_FUSED"); fu && fu[0] == '1') e->mv_fused = true;
    const uint32_t row_words = ((e->ASZP + 1 + e->ASZP / 4) + 3) & ~3u;  // row, meta, peers' failure classes
    e->ORW = e->mv_line ? 32 : row_words;
    ALLOC(e->own, N * e->ORW, 0);
    if (e->mv_line) e->mask = e->own + row_words;
    ALLOC(e->mv_vis, N, 0);
    ALLOC(e->mv_q[0], g.q_cap, 0);
    ALLOC(e->mv_q[1], g.q_cap, 0);
    ALLOC(e->mv_ctr, 4, 0);
    if (mode == GS_BFS_HYBRID) {
      ALLOC(e->hb_dist, N * e->hb_dsp, 0xFF);
      ALLOC(e->hb_pgo, N, 0);
      ALLOC(e->hb_F, 3 * N, 0);
      if (int s_ = hb_alloc(e, 1)) { destroy_engine(e); return s_; }
    } else {
      ALLOC(e->mv_T, g.rows_cap * g.TW, 0);
      ALLOC(e->mv_area, g.area_cap, 0);
      const uint32_t fno = mv_kept_bins(*e);  // a partition rank pools records to its own nodes only
      e->part_flo = e->vlo >> g.BSF;
      e->part_fno = fno;
      b0 = e->dev_bytes;
      ALLOC(e->mv_pool, (size_t)fno * g.pcap, 0);
      ALLOC(e->mv_pused, fno, 0);
      e->pair_bytes += e->dev_bytes - b0;
      if (pb_setup(*e)) {  // the persistent BFS (gs_bfs_pers.hip): its level records, T rows and entries
        ALLOC(e->pb_T[0], (size_t)(e->pb_G + 2) * e->pb_rows_cap, 0);
        ALLOC(e->pb_T[1], (size_t)(e->pb_G + 2) * e->pb_rows_cap, 0);
        ALLOC(e->pb_area[0], e->pb_area_cap, 0);
        ALLOC(e->pb_area[1], e->pb_area_cap, 0);
        ALLOC(e->pb_blk, pb_blk_words(), 0);
        ALLOC(e->pb_gq, (size_t)e->pb_G * e->pb_gq_cap, 0);
        pb_register(*e, true);
        e->pb_registered = true;
      }
    }
    ALLOC(e->mv_fcls, N, 0xFF);
    ALLOC(e->mv_fk, S, 0);
    ALLOC(e->mv_thr, S, 0);
    ALLOC(e->mv_gtab, (size_t)((S + g.GW - 1) / g.GW) * GT_STRIDE, 0);
    ALLOC(e->mv_seed, S, 0);
  }
  e->h_nfail_any.assign(S, 0);
  ALLOC(e->lvl, 512, 0);  // [256] level sizes; binned BFS: [256 + d] = 1 iff level d was binned this round
  ALLOC(e->rot_list, N, 0);
  ALLOC(e->rot_count, 2, 0);
  ALLOC(e->rot_changed, N * NB, 0);
  ALLOC(e->rs_u32, S * 4, 0);
  ALLOC(e->rs_ssum, S, 0);
  ALLOC(e->rs_hist, S * 256, 0);
  ALLOC(e->hist_acc, S * 256, 0);
  e->bm_words = (n + 31) / 32;
  ALLOC(e->bm, S * e->bm_words, 0);
  ALLOC(e->bm_cnt, (size_t)S * 64, 0);
  // recorded-round summaries stay on the device until read back: a ring of up to
  // 256 MiB (C2: ~1,400 rounds) so a measured run is never stalled by a drain
  e->sum_cap = (uint32_t)std::max<size_t>(64, std::min<size_t>(4096, (256ull << 20) / (S * sizeof(gs_round_summary))));
  ALLOC(e->sum, (size_t)e->sum_cap * S, 0);
  ALLOC(e->err, 4, 0);
  if (e->part_on) {  // prune records of a round: when a round has more, its exchange is dense (gs_part_exchange_sizes)
    e->part_rec_cap = part_record_cap(N, S, K);
    const size_t b1 = e->dev_bytes;
    ALLOC(e->part_rec, e->part_rec_cap, 0);
    e->pair_bytes += e->dev_bytes - b1;
    ALLOC(e->part_cnt, 1, 0);
    ALLOC(e->part_stats, part_stats_words(*e), 0);
    if (e->part_x) {
      e->x_send_cap = e->mv.area_cap + e->mv.nbc;
      ALLOC(e->x_send, e->x_send_cap, 0);
      ALLOC(e->x_T, (size_t)K * e->mv.TW, 0);
      ALLOC(e->x_bincnt, e->mv.nbc, 0);
      ALLOC(e->x_pos, 2 * (size_t)e->mv.nbc, 0);
      ALLOC(e->x_off, (size_t)K + 1, 0);
      ALLOC(e->x_bins, 2 * (size_t)K, 0);
      ALLOC(e->x_wlog, 256 * (size_t)K, 0);
    }
  }
  if (const char* pp = std::getenv("GS_PHASE_PROFILE"); pp && pp[0] == '1') ALLOC(e->phase_clk, 32, 0);
  if (e->rot_ahead_ok) {  // the rotation-ahead buffers at create: counted in the engine's memory, fail here
    if (int s_ = ensure_rot_ahead(e)) { destroy_engine(e); return s_; }
  }

  // stakes, buckets and the static rotation prefix sums
  std::vector<uint8_t> b(N);
  for (size_t i = 0; i < N; ++i) b[i] = (uint8_t)stake_bucket(stakes[i]);
  if (hipMemcpyAsync(e->stake, stakes, N * 8, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      hipMemcpyAsync(e->bucket, b.data(), N, hipMemcpyHostToDevice, e->st) != hipSuccess ||
      launch_prefix_weights(*e) != hipSuccess) {
    destroy_engine(e);
    return fail(GS_EHIP, "upload / prefix-weights launch failed");
  }
  // stake rank (ascending stake, ties by id) for the stranded-stake order statistics
  int s = sort_ids_by_key(*e, e->stake, e->by_srank);
  if (s) { destroy_engine(e); return s; }
  if (launch_scatter_rank(*e, e->by_srank, e->srank) != hipSuccess) {
    destroy_engine(e);
    return fail(GS_EHIP, "stake-rank scatter");
  }
  // prune rank: (stake desc, id asc) -- the order ReceivedCache::prune sorts by, ties canonical
  {
    std::vector<uint32_t> ids(N), pr(N);
    std::vector<uint64_t> ps(N);
    for (uint32_t i = 0; i < n; ++i) ids[i] = i;
    std::stable_sort(ids.begin(), ids.end(), [&](uint32_t x, uint32_t y) { return stakes[x] > stakes[y]; });
    for (uint32_t r = 0; r < n; ++r) { pr[ids[r]] = r; ps[r] = stakes[ids[r]]; }
    std::vector<uint4> pi(N), ri(N);
    for (uint32_t i = 0; i < n; ++i) {
      pi[i] = make_uint4(pr[i], 0u, (uint32_t)stakes[i], (uint32_t)(stakes[i] >> 32));
      ri[i] = make_uint4(ids[i], 0u, (uint32_t)ps[i], (uint32_t)(ps[i] >> 32));
    }
    if (hipMemcpyAsync(e->prank, pr.data(), N * 4, hipMemcpyHostToDevice, e->st) != hipSuccess ||
        hipMemcpyAsync(e->by_prank, ids.data(), N * 4, hipMemcpyHostToDevice, e->st) != hipSuccess ||
        hipMemcpyAsync(e->pstake, ps.data(), N * 8, hipMemcpyHostToDevice, e->st) != hipSuccess ||
        hipMemcpyAsync(e->pinfo, pi.data(), N * 16, hipMemcpyHostToDevice, e->st) != hipSuccess ||
        hipMemcpyAsync(e->rinfo, ri.data(), N * 16, hipMemcpyHostToDevice, e->st) != hipSuccess ||
        hipStreamSynchronize(e->st) != hipSuccess) {
      destroy_engine(e);
      return fail(GS_EHIP, "prune-rank upload");
    }
  }
  if (hipStreamSynchronize(e->st) != hipSuccess) { destroy_engine(e); return fail(GS_EHIP, "create sync"); }
  *out = reinterpret_cast<gs_engine*>(e);
  return GS_OK;
}

int gs_create(const gs_params* prm, const uint64_t* stakes, uint32_t n, uint32_t n_slots, gs_engine** out) {
  return create_engine(prm, stakes, n, n_slots, 0, 0, out);
}

int gs_create_part(const gs_params* prm, const uint64_t* stakes, uint32_t n, uint32_t n_slots, uint32_t rank,
                   uint32_t nranks, gs_engine** out) {
  if (nranks < 1 || rank >= nranks) return fail(GS_EINVAL, "rank must be < nranks");
  return create_engine(prm, stakes, n, n_slots, rank, nranks, out);
}

void gs_destroy(gs_engine* eh) { destroy_engine(reinterpret_cast<Engine*>(eh)); }

#define ENGINE(eh)                                                                           \
  Engine* e = reinterpret_cast<Engine*>(eh);                                                 \
  if (!e) return fail(GS_EINVAL, "null engine");                                             \
  if (e->broken) return fail(GS_ESTATE, "engine unusable after a grid-barrier timeout; destroy it"); \
  HIPC(hipSetDevice(e->prm.device));

// Zeroes every prune mask (in the multi BFS's node lines, only the mask words).
static hipError_t clear_masks(Engine* e) {
  if (e->mv_line)
    return hipMemset2DAsync(e->mask, (size_t)e->msu * 4, 0, (size_t)e->SP * 4, e->N, e->st);
  return hipMemsetAsync(e->mask, 0, e->mask_words * 4, e->st);
}

static int reset_pair_state(Engine* e) {
  HIPC(clear_masks(e));
  HIPC(hipMemsetAsync(e->cmeta, 0, e->PAIRS * 4, e->st));
  HIPC(hipMemsetAsync(e->egress_acc, 0, e->PAIRS * 4, e->st));
  HIPC(hipMemsetAsync(e->ingress_acc, 0, e->PAIRS * 4, e->st));
  HIPC(hipMemsetAsync(e->prune_acc, 0, e->PAIRS * 4, e->st));
  HIPC(hipMemsetAsync(e->strand, 0, e->PAIRS * 4, e->st));
  HIPC(hipMemsetAsync(e->hist_acc, 0, (size_t)e->S * 256 * 8, e->st));
  HIPC(hipMemsetAsync(e->hops, 0xFF, e->PAIRS, e->st));
  HIPC(hipMemsetAsync(e->cnt, 0, e->PAIRS * 4, e->st));
  HIPC(hipMemsetAsync(e->prune_round, 0, e->PAIRS, e->st));
  e->sum_used = 0;
  e->h_sum.clear();
  return GS_OK;
}

int gs_set_slots(gs_engine* eh, const gs_slot* slots, uint32_t n_slots) {
  ENGINE(eh);
  if (int s_ = flush_rot_clear(e)) return s_;
  if (!slots || n_slots != e->S) return fail(GS_EINVAL, "gs_set_slots: need exactly n_slots entries");
  std::vector<uint32_t> org(e->S), mi(e->S);
  std::vector<uint8_t> ob(e->S);
  std::vector<double> thr(e->S);
  std::vector<uint8_t> bh(e->N);
  HIPC(hipMemcpyAsync(bh.data(), e->bucket, e->N, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  for (uint32_t o = 0; o < e->S; ++o) {
    if (slots[o].origin >= e->N) return fail(GS_EINVAL, "slot origin out of range");
    if (!(slots[o].prune_stake_threshold >= 0.0) || std::isinf(slots[o].prune_stake_threshold))
      return fail(GS_EINVAL, "prune_stake_threshold must be finite and >= 0");
    org[o] = slots[o].origin;
    ob[o] = bh[slots[o].origin];
    mi[o] = slots[o].min_ingress_nodes;
    thr[o] = slots[o].prune_stake_threshold;
  }
  // from the first upload on, the device holds a mix of old and new slot state until this
  // call returns GS_OK: any failure below leaves the engine without slots (every BFS call
  // is refused until set_slots succeeds)
  e->slots_set = false;
  HIPC(hipMemcpyAsync(e->origin, org.data(), e->S * 4, hipMemcpyHostToDevice, e->st));
  HIPC(hipMemcpyAsync(e->obkt, ob.data(), e->S, hipMemcpyHostToDevice, e->st));
  HIPC(hipMemcpyAsync(e->min_ingress, mi.data(), e->S * 4, hipMemcpyHostToDevice, e->st));
  HIPC(hipMemcpyAsync(e->thr, thr.data(), e->S * 8, hipMemcpyHostToDevice, e->st));
  if (mv_layout(*e)) {
    std::vector<uint32_t> gtab;
    std::vector<uint2> seeds;
    mv_build_groups(*e, org, ob, bh, gtab, seeds);
    if (e->bfs_mode == GS_BFS_HYBRID) {  // entries per node at most: the own bucket's + one per lower origin bucket
      uint32_t parts = 1;
      for (size_t g = 0; g < e->mv_groups.size(); ++g) parts = std::max(parts, 1 + gtab[g * GT_STRIDE + 25]);
      if (int s_ = hb_alloc(e, parts)) return s_;
    }
    HIPC(hipMemcpyAsync(e->mv_gtab, gtab.data(), gtab.size() * 4, hipMemcpyHostToDevice, e->st));
    HIPC(hipMemcpyAsync(e->mv_seed, seeds.data(), seeds.size() * sizeof(uint2), hipMemcpyHostToDevice, e->st));
  }
  if (e->mv_prof) {  // new origins: no level profile to predict from (earlier rounds' are ignored)
    HIPC(hipStreamSynchronize(e->st));
    for (size_t g = 0; g < e->mv_pred.size(); ++g) {
      e->mv_pred[g].clear();
      e->mv_prof_seen[g] = ((volatile uint32_t*)e->mv_prof)[g * MV_PROF_WORDS];
    }
  }
  e->slots.assign(slots, slots + n_slots);
  e->slots_set = true;
  int r = reset_pair_state(e);
  if (r) return r;
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_sync(gs_engine* eh) {
  ENGINE(eh);
  return check_err(e);
}

int gs_init_active_sets(gs_engine* eh) {
  ENGINE(eh);
  if (int s_ = flush_rot_clear(e)) return s_;
  HIPC(launch_init_entries(*e));
  HIPC(clear_masks(e));
  return GS_OK;
}

int gs_set_active_set_entry(gs_engine* eh, uint32_t node, uint32_t bucket, const uint32_t* peers, uint32_t len) {
  ENGINE(eh);
  if (int s_ = flush_rot_clear(e)) return s_;
  if (node >= e->N || bucket >= (uint32_t)NB) return fail(GS_EINVAL, "node/bucket out of range");
  if (len > e->ASZ) return fail(GS_ERANGE, "entry longer than active_set_size");
  std::vector<uint32_t> row(e->ASZP, 0);
  for (uint32_t i = 0; i < len; ++i) {
    if (peers[i] >= e->N || peers[i] == node) return fail(GS_EINVAL, "bad peer id");
    for (uint32_t j = 0; j < i; ++j)
      if (peers[j] == peers[i]) return fail(GS_EINVAL, "duplicate peer in entry");
    row[i] = peers[i];
  }
  const size_t ent = (size_t)node * NB + bucket;
  uint16_t hv = (uint16_t)(len << 8);
  HIPC(hipMemcpyAsync(e->peers + ent * e->ASZP, row.data(), e->ASZP * 4, hipMemcpyHostToDevice, e->st));
  HIPC(hipMemcpyAsync(e->hl + ent, &hv, 2, hipMemcpyHostToDevice, e->st));
  e->rows2_stale = true;
  HIPC(launch_own_rows(*e, nullptr, nullptr));
  HIPC(launch_clear_slot_masks(*e, node, bucket, 0xFFFFFFFFu));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_get_active_set_entry(gs_engine* eh, uint32_t node, uint32_t bucket, uint32_t* peers, uint32_t cap,
                            uint32_t* len) {
  ENGINE(eh);
  if (node >= e->N || bucket >= (uint32_t)NB) return fail(GS_EINVAL, "node/bucket out of range");
  const size_t ent = (size_t)node * NB + bucket;
  std::vector<uint32_t> row(e->ASZP);
  uint16_t hv = 0;
  HIPC(hipMemcpyAsync(row.data(), e->peers + ent * e->ASZP, e->ASZP * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(&hv, e->hl + ent, 2, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  const uint32_t head = hv & 0xFF, L = hv >> 8;
  *len = L;
  if (L > cap) return fail(GS_ERANGE, "peers buffer too small");
  for (uint32_t j = 0; j < L; ++j) peers[j] = row[(head + j) % e->ASZ];
  return GS_OK;
}

int gs_fail_nodes(gs_engine* eh, const double* fraction) {
  ENGINE(eh);
  if (!fraction) return fail(GS_EINVAL, "null fractions");
  if (!e->failed_ranked) {
    DevScratch sc;
    uint64_t* keys = nullptr;
    uint32_t *ids = nullptr, *sorted = nullptr;
    if (!sc.get(&keys, e->N * 8ull) || !sc.get(&ids, e->N * 4ull) || !sc.get(&sorted, e->N * 4ull))
      return fail(GS_ENOMEM, "fail_nodes scratch");
    HIPC(launch_fail_keys(*e, keys, ids));
    if (int s = sort_ids_by_key(*e, keys, sorted)) return s;
    HIPC(launch_scatter_rank(*e, sorted, e->frank));
    HIPC(hipStreamSynchronize(e->st));
    e->failed_ranked = true;
  }
  std::vector<uint32_t> nf(e->S);
  HIPC(hipMemcpyAsync(nf.data(), e->nfail, e->S * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  for (uint32_t o = 0; o < e->S; ++o) {
    const double f = fraction[o] * (double)e->N;  // (fraction * nodes.len() as f64) as usize
    uint64_t k = (f > 0.0) ? (uint64_t)f : 0;     // saturating cast, NaN -> 0
    if (f >= 1.8446744073709552e19) k = ~0ull;
    if (k > e->N) return fail(GS_ERANGE, "fail_nodes: fraction * n exceeds the cluster (reference panics)");
    nf[o] = std::max(nf[o], (uint32_t)k);
    e->h_nfail_any[o] = nf[o] ? 1u : 0u;
  }
  HIPC(mv_update_failures(*e, nf));
  for (auto& pv : e->mv_pred) pv.clear();  // failures reshape the levels: the next round polls again
  if (e->mv_prof) {  // (and ignores profiles published before now)
    const size_t ng = e->mv_pred.size();
    for (size_t g = 0; g < ng; ++g) e->mv_prof_seen[g] = ((volatile uint32_t*)e->mv_prof)[g * MV_PROF_WORDS];
  }
  HIPC(hipMemcpyAsync(e->nfail, nf.data(), e->S * 4, hipMemcpyHostToDevice, e->st));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

static int need_slots(Engine* e) {
  if (!e->slots_set) return fail(GS_ESTATE, "gs_set_slots has not been called");
  return GS_OK;
}

// Applies a rotation's deferred prune-bit clear (left by the one-kernel gs_round)
// before anything else reads or changes the prune masks.
static int flush_rot_clear(Engine* e) {
  if (!e->rot_clear_pending) return GS_OK;
  e->rot_clear_pending = false;
  HIPC(launch_rotate_clear(*e));
  return GS_OK;
}

// The step-wise gather's inbound rows [capin][PAIRS]: the multi-source BFS allocates them
// on first use (its gs_round consumes the records on-chip and never needs them).
static int ensure_inb(Engine* e) {
  if (e->inb) return GS_OK;
  const size_t b0 = e->dev_bytes;
  const int s = dalloc(*e, &e->inb, (size_t)e->capin * e->PAIRS, 0);
  e->pair_bytes += e->dev_bytes - b0;
  return s;
}

static int refuse_part(Engine* e) {
  return e->part_on ? fail(GS_ESTATE, "a node-range partition rank runs rounds with gs_part_round") : GS_OK;
}

// Maps a BFS launcher's result: depth beyond u8 hops, a level that never finished, HIP errors.
static int bfs_result(Engine* e, hipError_t r, const char* what) {
  if (r == hipSuccess) return GS_OK;
  if (r == hipErrorNotSupported) return fail(GS_ERANGE, "BFS depth exceeds 254 hops (hop counts are u8)");
  if (r == hipErrorLaunchTimeOut)
    return fail(GS_EHIP, std::string(what) + ": BFS level " + std::to_string(e->bfs_level) +
                             " did not finish within GS_LEVEL_WAIT_S (default 60 s); the device is stuck");
  return fail(GS_EHIP, std::string(what) + ": " + hipGetErrorString(r));
}

static int do_bfs(Engine* e, bool record) {
  if (int s = refuse_part(e)) return s;
  if (int s = ensure_inb(e)) return s;
  hipEvent_t t0 = nullptr;
  const bool self_timed = mv_layout(*e);  // times its levels and its gather itself
  if (!self_timed) e->tbegin("bfs", &t0);
  hipError_t r = launch_bfs(*e, record);
  if (!self_timed) e->tend("bfs", t0);
  e->inb_valid = true;
  return bfs_result(e, r, "launch_bfs");
}

int gs_run_gossip(gs_engine* eh) {
  ENGINE(eh);
  if (int s = need_slots(e)) return s;
  if (int s = flush_rot_clear(e)) return s;
  return do_bfs(e, false);
}

static int do_cp(Engine* e, bool c, bool p, bool a, bool record = false) {
  if (int s = refuse_part(e)) return s;
  if (int s = flush_rot_clear(e)) return s;
  hipEvent_t t0;
  e->tbegin("consume", &t0);
  hipError_t r = launch_consume_prune(*e, c, p, a, record);
  e->tend("consume", t0);
  HIPC(r);
  return GS_OK;
}
int gs_consume_messages(gs_engine* eh) { ENGINE(eh); if (int s = need_slots(e)) return s; return do_cp(e, true, false, false); }
int gs_send_prunes(gs_engine* eh) { ENGINE(eh); if (int s = need_slots(e)) return s; return do_cp(e, false, true, false); }
int gs_prune_connections(gs_engine* eh) { ENGINE(eh); if (int s = need_slots(e)) return s; return do_cp(e, false, false, true); }

int gs_chance_to_rotate(gs_engine* eh, uint32_t round) {
  ENGINE(eh);
  if (int s = need_slots(e)) return s;
  if (round >= (1u << 27)) return fail(GS_ERANGE, "round index must be < 2^27");
  if (int s = flush_rot_clear(e)) return s;
  hipEvent_t t0;
  e->tbegin("rotate", &t0);
  hipError_t r = launch_rotate(*e, round, false);
  e->tend("rotate", t0);
  HIPC(r);
  return GS_OK;
}

static int drain_summaries(Engine* e) {
  if (!e->sum_used) return GS_OK;
  size_t n = (size_t)e->sum_used * e->S;
  size_t old = e->h_sum.size();
  e->h_sum.resize(old + n);
  HIPC(hipMemcpyAsync(e->h_sum.data() + old, e->sum, n * sizeof(gs_round_summary), hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  e->sum_used = 0;
  return GS_OK;
}

static int do_stats(Engine* e, int mode) {
  hipEvent_t t0;
  e->tbegin("stats", &t0);
  hipError_t r = launch_stats(*e, e->sum_used, mode);
  e->tend("stats", t0);
  HIPC(r);
  if (++e->sum_used == e->sum_cap) return drain_summaries(e);
  return GS_OK;
}

int gs_record_round(gs_engine* eh) {
  ENGINE(eh);
  if (int s = refuse_part(e)) return s;
  if (int s = need_slots(e)) return s;
  return do_stats(e, 0);
}

// The fused round with its rotation ahead (Engine::rot_ahead_ok): rotation `round` runs
// in workgroup 0 of the round kernel into the other row buffer, concurrently with the
// slots' workgroups on the current one, and the buffers swap after the launch (no rotation
// launch, nothing between two round kernels).
// The second row buffer and the alternate rotation list / changed-bit buffers. All four
// or none: a failed allocation frees the ones made, so a retried call allocates again
// (a partial set left peers2 set and a later round wrote through a null hl2).
static int ensure_rot_ahead(Engine* e) {
  if (e->peers2 && e->hl2 && e->rot_list_b[1] && e->rot_changed_b[1]) return GS_OK;
  const size_t N = e->N;
  int s = GS_OK;
  if (!e->peers2) s = dalloc(*e, &e->peers2, N * NB * e->ASZP, 0);
  if (!s && !e->hl2) s = dalloc(*e, &e->hl2, N * NB, 0);
  if (!s && !e->rot_list_b[1]) s = dalloc(*e, &e->rot_list_b[1], N, 0);
  if (!s && !e->rot_changed_b[1]) s = dalloc(*e, &e->rot_changed_b[1], N * NB, 0);
  if (s) {
    dfree(*e, e->peers2, N * NB * e->ASZP);
    dfree(*e, e->hl2, N * NB);
    dfree(*e, e->rot_list_b[1], N);
    dfree(*e, e->rot_changed_b[1], N * NB);
    return s;
  }
  e->rot_list_b[0] = e->rot_list;
  e->rot_changed_b[0] = e->rot_changed;
  e->rows2_stale = true;
  return GS_OK;
}

static int round_ahead(Engine* e, uint32_t round, bool rec) {
  if (int s = ensure_rot_ahead(e)) return s;
  if (e->rows2_stale) {  // (first round, or the rows changed in place since)
    HIPC(hipMemcpyAsync(e->peers2, e->peers, (size_t)e->N * NB * e->ASZP * 4, hipMemcpyDeviceToDevice, e->st));
    HIPC(hipMemcpyAsync(e->hl2, e->hl, (size_t)e->N * NB * 2, hipMemcpyDeviceToDevice, e->st));
    e->rows2_stale = false;
    e->rows2_pending = -1;
  }
  const uint32_t par = round & 1u;
  RotAhead ra;
  ra.peers2 = e->peers2;
  ra.hl2 = e->hl2;
  // the list / changed-bit buffers the round kernel's clear does not read (it reads the last rotation's)
  ra.list = e->rot_list == e->rot_list_b[0] ? e->rot_list_b[1] : e->rot_list_b[0];
  ra.changed = e->rot_changed == e->rot_changed_b[0] ? e->rot_changed_b[1] : e->rot_changed_b[0];
  ra.count = e->rot_count + par;
  ra.plist = e->rows2_pending >= 0 ? e->rot_list : nullptr;  // the previous ahead rotation's nodes
  ra.pcount = e->rot_count + (e->rows2_pending >= 0 ? (uint32_t)e->rows2_pending : 0u);
  ra.round = round;
  hipEvent_t t0;
  e->tbegin("round", &t0);
  const bool clr = e->rot_clear_pending;  // the last rotation's clear runs inside the round kernel
  hipError_t r = launch_round_wg(*e, rec, e->sum_used, clr, &ra);
  e->tend("round", t0);
  HIPC(r);
  std::swap(e->peers, e->peers2);
  std::swap(e->hl, e->hl2);
  e->rows2_pending = (int)par;
  e->rot_list = ra.list;
  e->rot_changed = ra.changed;
  e->rot_parity = par;
  e->rot_have_prev = true;
  e->rot_clear_pending = true;
  e->rot_cnt_dirty = true;  // (the other counter was not zeroed)
  e->inb_valid = false;
  if (rec && ++e->sum_used == e->sum_cap) return drain_summaries(e);
  return GS_OK;
}

int gs_round(gs_engine* eh, uint32_t round, int record) {
  ENGINE(eh);
  if (int s = refuse_part(e)) return s;
  if (int s = need_slots(e)) return s;
  const bool rec = record != 0;
  if (e->fused) {  // BFS + consume + prune + statistics in one kernel per slot
    if (round >= (1u << 27)) return fail(GS_ERANGE, "round index must be < 2^27");
    if (e->rot_ahead_ok && !(e->rot_have_prev && (round & 1u) == e->rot_parity)) return round_ahead(e, round, rec);
    hipEvent_t t0;
    e->tbegin("round", &t0);
    const bool clr = e->rot_clear_pending;  // the last rotation's clear runs inside the round kernel
    hipError_t r = launch_round_wg(*e, rec, e->sum_used, clr);
    e->tend("round", t0);
    HIPC(r);
    e->rot_clear_pending = false;
    e->inb_valid = false;
    e->tbegin("rotate", &t0);
    r = launch_rotate(*e, round, true);
    e->tend("rotate", t0);
    HIPC(r);
    if (rec && ++e->sum_used == e->sum_cap) return drain_summaries(e);
    return GS_OK;
  }
  if (int s = flush_rot_clear(e)) return s;
  if (e->bfs_mode == GS_BFS_MULTI && e->mv_fused) {  // gather fused with consume: the inbound rows stay on-chip
    hipError_t r = launch_bfs_multi(*e, rec, true);
    e->inb_valid = false;
    if (int s = bfs_result(e, r, "launch_bfs_multi")) return s;
    hipEvent_t t0;
    e->tbegin("consume", &t0);
    r = hipMemsetAsync(e->slot_prunes, 0, e->S * 4, e->st);
    if (r == hipSuccess) r = launch_consume_prune_g(*e, rec, false);
    e->tend("consume", t0);
    HIPC(r);
  } else {
    if (int s = do_bfs(e, rec)) return s;
    if (int s = do_cp(e, true, true, true, rec)) return s;
  }
  if (int s = gs_chance_to_rotate(eh, round)) return s;
  if (rec) return do_stats(e, e->bfs_mode == GS_BFS_WORKGROUP ? 2 : mv_layout(*e) ? 4 : 1);
  return GS_OK;
}

// ------------------------------------------------------------ readbacks ----
#define SLOT_CHECK(slot) \
  if ((slot) >= e->S) return fail(GS_EINVAL, "slot out of range");

int gs_read_hops(gs_engine* eh, uint32_t slot, uint8_t* hops) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  if (e->part_on) std::memset(hops, 0xFF, e->N);  // a partition rank knows its own nodes' hops
  HIPC(hipMemcpyAsync(hops + e->vlo, e->hops + (size_t)slot * e->NP, e->NP, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_read_inbound(gs_engine* eh, uint32_t slot, uint32_t* off, uint32_t* src, uint8_t* hop, size_t cap) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  if (!e->inb_valid)
    return fail(GS_ESTATE, "inbound records are kept on-chip by gs_round (the one-kernel round, or the "
                           "multi-source BFS's fused gather + consume); call gs_run_gossip to materialize them");
  const size_t N = e->N, base = (size_t)slot * N;
  std::vector<uint32_t> cnt(N), recs(N * e->capin);
  HIPC(hipMemcpyAsync(cnt.data(), e->cnt + base, N * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpy2DAsync(recs.data(), N * 4, e->inb + base, e->PAIRS * 4, N * 4, e->capin, hipMemcpyDeviceToHost,
                        e->st));
  HIPC(hipStreamSynchronize(e->st));
  size_t total = 0;
  for (size_t v = 0; v < N; ++v) total += cnt[v];
  if (total > cap) return fail(GS_ERANGE, "inbound buffer too small");
  off[0] = 0;
  size_t w = 0;
  std::vector<uint32_t> lst;
  for (size_t v = 0; v < N; ++v) {
    lst.clear();
    for (uint32_t j = 0; j < cnt[v]; ++j) lst.push_back(recs[(size_t)j * N + v]);
    std::sort(lst.begin(), lst.end());
    for (uint32_t r : lst) { src[w] = r & 0xFFFFFFu; hop[w] = (uint8_t)(r >> 24); ++w; }
    off[v + 1] = (uint32_t)w;
  }
  return GS_OK;
}

// Copies the cache columns of one slot and splits the slot words (ck_make):
// keys [CACHE_CAP][NP] node ids, scores [CACHE_CAP][NP] score | PRUNED_FLAG (column i =
// node vlo + i).
static int read_cache_slot(Engine* e, uint32_t slot, std::vector<uint32_t>& meta, std::vector<uint32_t>& keys,
                           std::vector<uint8_t>& scores) {
  const size_t N = e->NP, base = (size_t)slot * N;
  meta.resize(N); keys.resize(N * CACHE_CAP); scores.resize(N * CACHE_CAP);
  HIPC(hipMemcpyAsync(meta.data(), e->cmeta + base, N * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpy2DAsync(keys.data(), N * 4, e->ckey + base, e->PAIRS * 4, N * 4, CACHE_CAP, hipMemcpyDeviceToHost,
                        e->st));
  HIPC(hipStreamSynchronize(e->st));
  for (size_t i = 0; i < keys.size(); ++i) {
    scores[i] = (uint8_t)(keys[i] >> 24);
    keys[i] = ck_id(keys[i]);
  }
  return GS_OK;
}

int gs_read_prunes(gs_engine* eh, uint32_t slot, uint32_t* pruner, uint32_t* prunee, size_t cap, size_t* count) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  std::vector<uint32_t> meta, keys;
  std::vector<uint8_t> sc;
  if (int s = read_cache_slot(e, slot, meta, keys, sc)) return s;
  std::vector<std::pair<uint32_t, uint32_t>> pr;
  const size_t N = e->NP;  // a partition rank reports its own pruners
  for (size_t v = 0; v < N; ++v) {
    const uint32_t plen = (meta[v] >> 16) & 0xFF;
    for (uint32_t i = 0; i < plen; ++i)
      if (sc[i * N + v] & PRUNED_FLAG) pr.push_back({(uint32_t)(e->vlo + v), keys[i * N + v]});
  }
  std::sort(pr.begin(), pr.end());
  *count = pr.size();
  if (pr.size() > cap) return fail(GS_ERANGE, "prunes buffer too small");
  for (size_t i = 0; i < pr.size(); ++i) { pruner[i] = pr[i].first; prunee[i] = pr[i].second; }
  return GS_OK;
}

int gs_read_cache(gs_engine* eh, uint32_t slot, uint32_t node, uint32_t* up, uint32_t* keys, uint32_t* scores,
                  uint32_t cap, uint32_t* len) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (node >= e->N) return fail(GS_EINVAL, "node out of range");
  if (node - e->vlo >= e->NP) return fail(GS_EINVAL, "node is not owned by this partition rank");
  if (int s = check_err(e)) return s;
  const size_t p = (size_t)slot * e->NP + (node - e->vlo);
  uint32_t meta = 0;
  uint32_t* dk = nullptr;
  HIPC(hipMalloc(&dk, CACHE_CAP * 4));
  HIPC(hipMemcpyAsync(&meta, e->cmeta + p, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(launch_gather_strided_u32(*e, e->ckey + p, e->PAIRS, CACHE_CAP, dk));
  std::vector<uint32_t> k(CACHE_CAP);
  HIPC(hipMemcpyAsync(k.data(), dk, CACHE_CAP * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  hipFree(dk);
  const uint32_t L = meta & 0xFF;
  *up = (meta >> 8) & 0xFF;
  *len = L;
  if (L > cap) return fail(GS_ERANGE, "cache buffer too small");
  std::vector<std::pair<uint32_t, uint32_t>> v;
  for (uint32_t i = 0; i < L; ++i) v.push_back({ck_id(k[i]), ck_score(k[i])});
  std::sort(v.begin(), v.end());
  for (uint32_t i = 0; i < L; ++i) { keys[i] = v[i].first; scores[i] = v[i].second; }
  return GS_OK;
}

int gs_read_pruned(gs_engine* eh, uint32_t slot, uint32_t node, uint32_t* fifo_mask) {
  ENGINE(eh);
  if (int s_ = flush_rot_clear(e)) return s_;
  SLOT_CHECK(slot);
  if (node >= e->N) return fail(GS_EINVAL, "node out of range");
  if (int s = check_err(e)) return s;
  uint32_t m = 0, org = e->slots[slot].origin;
  uint8_t bn = 0, bo = 0;
  HIPC(hipMemcpyAsync(&m, e->mask + slot * e->mso + node * e->msu, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(&bn, e->bucket + node, 1, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(&bo, e->bucket + org, 1, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  const size_t ent = (size_t)node * NB + std::min(bn, bo);
  uint16_t hv = 0;
  HIPC(hipMemcpy(&hv, e->hl + ent, 2, hipMemcpyDeviceToHost));
  const uint32_t head = hv & 0xFF, L = hv >> 8;
  uint32_t out = 0;
  for (uint32_t j = 0; j < L; ++j)
    if ((m >> ((head + j) % e->ASZ)) & 1u) out |= 1u << j;
  *fifo_mask = out;
  return GS_OK;
}

int gs_read_active_sets(gs_engine* eh, uint32_t* peers, uint8_t* len) {
  ENGINE(eh);
  if (int s = check_err(e)) return s;
  const size_t ents = (size_t)e->N * NB;
  std::vector<uint32_t> rows(ents * e->ASZP);
  std::vector<uint16_t> hl(ents);
  HIPC(hipMemcpyAsync(rows.data(), e->peers, rows.size() * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(hl.data(), e->hl, ents * 2, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  for (size_t ent = 0; ent < ents; ++ent) {
    const uint32_t head = hl[ent] & 0xFF, L = hl[ent] >> 8;
    len[ent] = (uint8_t)L;
    for (uint32_t j = 0; j < e->ASZ; ++j)
      peers[ent * e->ASZ + j] = j < L ? rows[ent * e->ASZP + (head + j) % e->ASZ] : 0xFFFFFFFFu;
  }
  return GS_OK;
}

int gs_read_caches(gs_engine* eh, uint32_t slot, uint32_t* up, uint32_t* len, uint32_t* keys, uint32_t* scores) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  std::vector<uint32_t> meta, k;
  std::vector<uint8_t> sc;
  if (int s = read_cache_slot(e, slot, meta, k, sc)) return s;
  const size_t N = e->NP;
  std::vector<std::pair<uint32_t, uint32_t>> v;
  for (size_t n0 = 0; n0 < e->N; ++n0) {
    const size_t n = n0 - e->vlo;  // column of node n0 (a partition rank's own nodes only)
    const bool own = n < N;
    const uint32_t L = own ? meta[n] & 0xFF : 0u;
    up[n0] = own ? (meta[n] >> 8) & 0xFF : 0u;
    len[n0] = L;
    v.clear();
    for (uint32_t i = 0; i < L; ++i) v.push_back({k[i * N + n], (uint32_t)(sc[i * N + n] & 0x7F)});
    std::sort(v.begin(), v.end());
    for (uint32_t i = 0; i < CACHE_CAP; ++i) {
      keys[n0 * CACHE_CAP + i] = i < L ? v[i].first : 0xFFFFFFFFu;
      scores[n0 * CACHE_CAP + i] = i < L ? v[i].second : 0;
    }
  }
  return GS_OK;
}

// n elements of elem bytes, stride bytes apart, device -> host: one contiguous copy per
// chunk of 2^20 elements, picked on the host (a 2D copy of 1- or 4-byte rows runs row by
// row: minutes at 10M nodes).
static hipError_t strided_d2h(Engine* e, void* dst, const void* src, size_t elem, size_t stride, size_t n) {
  const size_t CH = (size_t)1 << 20;
  std::vector<uint8_t> tmp;
  for (size_t i0 = 0; i0 < n; i0 += CH) {
    const size_t c = std::min(CH, n - i0), span = (c - 1) * stride + elem;
    tmp.resize(span);
    hipError_t r = hipMemcpyAsync(tmp.data(), (const uint8_t*)src + i0 * stride, span, hipMemcpyDeviceToHost, e->st);
    if (r == hipSuccess) r = hipStreamSynchronize(e->st);
    if (r != hipSuccess) return r;
    for (size_t i = 0; i < c; ++i) std::memcpy((uint8_t*)dst + (i0 + i) * elem, tmp.data() + i * stride, elem);
  }
  return hipSuccess;
}

int gs_read_pruned_all(gs_engine* eh, uint32_t slot, uint32_t* fifo_mask) {
  ENGINE(eh);
  if (int s_ = flush_rot_clear(e)) return s_;
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  const size_t N = e->N;
  std::vector<uint32_t> m(N);
  std::vector<uint8_t> b(N);
  std::vector<uint16_t> hl(N * NB);
  if (e->msu == 1) {
    HIPC(hipMemcpyAsync(m.data(), e->mask + slot * e->mso, N * 4, hipMemcpyDeviceToHost, e->st));
  } else {
    HIPC(strided_d2h(e, m.data(), e->mask + slot * e->mso, 4, e->msu * 4, N));
  }
  HIPC(hipMemcpyAsync(b.data(), e->bucket, N, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(hl.data(), e->hl, N * NB * 2, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  const uint32_t bo = b[e->slots[slot].origin];
  for (size_t n = 0; n < N; ++n) {
    const uint16_t hv = hl[n * NB + std::min<uint32_t>(b[n], bo)];
    const uint32_t head = hv & 0xFF, L = hv >> 8;
    uint32_t out = 0;
    for (uint32_t j = 0; j < L; ++j)
      if ((m[n] >> ((head + j) % e->ASZ)) & 1u) out |= 1u << j;
    fifo_mask[n] = out;
  }
  return GS_OK;
}

int gs_read_counters(gs_engine* eh, uint32_t slot, uint32_t* egress, uint32_t* ingress, uint32_t* prune_sent) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  const size_t N = e->NP, base = (size_t)slot * N, o = e->vlo;  // a partition rank: its own nodes, 0 elsewhere
  std::vector<uint8_t> eg(N), hp(N), pr(N);
  if (e->esu == 1) {
    HIPC(hipMemcpyAsync(eg.data(), e->egress + slot * e->eso, N, hipMemcpyDeviceToHost, e->st));
  } else {
    HIPC(strided_d2h(e, eg.data(), e->egress + slot * e->eso, 1, e->esu, N));
  }
  HIPC(hipMemcpyAsync(hp.data(), e->hops + base, N, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(pr.data(), e->prune_round + base, N, hipMemcpyDeviceToHost, e->st));
  if (ingress) {
    if (e->part_on) std::memset(ingress, 0, (size_t)e->N * 4);
    HIPC(hipMemcpyAsync(ingress + o, e->cnt + base, N * 4, hipMemcpyDeviceToHost, e->st));
  }
  HIPC(hipStreamSynchronize(e->st));
  if (e->part_on) {
    if (egress) std::memset(egress, 0, (size_t)e->N * 4);
    if (prune_sent) std::memset(prune_sent, 0, (size_t)e->N * 4);
  }
  for (size_t v = 0; v < N; ++v) {
    if (egress) egress[o + v] = hp[v] != 0xFF ? eg[v] : 0;
    if (prune_sent) prune_sent[o + v] = pr[v];
  }
  return GS_OK;
}

int gs_read_round_summaries(gs_engine* eh, gs_round_summary* out, size_t cap, size_t* count) {
  ENGINE(eh);
  if (int s = check_err(e)) return s;
  if (int s = drain_summaries(e)) return s;
  *count = e->h_sum.size();
  if (e->h_sum.size() > cap) return fail(GS_ERANGE, "summary buffer too small");
  std::memcpy(out, e->h_sum.data(), e->h_sum.size() * sizeof(gs_round_summary));
  return GS_OK;
}

int gs_read_accumulators(gs_engine* eh, uint32_t slot, uint64_t* egress, uint64_t* ingress, uint64_t* prunes,
                         uint32_t* stranded_times, uint64_t* hop_hist) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (int s = check_err(e)) return s;
  const size_t N = e->NP, base = (size_t)slot * N, o = e->vlo;  // a partition rank: its own nodes, 0 elsewhere
  std::vector<uint32_t> a(N), b(N), c(N);
  HIPC(hipMemcpyAsync(a.data(), e->egress_acc + base, N * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(b.data(), e->ingress_acc + base, N * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(c.data(), e->prune_acc + base, N * 4, hipMemcpyDeviceToHost, e->st));
  if (stranded_times) {
    if (e->part_on) std::memset(stranded_times, 0, (size_t)e->N * 4);
    HIPC(hipMemcpyAsync(stranded_times + o, e->strand + base, N * 4, hipMemcpyDeviceToHost, e->st));
  }
  if (hop_hist) HIPC(hipMemcpyAsync(hop_hist, e->hist_acc + (size_t)slot * 256, 256 * 8, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  if (e->part_on) {
    if (egress) std::memset(egress, 0, (size_t)e->N * 8);
    if (ingress) std::memset(ingress, 0, (size_t)e->N * 8);
    if (prunes) std::memset(prunes, 0, (size_t)e->N * 8);
  }
  for (size_t v = 0; v < N; ++v) {
    if (egress) egress[o + v] = a[v];
    if (ingress) ingress[o + v] = b[v];
    if (prunes) prunes[o + v] = c[v];
  }
  return GS_OK;
}

int gs_read_failed(gs_engine* eh, uint32_t slot, uint8_t* failed) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  std::vector<uint32_t> fr(e->N);
  uint32_t nf = 0;
  HIPC(hipMemcpyAsync(fr.data(), e->frank, e->N * 4ull, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(&nf, e->nfail + slot, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  for (uint32_t v = 0; v < e->N; ++v) failed[v] = nf && fr[v] < nf;
  return GS_OK;
}

int gs_kernel_time(gs_engine* eh, const char* family, double* ms, uint64_t* launches) {
  ENGINE(eh);
  HIPC(hipStreamSynchronize(e->st));
  if (family && std::strncmp(family, "phase.", 6) == 0) {  // workgroup-ms per round-kernel phase (100 MHz clock)
    *ms = 0;
    *launches = 0;
    const int ph = family[6] - 'A';
    if (!e->phase_clk || ph < 0 || ph >= 32) return GS_OK;
    unsigned long long v[32];
    HIPC(hipMemcpy(v, e->phase_clk, sizeof(v), hipMemcpyDeviceToHost));
    *ms = (double)v[ph] * 1e-5;
    *launches = e->timers["round"].n;
    return GS_OK;
  }
  auto it = e->timers.find(family ? family : "");
  *ms = 0;
  *launches = 0;
  if (it == e->timers.end()) return GS_OK;
  auto& t = it->second;
  for (auto& pr : t.ev) {
    float x = 0;
    hipEventElapsedTime(&x, pr.first, pr.second);
    t.ms += x;
    t.n += 1;
    e->ev_pool.push_back(pr.first);
    e->ev_pool.push_back(pr.second);
  }
  t.ev.clear();
  *ms = t.ms;
  *launches = t.n;
  return GS_OK;
}

int gs_kernel_time_reset(gs_engine* eh) {
  ENGINE(eh);
  HIPC(hipStreamSynchronize(e->st));
  for (auto& kv : e->timers) {
    for (auto& pr : kv.second.ev) { e->ev_pool.push_back(pr.first); e->ev_pool.push_back(pr.second); }
    kv.second.ev.clear();
    kv.second.ms = 0;
    kv.second.n = 0;
  }
  if (e->phase_clk) HIPC(hipMemsetAsync(e->phase_clk, 0, 256, e->st));
  return GS_OK;
}

int gs_engine_round_kind(gs_engine* eh, uint32_t* fused) {
  ENGINE(eh);
  if (!fused) return fail(GS_EINVAL, "null argument");
  *fused = e->fused ? 1u : 0u;
  return GS_OK;
}

int gs_engine_bfs_geometry(gs_engine* eh, uint32_t* out, size_t n) {
  ENGINE(eh);
  if (!out || n < 5) return fail(GS_EINVAL, "gs_engine_bfs_geometry: need 5 words");
  const bool on = mv_layout(*e);
  out[0] = on ? e->mv.XT : 0;
  out[1] = on ? e->mv.nbc : 0;
  out[2] = on ? e->mv.nbf : 0;
  out[3] = on ? e->mv.GW : 0;
  out[4] = on ? (uint32_t)e->mv_groups.size() : 0;
  if (n >= 6) out[5] = pb_usable(*e) ? e->pb_G : 0;  // workgroups of the persistent BFS (0: launched level loop)
  return GS_OK;
}

int gs_engine_info(gs_engine* eh, uint32_t* n_nodes, uint32_t* n_slots, uint32_t* bfs_mode, uint64_t* bytes) {
  Engine* e = reinterpret_cast<Engine*>(eh);
  if (!e) return fail(GS_EINVAL, "null engine");
  if (n_nodes) *n_nodes = e->N;
  if (n_slots) *n_slots = e->S;
  if (bfs_mode) *bfs_mode = e->bfs_mode;
  if (bytes) *bytes = e->dev_bytes;
  return GS_OK;
}

int gs_engine_memory(gs_engine* eh, uint64_t* pair_bytes, uint64_t* other_bytes) {
  ENGINE(eh);
  if (pair_bytes) *pair_bytes = e->pair_bytes;
  if (other_bytes) *other_bytes = e->dev_bytes - e->pair_bytes;
  return GS_OK;
}

// ----------------------------------------------------------------- MST ----
// Cluster::mst (gossip.rs:580-591): the first discoverer of every reached node in the
// reference's FIFO queue order. The queue is level by level; within a level, nodes are
// in the order (queue position of the discoverer, index of the node in the
// discoverer's push list = PushActiveSet::get_nodes(..).take(fanout), failed peers
// included). The discoverer of w is its pusher from the previous level with the
// smallest queue position. Debug readback, from the step path's inbound records.
int gs_read_mst(gs_engine* eh, uint32_t slot, uint32_t* parent) {
  ENGINE(eh);
  SLOT_CHECK(slot);
  if (!parent) return fail(GS_EINVAL, "null argument");
  if (!e->inb_valid)
    return fail(GS_ESTATE, "inbound records are kept on-chip by gs_round (the one-kernel round, or the "
                           "multi-source BFS's fused gather + consume); call gs_run_gossip to materialize them");
  if (int s = refuse_part(e)) return s;
  if (e->N > (1u << 18)) return fail(GS_ERANGE, "gs_read_mst is a debug readback for n <= 262,144");
  const uint32_t N = e->N, org = e->slots[slot].origin;
  std::vector<uint8_t> hops(N);
  if (int s = gs_read_hops(eh, slot, hops.data())) return s;
  std::vector<uint32_t> cnt(N);
  HIPC(hipMemcpy(cnt.data(), e->cnt + (size_t)slot * N, N * 4ull, hipMemcpyDeviceToHost));
  size_t total = 0;
  for (uint32_t x : cnt) total += std::min(x, e->capin);
  std::vector<uint32_t> off(N + 1), src(total + 1);
  std::vector<uint8_t> rh(total + 1);
  if (int s = gs_read_inbound(eh, slot, off.data(), src.data(), rh.data(), total + 1)) return s;
  std::vector<uint32_t> peers((size_t)N * NB * e->ASZ), fifo(N);
  std::vector<uint8_t> lens((size_t)N * NB), bkt(N);
  if (int s = gs_read_active_sets(eh, peers.data(), lens.data())) return s;
  if (int s = gs_read_pruned_all(eh, slot, fifo.data())) return s;
  HIPC(hipMemcpy(bkt.data(), e->bucket, N, hipMemcpyDeviceToHost));
  // index of w in u's take(fanout) list (get_nodes skips pruned peers and the origin)
  auto take_index = [&](uint32_t u, uint32_t w) -> uint32_t {
    const size_t ent = (size_t)u * NB + std::min(bkt[u], bkt[org]);
    uint32_t t = 0;
    for (uint32_t i = 0; i < lens[ent] && t < e->fanout; ++i) {
      const uint32_t p = peers[ent * e->ASZ + i];
      if (((fifo[u] >> i) & 1u) || p == org) continue;
      if (p == w) return t;
      ++t;
    }
    return 63;  // not reached for a recorded push
  };
  std::vector<uint64_t> pos(N, UINT64_MAX);
  for (uint32_t v = 0; v < N; ++v) parent[v] = UINT32_MAX;
  uint32_t maxd = 0;
  for (uint32_t v = 0; v < N; ++v)
    if (hops[v] != 0xFF) maxd = std::max<uint32_t>(maxd, hops[v]);
  std::vector<std::vector<uint32_t>> level(maxd + 1);
  for (uint32_t v = 0; v < N; ++v)
    if (hops[v] != 0xFF) level[hops[v]].push_back(v);
  pos[org] = 0;
  for (uint32_t d = 1; d <= maxd; ++d) {
    std::vector<std::pair<uint64_t, uint32_t>> keyed;
    for (uint32_t w : level[d]) {
      uint32_t best = UINT32_MAX;
      for (uint32_t i = off[w]; i < off[w + 1]; ++i)
        if (rh[i] == d && (best == UINT32_MAX || pos[src[i]] < pos[best])) best = src[i];
      if (best == UINT32_MAX) return fail(GS_ESTATE, "reached node without a pusher from the previous level");
      parent[w] = best;
      keyed.push_back({(pos[best] << 6) | take_index(best, w), w});
    }
    std::sort(keyed.begin(), keyed.end());
    for (size_t r = 0; r < keyed.size(); ++r) pos[keyed[r].second] = r;
  }
  return GS_OK;
}

// ---------------------------------------------------- node-range partition ----
#define PART(eh)                                                            \
  ENGINE(eh);                                                               \
  if (!e->part_on) return fail(GS_ESTATE, "not a node-range partition rank (gs_create_part)");

static hipMemcpyKind kind_to(int dev) { return dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost; }
static hipMemcpyKind kind_from(int dev) { return dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice; }

int gs_part_sizes(gs_engine* eh, size_t* stats_words, uint32_t* lo, uint32_t* hi) {
  PART(eh);
  if (stats_words) *stats_words = part_stats_words(*e);
  if (lo) *lo = e->part_lo;
  if (hi) *hi = e->part_hi;
  return GS_OK;
}

int gs_part_round(gs_engine* eh, uint32_t round, int record, uint32_t* n_records) {
  PART(eh);
  if (e->part_x) return fail(GS_ESTATE, "a frontier-exchange rank runs its BFS with gs_part_xbfs_* (and gs_part_xround_finish)");
  if (!n_records) return fail(GS_EINVAL, "null argument");
  if (int s = need_slots(e)) return s;
  if (round >= (1u << 27)) return fail(GS_ERANGE, "round index must be < 2^27");
  if (int s = flush_rot_clear(e)) return s;
  const bool rec = record != 0;
  HIPC(hipMemsetAsync(e->part_cnt, 0, 4, e->st));
  hipError_t r = launch_bfs_multi(*e, rec, true);  // the whole BFS; gather + consume of own nodes
  e->inb_valid = false;
  if (int s = bfs_result(e, r, "launch_bfs_multi")) return s;
  hipEvent_t t0;
  e->tbegin("consume", &t0);
  r = hipMemsetAsync(e->slot_prunes, 0, e->S * 4, e->st);
  if (r == hipSuccess) r = launch_consume_prune_g(*e, rec, false);  // send_prunes of own pruners
  if (r == hipSuccess) r = launch_part_emit(*e);                    // ... as records for the other ranks
  e->tend("consume", t0);
  HIPC(r);
  HIPC(hipMemcpyAsync(e->h_err + 1, e->part_cnt, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  if (int s = check_err(e)) return s;
  e->part_nrec = e->h_err[1];  // (more than part_rec_cap: only the dense exchange can carry this round)
  *n_records = e->part_nrec;
  return GS_OK;
}

#define PARTX(eh)                                                                               \
  PART(eh);                                                                                     \
  if (!e->part_x) return fail(GS_ESTATE, "not a frontier-exchange rank (GS_FLAG_FRONTIER_EXCHANGE)");

int gs_part_xbfs_groups(gs_engine* eh, uint32_t* n_groups) {
  PARTX(eh);
  if (int s = need_slots(e)) return s;
  if (!n_groups) return fail(GS_EINVAL, "null argument");
  *n_groups = (uint32_t)e->mv_groups.size();
  return GS_OK;
}

int gs_part_xbfs_begin(gs_engine* eh, uint32_t group, uint32_t* n_local) {
  PARTX(eh);
  if (int s = need_slots(e)) return s;
  if (!n_local || group >= e->mv_groups.size()) return fail(GS_EINVAL, "bad group / null argument");
  if (int s = flush_rot_clear(e)) return s;
  if (group == 0) HIPC(hipMemsetAsync(e->part_cnt, 0, 4, e->st));
  e->x_group = group;
  e->x_level = 0;
  e->tbegin("bfs", &e->x_t0);
  HIPC(mvx_begin(*e, group, e->x_nlocal));
  *n_local = e->x_nlocal;
  return GS_OK;
}

int gs_part_xbfs_expand(gs_engine* eh, uint32_t level, uint64_t* words_to) {
  PARTX(eh);
  if (e->x_group == 0xFFFFFFFFu || level != e->x_level || !words_to)
    return fail(GS_ESTATE, "gs_part_xbfs_expand: begin the group first and take the levels in order");
  if (level >= 254) return fail(GS_ERANGE, "BFS depth exceeds 254 hops (hop counts are u8)");
  std::vector<uint64_t> w;
  HIPC(mvx_expand(*e, e->x_group, level, e->x_nlocal, w));
  for (uint32_t q = 0; q < e->part_K; ++q) words_to[q] = w[q];
  return check_err(e);
}

int gs_part_xbfs_send(gs_engine* eh, void* dst, int dev) {
  PARTX(eh);
  if (!dst) return fail(GS_EINVAL, "null argument");
  if (e->x_send_words) HIPC(hipMemcpyAsync(dst, e->x_send, e->x_send_words * 8, kind_to(dev), e->st));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_part_xbfs_apply(gs_engine* eh, uint32_t level, const void* src, const uint64_t* words_from, int dev,
                       uint32_t* n_local) {
  PARTX(eh);
  if (e->x_group == 0xFFFFFFFFu || level != e->x_level || !words_from || !n_local)
    return fail(GS_ESTATE, "gs_part_xbfs_apply: after gs_part_xbfs_expand of the same level");
  std::vector<uint64_t> wf(words_from, words_from + e->part_K);
  size_t total = 0;
  for (uint64_t x : wf) total += x;
  const unsigned long long* rec = reinterpret_cast<const unsigned long long*>(src);
  if (!dev && total) {  // host messages: through a pinned host buffer into a grow-only device buffer
    if (total > e->x_recv_cap) {
      HIPC(hipStreamSynchronize(e->st));
      if (e->x_recv) hipFree(e->x_recv);
      if (e->x_pin) hipHostFree(e->x_pin);
      e->x_recv = nullptr;
      e->x_pin = nullptr;
      e->x_recv_cap = 0;
      HIPC(hipMalloc(&e->x_recv, total * 8));
      HIPC(hipHostMalloc(&e->x_pin, total * 8, hipHostMallocDefault));
      e->x_recv_cap = total;

    }
    HIPC(hipStreamSynchronize(e->st));  // (the previous level's copy out of x_pin is done)
    std::memcpy(e->x_pin, src, total * 8);
    HIPC(hipMemcpyAsync(e->x_recv, e->x_pin, total * 8, hipMemcpyHostToDevice, e->st));
    rec = e->x_recv;
  }
  if (!rec) return fail(GS_EINVAL, "null messages");
  HIPC(mvx_apply(*e, e->x_group, level, rec, wf, e->x_nlocal));
  e->x_level = level + 1;
  *n_local = e->x_nlocal;
  return check_err(e);
}

int gs_part_xbfs_end(gs_engine* eh, int record) {
  PARTX(eh);
  if (e->x_group == 0xFFFFFFFFu) return fail(GS_ESTATE, "gs_part_xbfs_end: no group begun");
  e->tend("bfs", e->x_t0);
  if (!e->mv_fused)
    if (int s = ensure_inb(e)) return s;  // the gather's inbound rows (allocated on first use)
  hipEvent_t t0;
  e->tbegin("gather_consume", &t0);
  HIPC(mvx_gather_consume(*e, e->x_group, record != 0));
  e->tend("gather_consume", t0);
  e->x_group = 0xFFFFFFFFu;
  e->inb_valid = false;
  return check_err(e);
}

// The asynchronous level loop (fixed-capacity message slots; RCCL all-to-all on the engine's
// stream): nothing below waits on the host until gs_part_xbfs_async_status.
static uint32_t mvx_max_bins(const Engine& e) {
  uint32_t m = 0;
  for (uint32_t q = 0; q < e.part_K; ++q) {
    const size_t lo = std::min<size_t>(e.N, (size_t)q * e.part_C), hi = std::min<size_t>(e.N, lo + e.part_C);
    const uint32_t f = (uint32_t)(lo >> e.mv.BSC);
    const uint32_t nb = hi <= lo ? 0u : (uint32_t)(((hi + (1u << e.mv.BSC) - 1) >> e.mv.BSC) - f);
    m = std::max(m, nb);
  }
  return m;
}

int gs_part_xbfs_expand_async(gs_engine* eh, uint32_t level, uint64_t cap_words, void* send) {
  PARTX(eh);
  if (e->x_group == 0xFFFFFFFFu || level != e->x_level || !send)
    return fail(GS_ESTATE, "gs_part_xbfs_expand_async: begin the group first and take the levels in order");
  if (level >= 254) return fail(GS_ERANGE, "BFS depth exceeds 254 hops (hop counts are u8)");
  if (cap_words < mvx_max_bins(*e) || cap_words > 0xFFFFFFF0ull / e->part_K)
    return fail(GS_EINVAL, "gs_part_xbfs_expand_async: a slot must hold every rank's bin headers (and K slots < 2^32 words)");
  if (!e->x_bins_set) {
    HIPC(mvx_upload_bins(*e));
    e->x_bins_set = true;
  }
  HIPC(mvx_expand_async(*e, e->x_group, level, cap_words, reinterpret_cast<unsigned long long*>(send)));
  return GS_OK;
}

int gs_part_xbfs_apply_async(gs_engine* eh, uint32_t level, const void* recv, uint64_t cap_words) {
  PARTX(eh);
  if (e->x_group == 0xFFFFFFFFu || level != e->x_level || !recv)
    return fail(GS_ESTATE, "gs_part_xbfs_apply_async: after gs_part_xbfs_expand_async of the same level");
  HIPC(mvx_apply_async(*e, e->x_group, level, reinterpret_cast<const unsigned long long*>(recv), cap_words));
  e->x_level = level + 1;
  return GS_OK;
}

int gs_part_xbfs_async_status(gs_engine* eh, uint32_t* n_local, uint32_t* overflow, uint64_t* words_log,
                              size_t log_levels) {
  PARTX(eh);
  if (!n_local || !overflow) return fail(GS_EINVAL, "null argument");
  if (e->x_group == 0xFFFFFFFFu) return fail(GS_ESTATE, "gs_part_xbfs_async_status: no group begun");
  HIPC(hipMemcpyAsync(e->h_err + 1, e->lvl + e->x_level, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipMemcpyAsync(e->h_err, e->err, 4, hipMemcpyDeviceToHost, e->st));
  const size_t nl = std::min<size_t>(log_levels, e->x_level);
  if (words_log && nl)
    HIPC(hipMemcpyAsync(words_log, e->x_wlog, nl * e->part_K * 8, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  *overflow = (e->h_err[0] & ERR_MVX_CAP) ? 1u : 0u;
  if (*overflow) {  // (reported once: the caller redoes the group)
    e->h_err[0] &= ~ERR_MVX_CAP;
    HIPC(hipMemcpyAsync(e->err, e->h_err, 4, hipMemcpyHostToDevice, e->st));
    HIPC(hipStreamSynchronize(e->st));
  }
  e->x_nlocal = e->h_err[1];
  *n_local = e->x_nlocal;
  return check_err(e);
}

int gs_stream(gs_engine* eh, void** stream) {
  ENGINE(eh);
  if (!stream) return fail(GS_EINVAL, "null argument");
  *stream = (void*)e->st;
  return GS_OK;
}

int gs_part_xround_finish(gs_engine* eh, uint32_t round, int record, uint32_t* n_records) {
  PARTX(eh);
  if (!n_records) return fail(GS_EINVAL, "null argument");
  if (round >= (1u << 27)) return fail(GS_ERANGE, "round index must be < 2^27");
  const bool rec = record != 0;
  hipEvent_t t0;
  e->tbegin("consume", &t0);
  hipError_t r = hipMemsetAsync(e->slot_prunes, 0, e->S * 4, e->st);
  // consume_messages of every group's gathered rows (unless fused into xbfs_end), then
  // send_prunes of own pruners
  if (r == hipSuccess) r = launch_consume_prune_g(*e, rec, !e->mv_fused);
  if (r == hipSuccess) r = launch_part_emit(*e);                   // ... as records for the other ranks
  e->tend("consume", t0);
  HIPC(r);
  HIPC(hipMemcpyAsync(e->h_err + 1, e->part_cnt, 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  if (int s = check_err(e)) return s;
  e->part_nrec = e->h_err[1];
  *n_records = e->part_nrec;
  return GS_OK;
}

int gs_part_exchange_sizes(gs_engine* eh, size_t* record_cap, size_t* dense_words) {
  PART(eh);
  if (record_cap) *record_cap = e->part_rec_cap;
  if (dense_words) *dense_words = (size_t)e->S * e->N;
  return GS_OK;
}

int gs_part_prunes_out(gs_engine* eh, void* dst, int dev) {
  PART(eh);
  if (e->part_nrec > e->part_rec_cap)
    return fail(GS_ERANGE, "this round's prune records exceed the record buffer: exchange them dense "
                           "(gs_part_prunes_dense_out / _in)");
  if (e->part_nrec) HIPC(hipMemcpyAsync(dst, e->part_rec, (size_t)e->part_nrec * 8, kind_to(dev), e->st));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_part_prunes_in(gs_engine* eh, const void* src, size_t n, int dev) {
  PART(eh);
  if (n == 0) return GS_OK;
  const uint2* rec = reinterpret_cast<const uint2*>(src);
  if (!dev) {  // host records: staged in a grow-only device buffer
    if (n > e->part_in_cap) {
      if (e->part_in) hipFree(e->part_in);
      e->part_in = nullptr;
      e->part_in_cap = 0;
      HIPC(hipMalloc(&e->part_in, n * 8));
      e->part_in_cap = n;
    }
    HIPC(hipMemcpyAsync(e->part_in, src, n * 8, hipMemcpyHostToDevice, e->st));
    rec = e->part_in;
  }
  HIPC(launch_part_prunes_apply(*e, rec, n));
  HIPC(hipStreamSynchronize(e->st));
  return check_err(e);
}

int gs_part_prunes_dense_out(gs_engine* eh, void* dst, int dev) {
  PART(eh);
  if (!dst) return fail(GS_EINVAL, "null argument");
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  if (!dev) {  // host buffer: staged in a device buffer of the same size
    if (!e->part_dense) {
      const int s = dalloc(*e, &e->part_dense, (size_t)e->S * e->N, 0);
      if (s) return s;
    }
    d = e->part_dense;
  }
  HIPC(launch_part_emit_dense(*e, d));
  if (!dev) HIPC(hipMemcpyAsync(dst, d, (size_t)e->S * e->N * 4, hipMemcpyDeviceToHost, e->st));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_part_prunes_dense_in(gs_engine* eh, const void* src, int dev) {
  PART(eh);
  if (!src) return fail(GS_EINVAL, "null argument");
  const uint32_t* d = reinterpret_cast<const uint32_t*>(src);
  if (!dev) {
    if (!e->part_dense) {
      const int s = dalloc(*e, &e->part_dense, (size_t)e->S * e->N, 0);
      if (s) return s;
    }
    HIPC(hipMemcpyAsync(e->part_dense, src, (size_t)e->S * e->N * 4, hipMemcpyHostToDevice, e->st));
    d = e->part_dense;
  }
  HIPC(launch_part_dense_apply(*e, d));
  HIPC(hipStreamSynchronize(e->st));
  return check_err(e);
}

int gs_part_stats_out(gs_engine* eh, void* dst, int dev) {
  PART(eh);
  HIPC(launch_stats(*e, e->sum_used, 5));  // this rank's nodes: partials (and its egress accumulators)
  HIPC(launch_part_stats_pack(*e));
  HIPC(hipMemcpyAsync(dst, e->part_stats, part_stats_words(*e) * 8, kind_to(dev), e->st));
  HIPC(hipStreamSynchronize(e->st));
  return GS_OK;
}

int gs_part_stats_in(gs_engine* eh, const void* src, int dev) {
  PART(eh);
  HIPC(hipMemcpyAsync(e->part_stats, src, part_stats_words(*e) * 8, kind_from(dev), e->st));
  HIPC(launch_part_stats_unpack(*e));
  HIPC(launch_stats(*e, e->sum_used, 2));  // summary of the summed partials
  if (++e->sum_used == e->sum_cap) return drain_summaries(e);
  return GS_OK;
}

}  // extern "C"
