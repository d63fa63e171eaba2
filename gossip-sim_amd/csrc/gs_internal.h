// gs_internal.h -- engine state shared by the kernels' launchers and the C ABI.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <map>
#include <string>
#include <vector>

#include "../../include/gossip_hip.h"

namespace gs {

// Device-resident state. Layout (DESIGN.md "Data layout in HBM"):
//  per node      stake u64, bucket u8, fail rank u32, stake rank u32
//  per (node,k)  peers[ASZP] u32 ring + hl u16 (head | len << 8)      -- PushActiveSet
//  per k         prefix sums of rotation weights P[k][N+1] u64
//  per pair      (slot-major pair p = slot * NP + (node - vlo): NP = N, vlo = 0, except
//                on a node-range partition rank, which keeps its own nodes [vlo, vlo + NP))
//                hops u8, in-degree u32, prune mask u32 (bits = physical ring slots),
//                inbound records u32 [capin][pairs] (hop << 24 | src),
//                cache meta u32 (len | upserts << 8 | pruned-len << 16),
//                cache keys u32 [96][pairs], scores u8 [96][pairs] (bit 7 = pruned),
//                egress/prune-sent of the round u8, measured accumulators u32
// Geometry of the propagation-blocked BFS (gs_bfs_binned.hip): bins of 2^BS pairs,
// expand workgroups of PW frontier pairs (at most Gmax of them).
struct BinGeom {
  uint32_t BS = 0, nbins = 0, PW = 0, Gmax = 0, csr_cap = 0;
  size_t T_words = 0;
  bool narrow = false;  // 4-byte records (bins of 2^11 pairs, N <= 2^21)
};

// Geometry of the multi-source frontier BFS (gs_bfs_multi.hip): bins of 2^BS nodes,
// level records u64 = src | node-in-coarse-bin << UB | slot mask << (UB + BSC); pool records
// src | node-in-fine-bin << UB | hop << (UB + BSF) | slot mask << (UB + BSF + 8); slot groups of <= GW.
constexpr uint32_t GT_WORDS = 96;  // per-group table words (the part the level kernels copy to LDS)
// ... followed by the group's origin -> slot-mask hash (128 (id, mask) pairs, two probes;
// word GT_OTOK of the table = 1 when every origin is in it): a group's table is GT_STRIDE words
constexpr uint32_t GT_OT = GT_WORDS, GT_OTOK = 94, GT_STRIDE = GT_WORDS + 256;
struct MvGeom {
  uint32_t UB = 0, BSC = 0, BSF = 0, nbc = 0, nbf = 0, GW = 0, TW = 0, gcap = 0, gcap_c = 0;
  uint32_t XT = 256;  // frontier entries per expand slice (256, or 1,024 for wide T rows)
  size_t q_cap = 0, area_cap = 0, rows_cap = 0, pcap = 0;
};
struct MvGroup { uint32_t s0, sg, seed0, nseed; };

struct Engine {
  gs_params prm{};
  uint32_t N = 0, S = 0;
  uint32_t NP = 0, vlo = 0;  // nodes with per-pair state: [vlo, vlo + NP) (all N but on a partition rank)
  size_t PAIRS = 0;          // S * NP
  uint32_t ASZ = 0, ASZP = 0, fanout = 0, capin = 64;
  uint32_t bfs_mode = GS_BFS_LEVEL;
  uint32_t fcap = 0;             // min(fanout, active_set_size): pushes per node
  // (slot o, node u) strides of the prune masks and the round's egress bytes: slot-major
  // (N, 1), or node-major (1, SP) for the multi-source BFS, whose expansion reads every
  // slot's mask of a node at once (SP = slots rounded up to 4)
  size_t mso = 0, msu = 1, eso = 0, esu = 1, mask_words = 0;
  uint32_t SP = 0;
  bool fused = false;            // gs_round runs the one-kernel workgroup round
  bool inb_valid = true;         // inbound records materialized in HBM (step-wise BFS)
  hipStream_t st = nullptr;
  size_t dev_bytes = 0;
  size_t pair_bytes = 0;  // of which per-(slot, node) state (gs_engine_memory)
  std::vector<void*> allocs;

  // node arrays
  uint64_t* stake = nullptr;
  uint8_t* bucket = nullptr;
  uint64_t* P = nullptr;
  uint32_t* IX = nullptr;        // [25][ix_count(N)] index tables of the prefix sums (prefix_search_ix)
  uint32_t* peers = nullptr;
  uint16_t* hl = nullptr;
  uint32_t* frank = nullptr;
  uint32_t* srank = nullptr;
  uint32_t* by_srank = nullptr;
  uint32_t* prank = nullptr;     // rank by (stake desc, id asc): prune-order key
  uint32_t* by_prank = nullptr;
  uint64_t* pstake = nullptr;    // stake by prune rank
  uint4* pinfo = nullptr;        // by node id: {prune rank, 0, stake lo, stake hi} (one load per cache key)
  uint4* rinfo = nullptr;        // by prune rank: {node id, 0, stake lo, stake hi} (the round kernel's sorted entries)
  // slot arrays
  uint32_t* origin = nullptr;
  uint8_t* obkt = nullptr;
  uint32_t* min_ingress = nullptr;
  double* thr = nullptr;
  uint32_t* nfail = nullptr;
  uint32_t* slot_prunes = nullptr;  // prunees emitted in the current round
  // pair arrays
  uint8_t* hops = nullptr;
  uint32_t* cnt = nullptr;
  uint32_t* mask = nullptr;
  uint32_t* inb = nullptr;
  uint32_t* cmeta = nullptr;
  uint32_t* ckey = nullptr;  // received cache [CACHE_CAP][PAIRS] slot words: id | score << 24 | pruned << 31
  uint8_t* egress = nullptr;
  uint8_t* prune_round = nullptr;
  uint32_t* egress_acc = nullptr;
  uint32_t* ingress_acc = nullptr;
  uint32_t* prune_acc = nullptr;
  uint32_t* strand = nullptr;
  // level-synchronous BFS
  uint32_t* q[2] = {nullptr, nullptr};
  uint32_t* lvl = nullptr;  // frontier sizes per level [256]
  // propagation-blocked BFS (GS_BFS_BINNED, gs_bfs_binned.hip)
  BinGeom bin{};
  uint32_t* own = nullptr;      // [N][ORW] own-bucket entry rows (word ASZP = hl | bucket << 16; multi: + fcls)
  uint32_t ORW = 0;
  uint2* bin_area = nullptr;    // expand -> apply records (pair, src), per level, PAIRS * fcap
  uint32_t* bin_T = nullptr;    // [Gmax][nbins + 1] bin starts of each expand workgroup's run
  uint2* bin_pool = nullptr;    // apply -> gather records: one region of 2^BS * capin records per bin
  uint2* bin_Lt = nullptr;      // [256][nbins] (pool start, count) per level and bin
  uint32_t* bin_binoff = nullptr;  // [nbins] records used in each bin's pool region this round
  uint32_t* bin_vis = nullptr;  // [PAIRS / 32] visited bitmap of the round
  // multi-source frontier BFS (GS_BFS_MULTI, gs_bfs_multi.hip)
  MvGeom mv{};
  uint32_t* mv_vis = nullptr;     // [N] slot masks reached this round (current group)
  uint2* mv_q[2] = {nullptr, nullptr};  // frontier entries (node | entry << 24, slot mask) [q_cap]
  uint32_t* mv_T = nullptr;       // [rows_cap][TW] per expand workgroup of a level: run base, bin starts, total
  unsigned long long* mv_area = nullptr;  // [area_cap] records of a level
  uint32_t* mv_ctr = nullptr;     // [4] records used
  unsigned long long* mv_pool = nullptr;  // [nbf][pcap] records of the round per fine bin
  uint32_t* mv_pused = nullptr;   // [nbf]
  uint8_t* mv_fcls = nullptr;     // [N] failure class per node
  uint8_t* mv_fk = nullptr;       // [S] failure class index per slot
  uint32_t* mv_thr = nullptr;     // [S] distinct failure counts (scratch)
  uint32_t* mv_hlvl = nullptr;    // host-mapped [256] frontier sizes (host pointer)
  uint32_t* mv_hlvl_dev = nullptr;  // its device pointer
  uint32_t* mv_hstate_dev = nullptr;  // device pointer of mv_hlvl + 256 (small-level kernel's state)
  uint32_t* mv_dpair = nullptr;   // [258] level of each expand/apply pair of the predicted loop
  uint32_t* mv_prof = nullptr;    // host-mapped [groups][MV_PROF_WORDS]: the tail kernel's level profile
  uint32_t* mv_prof_dev = nullptr;
  std::vector<std::vector<uint32_t>> mv_pred;  // per group: the last known level sizes (empty: none yet)
  std::vector<uint32_t> mv_prof_seen;          // per group: the profile sequence number last read
  uint32_t mv_seq = 0;                         // profile sequence numbers handed to the tail kernels
  uint32_t* mv_gtab = nullptr;    // [groups][GT_STRIDE]
  uint2* mv_seed = nullptr;       // [S] seed entries (distinct origins) of every group
  std::vector<MvGroup> mv_groups;
  bool mv_attr_set = false;
  uint32_t bfs_level = 0;  // the level loop's current level (reported when a level wait times out)
  bool mv_diag = false;  // GS_MV_DIAG=1
  bool mv_line = false;   // multi: prune masks live in the row table's node lines (msu = 32)
  bool mv_vis_clean = true;  // mv_vis is all zero (allocated zeroed; a clearing gather ran last)
  bool mv_fused = false;  // gs_round: gather, then k_cg_consume; GS_MV_FUSED=1: fused gather + consume (slower at C4)
  // direction-optimizing BFS over the round's push graph (GS_BFS_HYBRID, gs_bfs_hybrid.hip);
  // it shares the multi BFS's layout, groups, queues, T rows and record area
  uint8_t* hb_dist = nullptr;      // [N][hb_dsp] distance of every slot of the current group
  uint32_t hb_dsp = 16;
  uint2* hb_pgo = nullptr;         // [N] {first, count} of each node's push-graph in-records
  uint32_t* hb_F = nullptr;        // [3][N] slots first reached at level d (buffer d % 3)
  unsigned long long* hb_pgr = nullptr;  // [nbc][hb_bin_cap] in-records src | slot mask << 32
  size_t hb_bin_cap = 0;
  uint32_t hb_parts = 0, hb_slices = 0;  // T rows per slice (entries per node at most), slices
  // persistent multi-source BFS (gs_bfs_pers.hip, round 6): one launch per slot group,
  // G workgroups (one per CU) that own interleaved fine bins; off on partition ranks
  bool pb_on = false, pb_registered = false;
  uint32_t pb_G = 0, pb_GL = 0, pb_FPW = 0, pb_LB = 0, pb_CH = 0, pb_rows_cap = 0, pb_gq_cap = 0;
  size_t pb_lds = 0, pb_attr_lds = 0, pb_area_cap = 0;
  uint32_t* pb_T[2] = {nullptr, nullptr};              // per level parity: [G + 2][rows_cap] T rows
  unsigned long long* pb_area[2] = {nullptr, nullptr}; // per level parity: records [area_cap]
  uint32_t* pb_blk = nullptr;                          // barrier + per-level slice counters
  uint2* pb_gq = nullptr;                              // [G][gq_cap] level entries beyond the LDS list
  std::vector<uint32_t> h_nfail_any;  // host copy: slot has failed nodes
  // rotation
  uint32_t* rot_list = nullptr;
  uint32_t* rot_count = nullptr;    // [2]: rotation r counts into [r & 1] and zeroes [(r + 1) & 1]
  uint32_t* rot_changed = nullptr;  // [N][25] replaced ring slots of the last rotation, per entry
  bool rot_clear_pending = false;   // the last rotation's prune-bit clear is still to be applied
  bool rot_have_prev = false;
  uint32_t rot_parity = 0;          // parity of the last rotation's round
  // Rotation ahead (round 5; fused round, N <= 16,384): rotation r runs in workgroup 0 of
  // the round kernel r, into the OTHER row buffer (peers2 / hl2), while the slots'
  // workgroups read the current one -- the rows change only by rotation, which depends on
  // (seed, node, round) and the rows, not on the round's BFS or prunes -- and the buffers
  // swap after the round. rot_list / rot_changed alternate between two buffers so the
  // round kernel's deferred clear of the previous rotation is not overwritten.
  bool rot_ahead_ok = false;        // enabled at create (its buffers allocated there); stays on: any
                                    // in-place row change (init, a step-wise rotation, an uploaded
                                    // entry) must set rows2_stale (a full copy before the next round)
  bool rows2_stale = true;          // peers2 / hl2 need a full copy of peers / hl
  bool rot_cnt_dirty = false;       // an ahead rotation did not zero the other counter
  int rows2_pending = -1;           // parity of the rotation applied to peers but not peers2
  uint32_t* peers2 = nullptr;
  uint16_t* hl2 = nullptr;
  uint32_t* rot_list_b[2] = {nullptr, nullptr};
  uint32_t* rot_changed_b[2] = {nullptr, nullptr};

  size_t rwg_attr_lds = 0;          // dynamic LDS the round kernel was last configured for
  bool rwg_attr_prof = false;       // ... and for which instantiation (phase clocks or not)
  // node-range partition (gs_partition.hip): this rank owns node ids [part_lo, part_hi)
  // (= [vlo, vlo + NP)) and the fine bins [part_flo, part_flo + part_fno) of the multi BFS
  bool part_on = false;
  uint32_t part_rank = 0, part_K = 1, part_lo = 0, part_hi = 0, part_flo = 0, part_fno = 0;
  uint2* part_rec = nullptr;        // prune records of this rank's round: (slot * N + prunee, ring bits)
  size_t part_rec_cap = 0;          // fixed at create (beyond it the round's exchange is dense)
  uint32_t* part_dense = nullptr;   // [N][S] dense prune words (allocated on the first dense host exchange)
  uint32_t* part_cnt = nullptr;     // [1]: prune records staged
  uint32_t part_nrec = 0;           // records of the last gs_part_round
  uint2* part_in = nullptr;         // every rank's prune records (gs_part_prunes_in), grow-only
  size_t part_in_cap = 0;
  uint64_t* part_stats = nullptr;   // packed stats partials [S][5 + 256 + bm_words]
  // frontier-exchange partition (GS_FLAG_FRONTIER_EXCHANGE): this rank expands its own frontier
  // and exchanges each level's push records with the owners of their destination bins
  bool part_x = false;
  uint32_t part_C = 0;                  // nodes per rank (whole coarse bins)
  unsigned long long* x_send = nullptr;  // packed messages of the level [x_send_cap] u64
  size_t x_send_cap = 0, x_send_words = 0;
  unsigned long long* x_recv = nullptr;  // host-exchanged messages staged on the device (grow-only)
  unsigned long long* x_pin = nullptr;   // pinned host staging of host-exchanged messages
  size_t x_recv_cap = 0;
  uint32_t* x_T = nullptr;              // [K][TW] T rows of the received level
  uint32_t* x_bincnt = nullptr;         // [nbc]
  unsigned long long* x_pos = nullptr;  // [2][nbc] header / record places in x_send
  unsigned long long* x_off = nullptr;  // [K + 1]
  uint32_t* x_bins = nullptr;           // [2K] every rank's first coarse bin and bin count (async loop)
  bool x_bins_set = false;
  unsigned long long* x_wlog = nullptr; // [256][K] words of each level's message to each rank (async loop)
  uint32_t x_group = 0xFFFFFFFFu, x_level = 0;
  uint32_t x_nlocal = 0;
  hipEvent_t x_t0 = nullptr;           // (timing of the group's levels)
  // stats
  uint32_t* rs_u32 = nullptr;   // per slot: visited, pushes, stranded, pad
  uint64_t* rs_ssum = nullptr;  // per slot: stranded stake sum
  uint32_t* rs_hist = nullptr;  // per slot: 256 hop bins of this round
  uint64_t* hist_acc = nullptr; // per slot: 256 hop bins over recorded rounds
  uint32_t* bm = nullptr;       // per slot: stranded bitmap over stake rank
  uint32_t bm_words = 0;
  uint32_t* bm_cnt = nullptr;       // [S][64] set bits per 1/64 of each slot's stranded bitmap
  gs_round_summary* sum = nullptr;  // device ring of recorded summaries [sum_cap][S]
  uint32_t sum_cap = 0, sum_used = 0;
  std::vector<gs_round_summary> h_sum;  // drained summaries
  uint32_t* err = nullptr;
  uint32_t* h_err = nullptr;  // pinned
  unsigned long long* phase_clk = nullptr;  // GS_PHASE_PROFILE=1: per-phase workgroup clock sums

  std::vector<gs_slot> slots;
  bool slots_set = false, failed_ranked = false;
  bool broken = false;  // a grid barrier of the persistent BFS timed out (ERR_SYNC): the engine refuses every call

  // profiling
  struct Timed { std::vector<std::pair<hipEvent_t, hipEvent_t>> ev; double ms = 0; uint64_t n = 0; };
  std::map<std::string, Timed> timers;
  std::string prof_only;  // ",fam1,fam2,": time only these families (GS_PROFILE_ONLY at create); empty: all
  std::vector<hipEvent_t> ev_pool;  // recycled events: no hipEventCreate per launch
  hipEvent_t ev_take();
  void tbegin(const char* fam, hipEvent_t* a);
  void tend(const char* fam, hipEvent_t a);
};

// (the same in a function returning void; unsupported sizes are refused at create)
#define GS_ASZP_DISPATCH_V(ASZP_VAL, CALL)        \
  switch (ASZP_VAL) {                             \
    case 4: { constexpr int A = 4; CALL; } break; \
    case 8: { constexpr int A = 8; CALL; } break; \
    case 12: { constexpr int A = 12; CALL; } break; \
    case 16: { constexpr int A = 16; CALL; } break; \
    case 20: { constexpr int A = 20; CALL; } break; \
    case 24: { constexpr int A = 24; CALL; } break; \
    case 28: { constexpr int A = 28; CALL; } break; \
    case 32: { constexpr int A = 32; CALL; } break; \
    default: break;                               \
  }
#define GS_ASZP_DISPATCH(ASZP_VAL, CALL)          \
  switch (ASZP_VAL) {                             \
    case 4: { constexpr int A = 4; CALL; } break; \
    case 8: { constexpr int A = 8; CALL; } break; \
    case 12: { constexpr int A = 12; CALL; } break; \
    case 16: { constexpr int A = 16; CALL; } break; \
    case 20: { constexpr int A = 20; CALL; } break; \
    case 24: { constexpr int A = 24; CALL; } break; \
    case 28: { constexpr int A = 28; CALL; } break; \
    case 32: { constexpr int A = 32; CALL; } break; \
    default: return hipErrorInvalidValue;         \
  }

// launchers (gs_kernels.hip, gs_round_wg.hip); all enqueue on e.st and return hipError_t
hipError_t launch_prefix_weights(Engine& e);
hipError_t launch_init_entries(Engine& e);
hipError_t launch_fail_keys(Engine& e, uint64_t* keys, uint32_t* ids);
hipError_t launch_scatter_rank(Engine& e, const uint32_t* sorted_ids, uint32_t* rank_out);
hipError_t launch_clear_slot_masks(Engine& e, uint32_t node, uint32_t bucket, uint32_t bits);
hipError_t launch_bfs(Engine& e, bool record);
hipError_t launch_bfs_binned(Engine& e, bool record);
// spin on a host-mapped word the device writes (MV_PENDING until then); checks the stream
// now and then so a stream that ended without writing it fails instead of hanging
constexpr uint32_t MV_PENDING = 0xFFFFFFFFu;
constexpr uint32_t MV_PROF_WORDS = 258;  // seq, levels, sizes of levels 0..255
// Extra expand/apply pairs the predicted level loops enqueue beyond the profile's levels
// (no-ops when the BFS ends as predicted; they take a level the profile did not expect
// instead of the one-workgroup tail kernel). GS_MV_MARGIN, default 1.
inline uint32_t mv_margin() {
  static const uint32_t m = [] {
    const char* x = std::getenv("GS_MV_MARGIN");
    return x ? (uint32_t)std::strtoul(x, nullptr, 10) : 1u;
  }();
  return m;
}
hipError_t mv_wait(volatile uint32_t* p, hipStream_t st, uint32_t& out);  // bounded: hipErrorLaunchTimeOut
// after the level loop enqueued levels through d - 1: is level d's frontier empty (syncs the stream)
hipError_t level_empty(Engine& e, uint32_t d, bool& empty);
hipError_t launch_bfs_level_step(Engine& e, bool record, uint32_t d, uint32_t qmin, uint32_t qmax);
void bin_geometry(uint32_t N, size_t PAIRS, uint32_t fcap, BinGeom& g, bool allow_narrow);
bool bin_supported(const BinGeom& g, uint32_t fcap);
void mv_geometry(uint32_t N, uint32_t S, uint32_t ASZ, uint32_t ASZP, MvGeom& g);
bool mv_supported(const MvGeom& g, uint32_t ASZP);
uint32_t mv_kept_bins(const Engine& e);
void mv_build_groups(Engine& e, const std::vector<uint32_t>& origins, const std::vector<uint8_t>& obkt,
                     const std::vector<uint8_t>& bucket, std::vector<uint32_t>& gtab, std::vector<uint2>& seeds);
// consume: gs_round's fused gather + consume (k_mv_consume) instead of the materializing
// gather; then only k_cg_prune remains (launch_consume_prune_g(e, record, false)).
hipError_t launch_bfs_multi(Engine& e, bool record, bool consume = false);
// GS_BFS_HYBRID: push graph, top-down / bottom-up levels, gather (gs_bfs_hybrid.hip)
hipError_t launch_bfs_hybrid(Engine& e, bool record);
void hb_geometry(Engine& e, uint32_t parts);  // area / T rows / in-record regions for `parts` entries per node
// the multi-source BFS's layout (node-major masks and egress, slot groups): MULTI and HYBRID
inline bool mv_layout(const Engine& e) { return e.bfs_mode == GS_BFS_MULTI || e.bfs_mode == GS_BFS_HYBRID; }
hipError_t mv_update_failures(Engine& e, const std::vector<uint32_t>& nf);
// persistent multi-source BFS (gs_bfs_pers.hip): geometry at create (false: not usable),
// the process-wide count of engines that may launch it, and whether it runs now
bool pb_setup(Engine& e);
void pb_register(Engine& e, bool on);
bool pb_usable(const Engine& e);
size_t pb_blk_words();
// frontier-exchange partition levels (gs_bfs_multi.hip): seed, expand + pack, apply, gather
hipError_t mvx_begin(Engine& e, uint32_t g, uint32_t& n_local);
hipError_t mvx_expand(Engine& e, uint32_t g, uint32_t d, uint32_t n_local, std::vector<uint64_t>& words_to);
hipError_t mvx_apply(Engine& e, uint32_t g, uint32_t d, const unsigned long long* recv,
                     const std::vector<uint64_t>& words_from, uint32_t& n_next);
hipError_t mvx_gather_consume(Engine& e, uint32_t g, bool record);
// the asynchronous level loop (fixed-capacity message slots, no host wait per level)
hipError_t mvx_expand_async(Engine& e, uint32_t g, uint32_t d, unsigned long long cap, unsigned long long* send);
hipError_t mvx_apply_async(Engine& e, uint32_t g, uint32_t d, const unsigned long long* recv, unsigned long long cap);
hipError_t mvx_upload_bins(Engine& e);
// own-bucket entry rows: all nodes (list == nullptr), or the `*count` nodes of `list`
hipError_t launch_own_rows(Engine& e, const uint32_t* list, const uint32_t* count);
// the rotation that runs inside the fused round kernel (its workgroup 0) on the other row buffer
struct RotAhead {
  uint32_t* peers2;
  uint16_t* hl2;
  uint32_t* list;            // this rotation's rotating nodes ...
  uint32_t* count;           // ... their number ...
  uint32_t* changed;         // ... and each rotated entry's replaced ring slots
  const uint32_t* plist;     // the previous ahead rotation's nodes (to copy first; null: none)
  const uint32_t* pcount;
  uint32_t round;
};
hipError_t launch_consume_prune(Engine& e, bool consume, bool prune, bool apply, bool record);
hipError_t launch_consume_prune_g(Engine& e, bool record, bool consume = true, bool zero_slot_prunes = false);
// node-range partition (gs_partition.hip)
size_t part_stats_words(const Engine& e);
hipError_t launch_part_stats_pack(Engine& e);
hipError_t launch_part_stats_unpack(Engine& e);
hipError_t launch_part_prunes_apply(Engine& e, const uint2* rec, size_t n);
hipError_t launch_part_emit(Engine& e);  // this round's prune records -> part_rec (count in part_cnt)
hipError_t launch_part_emit_dense(Engine& e, uint32_t* dense);         // ... as dense words [N][S] (zeroed first)
hipError_t launch_part_dense_apply(Engine& e, const uint32_t* dense);  // masks |= the summed dense words
// Rotation of round `round` (decide + entries); the prune-bit clear of the replaced
// ring slots runs now, or with defer_clear it is left pending for the next one-kernel
// round (which applies it to its LDS copy of the masks) or launch_rotate_clear.
hipError_t launch_rotate(Engine& e, uint32_t round, bool defer_clear);
hipError_t launch_rotate_clear(Engine& e);
hipError_t launch_stats(Engine& e, uint32_t rec_index, int mode);
hipError_t launch_round_wg(Engine& e, bool record, uint32_t rec_index, bool rot_clear, const RotAhead* ra = nullptr);
size_t round_wg_lds_bytes(uint32_t N, uint32_t fcap, uint32_t ASZP);
size_t bfs_wg_lds_bytes(uint32_t N);
hipError_t launch_gather_strided_u32(Engine& e, const uint32_t* src, size_t stride, uint32_t n, uint32_t* dst);

}  // namespace gs
