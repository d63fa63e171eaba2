/*
 * gossip_hip.h -- C ABI of the MI355X push-propagation engine for gossip-sim.
 *
 * Drop-in boundary for the per-iteration hot path of gregcusack/gossip-sim
 * (src/gossip_main.rs:449-514). The reference has no FFI seam of its own; every
 * entry point below names the reference method it replaces. A Rust maintainer
 * binds these with `extern "C"` declarations; the C++
 * `gossip-sim` driver and the pytest/ctypes parity tests call them directly.
 *
 * Conventions
 *  - Every int-returning call returns GS_OK (0) or a negative gs_status; the
 *    message of the last failure on this thread is gs_last_error(). Nothing
 *    throws across the ABI.
 *  - Nodes are addressed by id = rank of the node's base58 pubkey string
 *    (so the reference's consume tie-break, gossip.rs:639-645, is id order).
 *    stakes[] is indexed by id.
 *  - One engine = one HIP device + one stream + one shared active-set
 *    trajectory, carrying n_slots independent simulations ("slots"). A slot is
 *    one reference Cluster run: its own origin, prune/cache overlay, failed set
 *    and statistics. Sims that share seed/fanout/active-set-size/rotation
 *    probability (an origin-rank, min-ingress, prune-threshold or fail-nodes
 *    sweep, or "all origins") batch into one engine.
 *  - The engine owns all device memory. Inputs are copied at call time; outputs
 *    go to caller buffers with explicit capacities (too small => GS_ERANGE).
 *  - An engine is not re-entrant; use one engine per device per host thread.
 *  - Randomness follows the Philox determinism contract: results
 *    are a pure function of (stakes, params, slots, call sequence).
 */
#ifndef GOSSIP_HIP_H
#define GOSSIP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum gs_status {
  GS_OK = 0,
  GS_EINVAL = -1,  /* bad argument */
  GS_EHIP = -2,    /* HIP runtime failure (no device, launch error, ...) */
  GS_ENOMEM = -3,  /* device or host allocation failed */
  GS_ERANGE = -4,  /* a capacity or limit was exceeded (see gs_last_error) */
  GS_ESTATE = -5   /* call out of order */
} gs_status;

enum { GS_NUM_BUCKETS = 25, GS_MAX_ACTIVE_SET_SIZE = 32, GS_MAX_NODES = (1 << 24) - 1, GS_HOP_UNREACHED = 0xFF };
/* BFS strategies (results are identical): WORKGROUP = one workgroup per slot with
 * LDS state (small clusters, many slots); LEVEL = level-synchronous over all
 * slots with a global atomic per push; BINNED = level-synchronous,
 * propagation-blocked (pushes binned by destination range, LDS counters per
 * bin); MULTI = batched multi-source frontier BFS (a frontier entry is a node and
 * the mask of slots reaching it at that level: one row expansion and one record
 * per pushed-to peer serve every such slot; large clusters). AUTO picks
 * WORKGROUP (n <= 8,192 and >= 64 slots), else MULTI (when its bin geometry fits LDS
 * and its level area stays below 2^32 records), else BINNED, else LEVEL.
 * HYBRID = direction-optimizing multi-source BFS over the round's push graph: every node's
 * pushes for every slot built once per round as in-records grouped by destination, then
 * levels carrying only slot masks and distances -- top-down (frontier entries, atomicOr on
 * visited masks) for small frontiers, bottom-up (nodes still missing slots scan their
 * in-records for pushers at the current distance) for large ones -- and one gather. */
enum { GS_BFS_AUTO = 0, GS_BFS_WORKGROUP = 1, GS_BFS_LEVEL = 2, GS_BFS_BINNED = 3, GS_BFS_MULTI = 4,
       GS_BFS_HYBRID = 5 };
enum { GS_FLAG_PROFILE = 1, GS_FLAG_SPLIT_ROUND = 2, GS_FLAG_NARROW_WAVE_PATH = 4, GS_FLAG_BINNED_ALL_LEVELS = 8,
       GS_FLAG_WIDE_RECORDS = 16, GS_FLAG_NO_SMALL_LEVELS = 32, GS_FLAG_MISPREDICT_LEVELS = 64,
       GS_FLAG_FRONTIER_EXCHANGE = 128 };

typedef struct gs_params {
  uint32_t push_fanout;         /* Config::gossip_push_fanout (gossip.rs:113) */
  uint32_t active_set_size;     /* Config::gossip_active_set_size, 1..32 */
  double rotation_probability;  /* Config::probability_of_rotation, [0,1] */
  uint64_t seed;                /* Philox key of the INIT/ROTATE/DECIDE/FAIL streams */
  int32_t device;               /* HIP device ordinal */
  uint32_t bfs_mode;            /* GS_BFS_* (results are identical in every mode) */
  uint32_t inbound_capacity;    /* per-(slot,node) inbound records per round; 0 = 64 */
  uint32_t flags;               /* GS_FLAG_PROFILE: time kernels with hipEvents; GS_FLAG_SPLIT_ROUND:
                                   gs_round launches the step kernels instead of the one-kernel
                                   workgroup round (same results; for A/B measurement);
                                   GS_FLAG_NARROW_WAVE_PATH: the one-kernel round sends in-degrees
                                   > 24 (not > 64) to its ordered single-lane consume, and the
                                   step-kernel round uses register paths for in-degree / entries
                                   <= 4 (not 16) and the wave consume for in-degree <= 8 (not 64)
                                   and the binned gather places records directly beyond 256
                                   per bin (same results; lets small test clusters cover every path);
                                   GS_FLAG_BINNED_ALL_LEVELS: GS_BFS_BINNED bins every level, not
                                   only levels with >= 2^17 frontier pairs (same results);
                                   GS_FLAG_WIDE_RECORDS: GS_BFS_BINNED keeps 8-byte push records
                                   even where 4-byte ones fit (same results);
                                   GS_FLAG_NO_SMALL_LEVELS: GS_BFS_BINNED / GS_BFS_MULTI run no level
                                   in their single-workgroup small-level kernels (every level
                                   through the grid-wide kernels; same results);
                                   GS_FLAG_MISPREDICT_LEVELS: GS_BFS_BINNED's predicted level loop
                                   inverts its binned/direct choice per level every other round
                                   (same results; a test of the misprediction path);
                                   GS_FLAG_FRONTIER_EXCHANGE: gs_create_part makes a frontier-exchange
                                   rank (gs_part_xbfs_*: it expands only its own frontier and
                                   exchanges each level's push records with their owners) */
} gs_params;

typedef struct gs_slot {
  uint32_t origin;               /* node id of the CRDS value owner (gossip_main.rs:360) */
  uint32_t min_ingress_nodes;    /* Config::min_ingress_nodes */
  double prune_stake_threshold;  /* Config::prune_stake_threshold */
} gs_slot;

/* Per slot, per recorded round: every integer the reference's per-round
 * statistics are built from (gossip_main.rs:480-563). f64 summaries are
 * computed on the host in the reference's order (gs_stats_*). */
typedef struct gs_round_summary {
  uint32_t visited;      /* n of RelativeMessageRedundancy: nodes reached incl. origin */
  uint32_t pushes;       /* pushes to non-failed peers (the m increments of gossip.rs:571) */
  uint32_t prunes;       /* prunees emitted by send_prunes (gossip.rs:684-687) */
  uint32_t stranded;     /* unreached, non-failed nodes (gossip.rs:329-345) */
  uint64_t hop_sum;      /* sum of hops over reached non-origin nodes */
  uint32_t hop_count;    /* number of reached non-origin nodes */
  uint32_t hop_min, hop_max, hop_med_lo, hop_med_hi; /* order statistics of those hops */
  uint32_t pad0;
  uint64_t stranded_stake_sum;
  uint64_t stranded_stake_min, stranded_stake_max, stranded_med_lo, stranded_med_hi;
} gs_round_summary;

typedef struct gs_engine gs_engine;

/* --- lifetime --------------------------------------------------------- */
int gs_create(const gs_params* params, const uint64_t* stakes, uint32_t n_nodes, uint32_t n_slots,
              gs_engine** out);
void gs_destroy(gs_engine* e);
const char* gs_last_error(void);
/* sha256 prefix (16 hex digits) of the device sources this library was built from; the
 * profiles under profiles/ are stamped with it (not a reference interface: measurement) */
const char* gs_kernel_hash(void);
int gs_device_count(int* n); /* HIP devices visible to this process (0 without a GPU) */
int gs_set_slots(gs_engine* e, const gs_slot* slots, uint32_t n_slots);
int gs_sync(gs_engine* e); /* waits for the stream and reports deferred device-side errors */

/* --- active sets: push_active_set.rs -------------------------------------- */
/* Node::initialize_gossip for every node (gossip.rs:805-813, gossip_main.rs:263-277). */
int gs_init_active_sets(gs_engine* e);
/* Overwrite / read one PushActiveSetEntry (push_active_set.rs:30) in FIFO order.
 * Setting an entry clears the prune state of its slots for every origin. */
int gs_set_active_set_entry(gs_engine* e, uint32_t node, uint32_t bucket, const uint32_t* peers, uint32_t len);
int gs_get_active_set_entry(gs_engine* e, uint32_t node, uint32_t bucket, uint32_t* peers, uint32_t cap,
                            uint32_t* len);

/* --- the per-iteration steps: gossip.rs Cluster -------------------------- */
int gs_fail_nodes(gs_engine* e, const double* fraction_per_slot); /* Cluster::fail_nodes gossip.rs:756 */
int gs_run_gossip(gs_engine* e);                  /* Cluster::run_gossip gossip.rs:494 */
int gs_consume_messages(gs_engine* e);            /* Cluster::consume_messages gossip.rs:618 */
int gs_send_prunes(gs_engine* e);                 /* Cluster::send_prunes gossip.rs:657 */
int gs_prune_connections(gs_engine* e);           /* Cluster::prune_connections gossip.rs:701 */
int gs_chance_to_rotate(gs_engine* e, uint32_t round); /* Cluster::chance_to_rotate gossip.rs:739 */
int gs_record_round(gs_engine* e);                /* stats inserts gossip_main.rs:480-563 */
/* One iteration of gossip_main.rs:449-564 for every slot: run_gossip ->
 * consume -> send_prunes -> prune_connections -> chance_to_rotate(round) ->
 * (record != 0: the measured-round statistics). */
int gs_round(gs_engine* e, uint32_t round, int record);

/* --- readbacks (synchronise the engine stream) ----------------------------- */
int gs_read_hops(gs_engine* e, uint32_t slot, uint8_t* hops /*[n]*/); /* distances; 0xFF = u64::MAX */
/* orders (gossip.rs:601-607) as CSR by destination, each list in consume order
 * (hop, then id). off has n+1 entries. */
int gs_read_inbound(gs_engine* e, uint32_t slot, uint32_t* off, uint32_t* src, uint8_t* hop, size_t cap);
/* prunes of the last send_prunes (pruner, prunee) pairs sorted by (pruner, prunee). */
int gs_read_prunes(gs_engine* e, uint32_t slot, uint32_t* pruner, uint32_t* prunee, size_t cap, size_t* count);
/* ReceivedCache entry (received_cache.rs:13-17) of `node` for the slot's origin, keys sorted. */
int gs_read_cache(gs_engine* e, uint32_t slot, uint32_t node, uint32_t* num_upserts, uint32_t* keys,
                  uint32_t* scores, uint32_t cap, uint32_t* len);
/* Prune state of `node`'s entry for the slot's origin, bit i = i-th peer in FIFO order pruned. */
int gs_read_pruned(gs_engine* e, uint32_t slot, uint32_t node, uint32_t* fifo_mask);
/* Bulk forms for parity diffing: every entry in FIFO order (peers[(node*25+k)*active_set_size + i],
 * len[node*25+k]); every node's cache for the slot (keys sorted, 96 per node); every node's FIFO prune mask. */
int gs_read_active_sets(gs_engine* e, uint32_t* peers, uint8_t* len);
int gs_read_caches(gs_engine* e, uint32_t slot, uint32_t* num_upserts, uint32_t* len, uint32_t* keys,
                   uint32_t* scores);
int gs_read_pruned_all(gs_engine* e, uint32_t slot, uint32_t* fifo_mask);
/* this round's egress/ingress/prune-sent counts (gossip.rs:185-189); egress of an
 * unreached node reads 0 */
int gs_read_counters(gs_engine* e, uint32_t slot, uint32_t* egress, uint32_t* ingress, uint32_t* prune_sent);
/* recorded rounds so far: out[r * n_slots + slot] */
int gs_read_round_summaries(gs_engine* e, gs_round_summary* out, size_t cap, size_t* count);
/* measured-round accumulators: message trackers (gossip_stats.rs:359-461), times
 * stranded per node (gossip_stats.rs:849) and the hop histogram (raw_hop_collection) */
int gs_read_accumulators(gs_engine* e, uint32_t slot, uint64_t* egress, uint64_t* ingress, uint64_t* prunes,
                         uint32_t* stranded_times, uint64_t* hop_hist /*[256]*/);
int gs_read_failed(gs_engine* e, uint32_t slot, uint8_t* failed /*[n]*/);
/* Cluster::mst (gossip.rs:580-591): parent[v] = the node that first discovered v in the
 * reference's FIFO queue order, UINT32_MAX for the origin and unreached nodes (debug
 * readback after gs_run_gossip, n <= 262,144). */
int gs_read_mst(gs_engine* e, uint32_t slot, uint32_t* parent /*[n]*/);
/* GS_FLAG_PROFILE: summed device time of a kernel family ("bfs", "consume",
 * "rotate", "stats") since the last reset, and its launch count. */
int gs_kernel_time(gs_engine* e, const char* family, double* ms, uint64_t* launches);
int gs_kernel_time_reset(gs_engine* e);
int gs_engine_info(gs_engine* e, uint32_t* n_nodes, uint32_t* n_slots, uint32_t* bfs_mode, uint64_t* device_bytes);
/* device_bytes split: per-(slot, node) state (hops, in-degrees, caches, counters,
 * accumulators, record pools; a partition rank's own nodes) and everything else (rows,
 * masks, per-node and per-slot tables, BFS queues). */
int gs_engine_memory(gs_engine* e, uint64_t* pair_bytes, uint64_t* other_bytes);
/* 1 if gs_round runs the one-kernel workgroup round (BFS, consume, prune and
 * statistics per slot in one workgroup), 0 if it launches the step kernels. */
int gs_engine_round_kind(gs_engine* e, uint32_t* fused);
/* Geometry of the multi-source / hybrid BFS (diagnostics; not a reference interface): out[0]
 * frontier entries (multi) or nodes (hybrid) per expand slice, out[1] coarse destination bins,
 * out[2] fine bins, out[3] slots per slot group, out[4] slot groups; with n >= 6, out[5] the
 * workgroups of the persistent BFS launch (0: the launched level loop runs). n >= 5; zeros in
 * other modes. */
int gs_engine_bfs_geometry(gs_engine* e, uint32_t* out, size_t n);

/* --- node-range partition ------------------------------
 * K engines, one per rank/GPU, created with gs_create_part on the same stakes, params
 * (bfs_mode GS_BFS_MULTI or AUTO), slots and seed. Rank r owns the node ids
 * [node_lo, node_hi) (gs_part_sizes): K contiguous ranges of whole 1,024-id bins of
 * C = ceil(n / K) rounded up to 1,024; every rank must own a node ((K - 1) * C < n, else
 * gs_create_part fails with GS_EINVAL on the empty ranks -- check before creating).
 * K = 1 gives one rank owning every node (the exchange calls work; a one-rank group). 
 * Replicated on every rank: active sets, prune masks, failed flags (the same rotations,
 * failures and prune bits are applied everywhere). Kept for owned nodes only: every
 * per-(slot, node) array -- hops, in-degrees, received caches, round counters,
 * accumulators -- i.e. S x (node_hi - node_lo) pairs. Each rank runs the whole BFS over
 * its replicated tables (no exchange per level) and gathers, consumes and prunes for
 * its own nodes. One iteration of gossip_main.rs:449-564 is:
 *   gs_part_round(round, record, &n)        run_gossip + consume + send_prunes; n prune records
 *   ALL-GATHER the n's, then prune_connections by ONE of (every rank picks the same):
 *     records: ALL-GATHER the ranks' records (gs_part_prunes_out, n x 2 u32 words: slot *
 *       n_nodes + prunee, ring-slot bits) -> gs_part_prunes_in(all records); only while
 *       every n <= record_cap (gs_part_exchange_sizes) and the records are the smaller form;
 *     dense: gs_part_prunes_dense_out (dense_words u32 = [n_nodes][n_slots] ring-slot bits)
 *       -> SUM ALL-REDUCE (the ranks' bits are disjoint: SUM = OR) -> gs_part_prunes_dense_in;
 *   gs_chance_to_rotate(round);
 *   if recorded: gs_part_stats_out -> SUM over ranks -> gs_part_stats_in.
 * The exchanges are the caller's: RCCL on device buffers over xGMI, or host buffers
 * (dst_device / src_device select which). Readbacks of per-pair arrays fill the owned
 * nodes (hops 0xFF, counters 0 and empty caches elsewhere); gs_round and the step-wise
 * calls (gs_run_gossip ...) return GS_ESTATE on a partition rank.
 * Replaces: the same loop as gs_round over one engine (results identical on owned nodes). */
int gs_create_part(const gs_params* params, const uint64_t* stakes, uint32_t n_nodes, uint32_t n_slots,
                   uint32_t rank, uint32_t nranks, gs_engine** out);
int gs_part_sizes(gs_engine* e, size_t* stats_words, uint32_t* node_lo, uint32_t* node_hi);
int gs_part_round(gs_engine* e, uint32_t round, int record, uint32_t* n_records);
int gs_part_prunes_out(gs_engine* e, void* dst, int dst_device);                 /* [n_records][2] u32 */
int gs_part_prunes_in(gs_engine* e, const void* src, size_t n_records, int src_device);
int gs_part_exchange_sizes(gs_engine* e, size_t* record_cap, size_t* dense_words);
int gs_part_prunes_dense_out(gs_engine* e, void* dst, int dst_device);           /* [n_nodes][n_slots] u32 */
int gs_part_prunes_dense_in(gs_engine* e, const void* src, int src_device);
/* Frontier exchange (params.flags GS_FLAG_FRONTIER_EXCHANGE; SURVEY 8(e), the north star's
 * "node-range partition with RCCL frontier exchange"). Ranks own whole coarse destination bins
 * (C = ceil(n / K) rounded up to max(1,024, the multi BFS's coarse bin)); each rank expands
 * ONLY the frontier entries of its own nodes, and each level's push records go to the rank
 * owning their destination, which applies them (first arrivals, pool records, its own
 * next-level entries). For each slot group g < n_groups, the BFS is
 *   gs_part_xbfs_begin(g, &n)                        seeds the group's own origins; n own entries
 *   level d = 0, 1, ... while the SUM of n over ranks > 0:
 *     gs_part_xbfs_expand(d, words_to[K])            expand own entries, pack per owner rank
 *     ALL-TO-ALL the K counts, then gs_part_xbfs_send(buf) -> ALL-TO-ALL (split by words_to /
 *       words_from, u64 words: per message the owner's bin counts, then the records)
 *     gs_part_xbfs_apply(d, recv, words_from[K], &n)  apply what every rank pushed here
 *   gs_part_xbfs_end(record)                         gather of the group's own nodes (inbound rows)
 * then gs_part_xround_finish(round, record, &n_records) (consume_messages of every group's rows,
 * send_prunes of own pruners; with GS_MV_FUSED=1 the consume runs fused in xbfs_end instead)
 * in place of gs_part_round; the prune and statistics exchanges follow as above. */
int gs_part_xbfs_groups(gs_engine* e, uint32_t* n_groups);
int gs_part_xbfs_begin(gs_engine* e, uint32_t group, uint32_t* n_local);
int gs_part_xbfs_expand(gs_engine* e, uint32_t level, uint64_t* words_to /*[K]*/);
int gs_part_xbfs_send(gs_engine* e, void* dst, int dst_device);
int gs_part_xbfs_apply(gs_engine* e, uint32_t level, const void* src, const uint64_t* words_from /*[K]*/,
                       int src_device, uint32_t* n_local);
int gs_part_xbfs_end(gs_engine* e, int record);
/* The same level loop without a host wait per level (round 6): every rank's message to rank q
 * goes to the fixed slot [q * cap_words, (q + 1) * cap_words) of `send` (device memory, K
 * slots), so the all-to-all moves K equal slots and no size reaches the host. The caller
 * runs the predicted number of levels (the previous round's, agreed by all ranks; levels
 * past the BFS's end are no-ops), enqueues the collective on the engine's stream
 * (gs_stream), then calls gs_part_xbfs_async_status once: n_local = this rank's entries of
 * the next level (all ranks 0: the BFS is over, else continue with gs_part_xbfs_expand /
 * _apply from that level), overflow = 1 if a message outgrew its slot (then every rank
 * redoes the group: gs_part_xbfs_begin again), words_log [levels][K] = the words each
 * level sent to each rank (the next round's slot sizes). cap_words must hold every rank's
 * bin headers. Replaces the per-level size exchange of gossip.rs:511-609's partitioned
 * form; no reference interface. */
int gs_part_xbfs_expand_async(gs_engine* e, uint32_t level, uint64_t cap_words, void* send);
int gs_part_xbfs_apply_async(gs_engine* e, uint32_t level, const void* recv, uint64_t cap_words);
int gs_part_xbfs_async_status(gs_engine* e, uint32_t* n_local, uint32_t* overflow, uint64_t* words_log,
                              size_t log_levels);
/* The engine's HIP stream (hipStream_t), e.g. to enqueue a collective behind its kernels. */
int gs_stream(gs_engine* e, void** stream);
int gs_part_xround_finish(gs_engine* e, uint32_t round, int record, uint32_t* n_records);
int gs_part_stats_out(gs_engine* e, void* dst, int dst_device);          /* [S][5 + 256 + W] u64 */
int gs_part_stats_in(gs_engine* e, const void* src, int src_device);

/* --- host-side statistics (gossip_stats.rs), f64 in the reference's order --- */
typedef struct gs_hops_stat { double mean, median; uint64_t max, min; } gs_hops_stat;
typedef struct gs_stat4 { double mean, median, max, min; } gs_stat4;
/* HopsStat::new (gossip_stats.rs:47-98) over raw distances (u64::MAX = unreached). */
int gs_hops_stat_new(const uint64_t* hops, size_t n, gs_hops_stat* out);
/* StatCollection::calculate_stats (gossip_stats.rs:266-295). */
int gs_stat_collection_calculate(const double* values, size_t n, gs_stat4* out);

/* --- whole simulations: gossip_main.rs run_simulation ---------------------- */
typedef struct gs_sim_config {  /* gossip.rs Config (gossip.rs:111-133) */
  uint32_t push_fanout, active_set_size, iterations, warm_up_rounds;
  uint32_t min_ingress_nodes, when_to_fail;
  double rotation_probability, prune_stake_threshold, fraction_to_fail;
  uint64_t num_buckets_stranded, num_buckets_message, num_buckets_hops;
  int32_t test_type;  /* 0 none, 1 active-set-size, 2 min-ingress-nodes, 3 push-fanout,
                         4 prune-stake-threshold, 5 fail-nodes, 6 origin-rank, 7 rotate-probability */
  uint64_t seed;
  int32_t device;
  uint32_t bfs_mode;
} gs_sim_config;

typedef struct gs_sim_result gs_sim_result;
/* Runs n_sims simulations that share one active-set trajectory as slots of one
 * engine; sims differ only in origin_rank / min_ingress / threshold / fraction. */
int gs_run_simulations(const gs_sim_config* cfg, const uint64_t* stakes, uint32_t n_nodes, uint32_t n_sims,
                       const uint32_t* origin_ranks, const uint32_t* min_ingress, const double* thresholds,
                       const double* fractions, gs_sim_result** out);
void gs_result_free(gs_sim_result* r);
/* Named arrays of a finished sim (same names as the oracle): e.g. "coverage",
 * "rmr", "coverage_stats", "stranded", "hops_hist" ... Returns the element
 * count (copies min(count, cap)); SIZE_MAX for an unknown name. */
size_t gs_result_f64(const gs_sim_result* r, uint32_t sim, const char* name, double* out, size_t cap);
size_t gs_result_u64(const gs_sim_result* r, uint32_t sim, const char* name, uint64_t* out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_HIP_H */
