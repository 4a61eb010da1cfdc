/*
 * gossip.h -- C ABI of the MI355X gossip-propagation engine (libgossip.so).
 *
 * Drop-in boundary for the reference's hot path
 *     P2PNode::HandleRead -> seen-set check -> GossipShareToPeers
 * (p2pnode.cc:127-199), which NS-3 drives one packet at a time through the socket
 * receive callback bound at p2pnode.cc:74 and p2pnetwork.cc:142.  This ABI replaces
 * that callback chain with a tick-synchronous bulk engine (one tick = --Latency) whose
 * hot loop runs as hand-written gfx950 HIP kernels.
 *
 * Conventions
 *   - Every call returns 0 on success or a negative GOSSIP_E* code; the text of the last
 *     error on the calling thread is available from gossip_last_error().  No C++
 *     exception crosses this boundary (the reference propagates no errors at all:
 *     p2pnode.cc:147-151 silently erases a socket on a failed Send).
 *   - Handles are opaque and NOT thread-safe per handle, like the single-threaded NS-3
 *     event loop they replace (p2pnetwork.cc:216).
 *   - Device buffers are engine-owned; host arrays are caller-owned and only read or
 *     written during the call.
 *   - There is no CPU fallback: without a HIP device gossip_engine_create fails.
 */
#ifndef GOSSIP_H
#define GOSSIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GOSSIP_OK 0
#define GOSSIP_EINVAL (-1)   /* bad argument                                  */
#define GOSSIP_EHIP (-2)     /* HIP runtime error (no device, launch failure) */
#define GOSSIP_ENOMEM (-3)   /* host or device allocation failed              */
#define GOSSIP_ESTATE (-4)   /* call out of order (e.g. run before graph)     */
#define GOSSIP_ECAPACITY (-5) /* live-share window exceeded the frontier capacity */

const char* gossip_last_error(void);
const char* gossip_version(void);

/* ------------------------------------------------------------------------------------
 * Time (ns-3 Time semantics, ns resolution).  Seconds()/MilliSeconds() as used at
 * p2pnode.cc:101, p2pnetwork.cc:93,114,206: exact round-half-up of value*10^k.
 * ---------------------------------------------------------------------------------- */
int64_t gossip_seconds_to_ns(double seconds);
int64_t gossip_milliseconds_to_ns(double ms);

/* ------------------------------------------------------------------------------------
 * Topology: replaces P2PGossipNetworkSimulation::CreateRandomTopology +
 * ConnectNodes + makeconnections/ConnectPeerSockets + the REGISTER branch of HandleRead
 * (p2pnetwork.cc:62-150, p2pnode.cc:77-89,178-188).
 *
 * A "link" is a key (a,b) of the reference's `connections` map (p2pnetwork.cc:30).
 * Peer lists follow from the keys: key (a,b) puts b in peers(a) (AddPeer, de-duplicated)
 * and a in peers(b) (REGISTER, not de-duplicated), so a parallel link gives multiplicity 2.
 * ---------------------------------------------------------------------------------- */
typedef struct gossip_topology gossip_topology;

#define GOSSIP_TOPO_EXACT 0 /* the reference's mt19937 stream: O(n^2) draws, bit-exact   */
#define GOSSIP_TOPO_SKIP 1  /* geometric skipping, Philox4x32-10 per row: O(links), for
                               n far beyond the reference's limit; same fix-up rule      */

int gossip_topology_create(uint32_t num_nodes, double connection_prob, uint32_t seed,
                           int kind, int num_threads, gossip_topology** out);
/* Import an explicit key list (e.g. a dump of an NS-3 run); keys are (a,b), a != b. */
int gossip_topology_from_links(uint32_t num_nodes, uint64_t num_links, const uint32_t* a,
                               const uint32_t* b, gossip_topology** out);
/* Read a key list written by gossip_sim --dumpLinks: one "a b" pair of unsigned decimals per line
 * (spaces or tabs, blank lines skipped).  Strict: a missing or extra field, a sign, a non-digit,
 * an overflow, a node >= num_nodes or a self-loop is GOSSIP_EINVAL naming the line (the
 * reference's own parser, Share::FromString p2pnode.cc:13-30, leaves fields uninitialised on
 * malformed input).  Then as gossip_topology_from_links. */
int gossip_topology_load_links(uint32_t num_nodes, const char* path, gossip_topology** out);
uint32_t gossip_topology_num_nodes(const gossip_topology* t);
uint64_t gossip_topology_num_links(const gossip_topology* t);
/* Keys in std::map order. */
int gossip_topology_get_links(const gossip_topology* t, uint32_t* a, uint32_t* b);
/* Directed adjacency with multiplicity: CSR over distinct neighbours. */
uint64_t gossip_topology_num_entries(const gossip_topology* t);
int gossip_topology_get_csr(const gossip_topology* t, int64_t* row_ptr, int32_t* col,
                            uint8_t* mult);
/* Per node: |peers| (PrintStatistics "Peer count", p2pnetwork.cc:276) and
 * |peersockets| ("Socket connections", :277). */
int gossip_topology_get_degrees(const gossip_topology* t, uint32_t* peers, uint32_t* sockets);
void gossip_topology_destroy(gossip_topology* t);

/* ------------------------------------------------------------------------------------
 * Share-generation schedule: replaces P2PNode's per-node mt19937 seeding and the
 * ScheduleNextShare / GenerateAndGossipShare / GenerateUniqueShareId chain
 * (p2pnode.cc:33-43, 91-125, 201-209).  Only COUNTED generations are emitted:
 * t_start_ns <= t < t_cut_ns (earlier events hit the peers.empty() branch, later ones
 * happen after PrintStatistics).
 * ---------------------------------------------------------------------------------- */
typedef struct gossip_gen_event {
    int64_t ns;        /* Simulator::Now() at GenerateAndGossipShare        */
    uint32_t node;     /* originNodeId                                      */
    uint32_t share_id; /* GenerateUniqueShareId(): the seen-set key         */
} gossip_gen_event;

typedef struct gossip_schedule gossip_schedule;

/* node_seed replaces std::random_device at p2pnode.cc:41 (node i seeds node_seed + i).
 * id_mask != 0 ANDs every shareId (test knob that forces id collisions at small n).
 * t_gen_end_ns (<= t_cut_ns, or 0 for t_cut_ns) stops emitting early for bounded runs. */
int gossip_schedule_create(uint32_t num_nodes, uint32_t node_seed, int64_t t_start_ns,
                           int64_t t_cut_ns, int64_t t_gen_end_ns, uint32_t id_mask,
                           int num_threads, gossip_schedule** out);
/* Events in any order (sorted here); a negative ns is GOSSIP_EINVAL. */
int gossip_schedule_from_events(uint64_t num_events, const gossip_gen_event* ev,
                                gossip_schedule** out);
/* Read events written by gossip_sim --dumpEvents: "ns node shareId" per line, parsed as strictly
 * as gossip_topology_load_links (ns <= INT64_MAX, node < num_nodes unless num_nodes is 0). */
int gossip_schedule_load_events(uint32_t num_nodes, const char* path, gossip_schedule** out);
/* Synthetic schedule generated on GPU `device` (schedule_gpu.hip): the reference's rules --
 * first event at U(2,5) s, then every U(2,5) s; counted iff t_start <= t < t_cut (and
 * < t_gen_end if nonzero); shareId from GenerateUniqueShareId's formula -- with each node's
 * U(2,5) draws taken from a counter-based Philox4x32-10 stream keyed by (seed, node) instead of
 * the reference's mt19937(seed + node).  For large synthetic runs; not the reference's stream. */
int gossip_schedule_create_philox(uint32_t num_nodes, uint32_t seed, int64_t t_start_ns,
                                  int64_t t_cut_ns, int64_t t_gen_end_ns, int32_t device,
                                  gossip_schedule** out);
uint64_t gossip_schedule_size(const gossip_schedule* s);
/* Events sorted by (ns, node). */
int gossip_schedule_get(const gossip_schedule* s, gossip_gen_event* out);
void gossip_schedule_destroy(gossip_schedule* s);

/* Multi-GPU sharding rule (the one every engine with shard_count > 1 applies): owner[k] =
 * the shard that simulates event k.  Generations sharing an id inside one connected
 * component (one seen-set entry, p2pnode.cc:189) always land on the same shard, so shards
 * never interact and per-node counters add up exactly across shards. */
/* The birth-tick rule (GOSSIP_F_SHARD_BY_TICK): owner[k] = (floor(first ns of k's instance /
 * latency_ns)) mod shard_count, the instance being k's (id, node) when k's id is unique and its
 * (id, connected component) otherwise -- colliding-id instances stay whole. */
int gossip_shard_events_by_tick(const gossip_topology* t, uint64_t num_events, const gossip_gen_event* ev,
                                uint32_t shard_count, int64_t latency_ns, uint32_t* owner);
int gossip_shard_events(const gossip_topology* t, uint64_t num_events, const gossip_gen_event* ev,
                        uint32_t shard_count, uint32_t* owner);

/* ------------------------------------------------------------------------------------
 * Engine: replaces the per-packet HandleRead -> ReceiveShare -> GossipShareToPeers
 * loop (p2pnode.cc:127-199) for all nodes at once, one tick (= Latency) per step.
 * ---------------------------------------------------------------------------------- */
typedef struct gossip_engine gossip_engine;

#define GOSSIP_MODE_AUTO 0 /* DENSE when nnz >= 0.05 n^2 and 2048 <= n <= 2^19, else CSR */
#define GOSSIP_MODE_CSR 1 /* bit-sliced frontier, CSR pull kernel              */
#define GOSSIP_MODE_DENSE 2 /* adjacency x frontier as an int8 MFMA contraction (int32
                               accumulate: exact per-node copy counts); dense graphs,
                               n up to ~10^5 (the adjacency is n^2 bytes of HBM)      */

typedef struct gossip_config {
    uint32_t num_nodes;
    int64_t latency_ns;   /* MilliSeconds(--Latency), channel Delay p2pnetwork.cc:114 */
    int64_t t_start_ns;   /* makeconnections time, Seconds(5) p2pnetwork.cc:93        */
    int64_t t_cut_ns;     /* PrintStatistics time, Seconds(simTime-0.1) :206           */
    int32_t device;       /* HIP device ordinal                                        */
    int32_t mode;         /* GOSSIP_MODE_*                                             */
    uint32_t max_words;   /* frontier capacity, 64-share words per node (0 = auto)     */
    uint32_t shard_rank;  /* share-class sharding across engines (multi-GPU)           */
    uint32_t shard_count; /* 0 or 1 = no sharding                                      */
    uint32_t flags;       /* GOSSIP_F_*                                                */
} gossip_config;

#define GOSSIP_F_TRACE 1u  /* record first-contact (node, shareId, tick) for tests  */
#define GOSSIP_F_TIMING 2u /* time each pull-kernel launch with HIP events          */
#define GOSSIP_F_NOSKIP 4u /* diagnostic: dense pull (no dead/saturated skipping);
                              results are identical, only the bytes read change       */
/* (flag values 8 and 16 -- the round-1 scalar-peer pull kernel and its opposite -- are retired
 *  and ignored) */
#define GOSSIP_F_TILE_PER_TICK 32u /* open a fresh 1024-share tile every tick: tests (wide,
                                      sparsely filled windows at small n) and the birth-tick
                                      share shards (bench.py shard_flags: single-age tiles) */
#define GOSSIP_F_HOP_BATCH 128u /* hop-batched run: generation g of every node is simulated in
                                   batched tick g (its phase kept) and the cut / snapshots are
                                   applied per share from the real times -- exact when no two
                                   generations share an id (n <= 128,849; EINVAL otherwise).
                                   Thousands of concurrent shares per step instead of a few:
                                   the dense (MFMA) path's mode for small graphs.  The run ends
                                   when every flood has retired (end_tick is not meaningful);
                                   snapshots are read after the complete run.                  */
#define GOSSIP_F_HANDSHAKE 64u /* NS-3 handshake window (p2pnetwork.cc:133-150,
                                  p2pnode.cc:178-188): shares a node sends before t_start + 2
                                  latency ride its REGISTER segment and are lost (still counted
                                  as sent); until REGISTER arrives at t_start + 3 latency a
                                  node's peers are its connector-side keys only.  Needs
                                  gossip_engine_set_topology, CSR mode, t_start % latency == 0
                                  and t_cut >= t_start + 3 latency.                          */
#define GOSSIP_F_SHARD_BY_TICK 256u /* share shards (shard_count > 1) by birth tick: an instance
                                       belongs to shard (tick of its first generation) mod
                                       shard_count instead of a hash of its key, so a shard's
                                       births of a tick fill whole tiles of one age
                                       (gossip_shard_events_by_tick; every engine of a job must
                                       use the same rule)                                        */

int gossip_engine_create(const gossip_config* cfg, gossip_engine** out);
/* Graph: CSR over distinct neighbours with multiplicity in {1,2} (see topology above). */
int gossip_engine_set_graph(gossip_engine* e, uint32_t num_nodes, const int64_t* row_ptr,
                            const int32_t* col, const uint8_t* mult);
int gossip_engine_set_topology(gossip_engine* e, const gossip_topology* t);
/* Generation events (any order; the engine buckets them by tick). */
int gossip_engine_set_schedule(gossip_engine* e, uint64_t num_events,
                               const gossip_gen_event* ev);
int gossip_engine_set_schedule_obj(gossip_engine* e, const gossip_schedule* s);
/* Stats snapshots at absolute times (PrintPeriodicStats, p2pnetwork.cc:201-204). */
int gossip_engine_add_snapshot(gossip_engine* e, int64_t t_ns);
/* Row partition (the north star's multi-GPU layout): engine `rank` of `count`
 * pulls, dedups and counts only its block of node rows (512-row blocks, rank r owns
 * [r*B, min(n, (r+1)*B)) with B = roundup(ceil(n/count), 512)) and every rank holds the whole
 * graph and frontier: after each tick the ranks exchange their rows of the new frontier, their
 * tile-occupancy words and their liveness words.  Exchange backends: RCCL over xGMI
 * (gossip_rccl_unique_id on one rank, shared out of band, then gossip_engine_connect_rccl on
 * every rank; gossip_engine_run then exchanges on the engine's stream), or
 * gossip_engine_group_run, which steps the engines of a partition in lockstep in one thread
 * with device copies (one device: the rehearsal/test backend).  Per-node counters are non-zero
 * only on the owning rank: sum them (and snapshot processed totals) over ranks; snapshot
 * generation totals are global on every rank.  Call before the graph; not with
 * GOSSIP_F_HANDSHAKE or share sharding. */
int gossip_engine_set_row_partition(gossip_engine* e, uint32_t rank, uint32_t count);
int gossip_rccl_unique_id(uint8_t* out, uint32_t len); /* len >= 128 (ncclUniqueId) */
int gossip_engine_connect_rccl(gossip_engine* e, const uint8_t* unique_id, uint32_t len);
/* Abort the engine's RCCL communicator (ncclCommAbort).  The one call that may be made from
 * another thread while the engine is inside gossip_engine_run: when one rank of a partition
 * fails, its peers are blocked in a collective that can never complete; aborting their
 * communicators makes their gossip_engine_run return GOSSIP_EHIP instead of hanging.  The
 * engine is then only good for gossip_engine_destroy: every later step (gossip_engine_run,
 * group_run, tick_begin) and every collective its thread would still issue returns
 * GOSSIP_ESTATE, with or without a communicator. */
int gossip_engine_abort(gossip_engine* e);
/* Lockstep backend: the ranks' engines must all be on ONE device (the unpack reads the other
 * ranks' messages in place; no peer access is enabled). */
int gossip_engine_group_run(gossip_engine** engines, uint32_t count, int64_t tick_end);
/* The exchange moves only OCCUPIED 16-word tile rows of F_next (the tile-occupancy bits), with
 * the occupancy words, per-node row offsets and the rank's liveness words: one message per rank
 * and tick.  Host-staged backend (any transport: gloo, MPI, sockets): per tick every rank calls
 *   gossip_engine_tick_begin       pull + births of the tick, packs the rank's message
 *                                  (returns 1 instead of 0 when the run is complete)
 *   gossip_engine_exchange_export  copies the message to host memory (buf NULL: size only)
 *   gossip_engine_exchange_import  once per other rank, with that rank's message
 *   gossip_engine_tick_end         liveness, retirement, next tick
 * Pipelined form (what the RCCL backend does): the own rows are pulled in
 * gossip_engine_exchange_chunks(e) row chunks (option "xchunks", default 4, equal on every rank;
 * 512-row blocks), and chunk c's message can leave as soon as that chunk is computed, while the
 * GPU computes chunk c + 1: per chunk c, export_chunk then import_chunk from every other rank
 * (the rank's liveness words ride in its last chunk).  tick_begin only enqueues the tick's
 * kernels; an export waits for its chunk on the engine's exchange stream.  The whole-rows
 * export/import above are the same exchange in one message per rank (not to be mixed with the
 * chunked calls inside one tick). */
int gossip_engine_tick_begin(gossip_engine* e);
int gossip_engine_exchange_export(gossip_engine* e, void* buf, uint64_t cap_bytes, uint64_t* bytes);
int gossip_engine_exchange_import(gossip_engine* e, uint32_t rank, const void* buf, uint64_t bytes);
int gossip_engine_exchange_chunks(const gossip_engine* e);
int gossip_engine_exchange_export_chunk(gossip_engine* e, uint32_t chunk, void* buf, uint64_t cap_bytes,
                                        uint64_t* bytes);
int gossip_engine_exchange_import_chunk(gossip_engine* e, uint32_t rank, uint32_t chunk, const void* buf,
                                        uint64_t bytes);
int gossip_engine_tick_end(gossip_engine* e);

/* NS-3 link timing: every hop of a share costs
 *     latency + send_defer_ns + (len(message) + header_bytes) * ns_per_byte
 * instead of the bare channel delay.  message = Share::ToString() (p2pnode.cc:6-11),
 * "SHARE:<origin>:<shareId>:<timestamp>" with the timestamp streamed as a double in
 * seconds (%g, 6 significant digits), so a share keeps one per-hop delay along its whole
 * flood (a forwarded share is re-serialised from the parsed fields, p2pnode.cc:13-30,138).
 * The 5 Mbps links of p2pnetwork.cc:113 give ns_per_byte = 1600; a data segment carries
 * PPP(2) + IPv4(20) + TCP with the timestamp option (32) = 54 header bytes; TcpSocketBase
 * defers SendPendingData by one TimeStep (send_defer_ns = 1).  Hop counts are unchanged
 * (the delay is uniform along a flood); the PrintStatistics cut and the periodic snapshots
 * see the later arrival times.  Needs GOSSIP_F_HOP_BATCH (hence unique share ids); call
 * before gossip_engine_set_schedule.  gossip_share_message_length gives len(message). */
int gossip_engine_set_link_timing(gossip_engine* e, int64_t ns_per_byte, uint32_t header_bytes,
                                  int64_t send_defer_ns);
uint32_t gossip_share_message_length(uint32_t origin, uint32_t share_id, int64_t t_ns);
/* Tuning options of one engine (results never depend on them; A/B runs and tests).  The
 * environment variable in brackets gives the default:
 *   "pull_nt"          -1 auto (non-temporal rows when the live frontier n x wact x 8 B exceeds
 *                      16 GiB), 0 / 1 forced                              [GOSSIP_PULL_NT]
 *   "pull_grid"        blocks per pull launch, 0 = auto (16,384 non-temporal, else 4,096)
 *                                                                         [GOSSIP_PULL_GRID]
 *   "pull_tile_order"  1: k_pull's tile lists in age order inside each occupancy word (default),
 *                      0: in tile order                                [GOSSIP_PULL_TILE_ORDER]
 *   "dense_min_tiles"  MFMA block tiles the K split aims for (512)  [GOSSIP_DENSE_MIN_TILES]
 *   "dense_fused"      1: a DENSE tick runs as one k_dense_fused launch when it can (no id-group
 *                      words, no row partition, no no-skip diagnostic; the default), 0: always
 *                      k_transpose + k_dense_bits + k_dense_dedup            [GOSSIP_DENSE_FUSED]
 *   "young"            young-tile slots (k_pull_young): -1 auto (CSR tick engine, n >= 2^20),
 *                      0 off, 1 on (before the schedule)                    [GOSSIP_YOUNG]
 *   "young_age"        tiles stay in slots while their oldest shares are <= this many hops (5)
 *                                                                          [GOSSIP_YOUNG_AGE]
 *   "young_cap"        slot entries per node before it falls back to dense rows (1..127)
 *                                                                          [GOSSIP_YOUNG_CAP]
 *   "pull_gate"        1: k_pull skips the own-seen loads of tiles no peer holds a row of (the
 *                      default), 0: reads every live pair                     [GOSSIP_PULL_GATE]
 *   "pull_sat"         1: k_pull keeps a saturation bit per (node, tile) -- every live column of
 *                      the tile seen -- and skips saturated tiles until a birth lands in them
 *                      (default), 0: off                                       [GOSSIP_PULL_SAT]
 *   "dense_rows"       tiles whose frontier rows are expected dense everywhere are written whole
 *                      (zeros included) and read the next tick without occupancy words: -1 auto
 *                      (BFS layer model of the graph, default), 0 off, 1 every listed tile
 *                      (tests)                                                [GOSSIP_DENSE_ROWS]
 *   "young_grid"       k_pull_young blocks, 0 = twice the pull grid          [GOSSIP_YOUNG_GRID]
 *   "young_list_cap"   seen-list entries per node (1..127, default 127): beyond it a list overflows
 *                      to dense seen rows (tests: small lists exercise the overflow paths)
 *   "young_nt"         1: k_pull_young reads its peers' slot lines non-temporally (default), 0:
 *                      cached                                                  [GOSSIP_YOUNG_NT]
 *   "pull_push"        push marks: rows of tiles whose next frontier sits on few nodes mark their
 *                      writers' peers, and the next tick's k_pull skips those tiles at unmarked
 *                      nodes; -1 auto (BFS layer model: marked nodes expected < 50 %, default), 0
 *                      off, 1 every listed tile that is not dense-row (tests)  [GOSSIP_PULL_PUSH]
 *   "young_idle"       1: on a tick whose k_pull_young reads only stamped slots and keeps every seen
 *                      list, nodes without a stamped peer skip the per-node walk (default), 0: off
 *                                                                          [GOSSIP_YOUNG_IDLE]
 *   "young_skip"       empty-slot skipping: on a tick whose slots are expected mostly empty, every
 *                      writer of a non-empty slot stamps its peers' hint bytes and the next tick's
 *                      k_pull_young loads only the stamped peers' slot lines; -1 auto (the BFS
 *                      layer model expects < 30 % of the slots non-empty, default), 0 off, 1 every
 *                      tick (tests)                                          [GOSSIP_YOUNG_SKIP]
 *   "young_overlap"    0: k_pull_young after k_pull on the engine stream; 1: the two run
 *                      concurrently on two streams, k_pull_young launched first (default)
 *                                                                   [GOSSIP_YOUNG_OVERLAP]
 *   "mem_limit"        bytes of device memory the engine may hold, 0 = what the device has
 *                      free; a window that outgrows it fails with GOSSIP_ECAPACITY / ENOMEM
 *                      (callers then split the shares into more shards)   [GOSSIP_MEM_LIMIT]
 *   "late_age"         k_pull stops gathering a node's peer rows of a tile at least this many
 *                      ticks old once they cover every bit it can still take (bottom-up early
 *                      exit); 0 = off, -1 = auto (1: every tile of a CSR pull; 0 in DENSE
 *                      mode, which gathers nothing)                          [GOSSIP_LATE_AGE]
 *   "xchunks"          row partition: row chunks per tick of the pipelined exchange, 1..16 (4);
 *                      equal on every rank of a partition                    [GOSSIP_XCHUNKS]
 *   "rehearse_rows"    diagnostic, R >= 2 on an unpartitioned CSR engine (before the schedule;
 *                      young tiles off, as on a row rank): the pull runs as R launches over the
 *                      row blocks of an R-rank partition, and after each tick every block's
 *                      F_next rows go through the exchange's pack and unpack kernels (unpacked
 *                      into the same rows: results unchanged), each step timed per block with
 *                      GOSSIP_F_TIMING -- one rank's compute and exchange work, measured on one
 *                      GPU over the whole graph's data (gossip_engine_get_rehearsal) */
int gossip_engine_set_option(gossip_engine* e, const char* name, int64_t value);
/* The value an option holds (what set_option or its environment default set; 0 / -1 = auto where
 * the table above says so).  GOSSIP_EINVAL for an unknown name. */
int gossip_engine_get_option(const gossip_engine* e, const char* name, int64_t* value);
/* The mode the engine runs (AUTO resolves at gossip_engine_set_graph). */
int gossip_engine_mode(const gossip_engine* e);
/* First tick of the run window (floor(t_start/L)) and one past the last tick. */
int64_t gossip_engine_first_tick(const gossip_engine* e);
int64_t gossip_engine_end_tick(const gossip_engine* e);
int64_t gossip_engine_current_tick(const gossip_engine* e);
/* Advance the simulation to tick_end (exclusive); returns when the work is enqueued
 * and the host has caught up (call gossip_engine_sync to wait for the device). */
int gossip_engine_run(gossip_engine* e, int64_t tick_end);
int gossip_engine_sync(gossip_engine* e);

/* Per-node report (PrintStatistics p2pnetwork.cc:271-277).  NULL pointers skipped. */
int gossip_engine_get_stats(gossip_engine* e, uint32_t* gen, uint32_t* recv, uint32_t* fwd,
                            uint64_t* sent, uint32_t* processed, uint32_t* peers,
                            uint32_t* sockets);
/* Snapshot k: time, total generated, total processed (uint64, no wrap). */
int gossip_engine_get_snapshot(gossip_engine* e, uint32_t k, int64_t* t_ns,
                               uint64_t* total_gen, uint64_t* total_processed);

typedef struct gossip_counters {
    uint64_t edge_events;      /* sum of sends so far (= "Total shares sent")      */
    uint64_t receptions;       /* first arrivals (ReceiveShare calls)               */
    uint64_t generations;      /* counted generations                               */
    uint64_t ticks;            /* ticks simulated                                   */
    uint64_t pull_launches;    /* pull-kernel launches                              */
    double pull_ms;            /* summed HIP-event time of pull launches (TIMING)   */
    uint64_t pull_bytes;       /* SURVEY 8d dense-pull bytes of those launches:
                                  8(n+1) + 4nnz + 8*Wq*nnz + 24*Wq*n + 16n each       */
    uint32_t words_hw;         /* high-water frontier words per node                */
    uint32_t words_cap;        /* frontier capacity (words per node)                */
    uint64_t device_bytes;     /* device memory held by the engine                  */
    uint64_t pull_bytes_moved; /* bytes the pull kernels actually had to move after
                                  dead-word / saturated-node skipping (since reset)   */
    uint64_t pull_pair_edges;  /* (edge, 16-B word pair) neighbour reads (since reset) */
    uint64_t dense_ops;        /* DENSE mode: int8 MAC ops x2 of the MFMA work computed =
                                  2 * 256 * 256 * 1024 per (256x256 output tile, 1,024-node K
                                  stage) computed; empty stages are skipped, not counted */
    uint64_t dense_tiles_skipped; /* DENSE mode: output tiles skipped as dead           */
    /* pull traffic breakdown since reset (each a count of the unit in brackets):         */
    uint64_t pull_col_ids;     /* peer ids loaded [4 B]                                 */
    uint64_t pull_seen_reads;  /* own seen pairs used by live work items [16 B]         */
    uint64_t pull_seen_writes; /* own seen pairs written [16 B]                         */
    uint64_t pull_f_writes;    /* F_next pairs written [16 B]                           */
    uint64_t pull_nz_reads;    /* peer tile-occupancy words loaded [8 B]                */
    uint32_t pull_nt;          /* variant of the last pull launch: 1 = non-temporal rows */
    uint32_t pull_grid;        /* blocks of the last pull launch                        */
    /* young tiles (k_pull_young) since reset; its time is NOT in pull_ms                  */
    double young_ms;           /* summed HIP-event time of k_pull_young (TIMING)        */
    uint64_t young_launches;
    uint64_t young_bytes_moved;   /* bytes k_pull_young had to move                     */
    uint64_t young_slot_lines;    /* peer slot lines read [128 B]                        */
    uint64_t young_col_ids;       /* peer ids loaded [4 B]                               */
    uint64_t young_fallback_rows; /* dense rows read from overflowed peers [128 B]       */
    uint64_t young_seen_reads;    /* own seen words read [8 B]                           */
    uint64_t young_seen_writes;   /* own seen words written [8 B]                        */
    uint64_t young_rows_written;  /* dense tile rows written [128 B]                     */
    uint64_t young_slot_writes;   /* slot lines written [128 B]                          */
    /* row partition: bytes of the compressed frontier exchange (packed own rows sent,
       other ranks' rows received) since creation                                            */
    uint64_t exchange_bytes_sent;
    uint64_t exchange_bytes_received;
    /* wall time of the pull phase (k_pull and k_pull_young, concurrent on two streams when the
     * young_overlap option is on), HIP events on the engine stream (TIMING) */
    double pull_phase_ms;
    uint64_t young_line2_misses; /* second slot lines fetched without a hint (k_pull_young) */
    uint32_t pull_late_age;      /* late_age in effect for the last pull (0: no early exit) */
    uint32_t pull_tiles;         /* 1: the last tick's k_pull passes ran over tile lists (option pull_tiles) */
    uint64_t young_fresh_lines;  /* seen rows k_pull_young wrote whole [128 B]: materialised from the
                                    seen lists of tiles leaving the young set, and fresh tiles cleared
                                    at nodes whose list overflowed; in young_bytes_moved */
    uint32_t pull_lpw;           /* word-lanes per node of the last k_pull launch (32: k_pull<32,1>) */
    uint32_t pull_dense_tiles;   /* tiles the last tick's k_pull read as dense rows (option dense_rows) */
    uint64_t pull_sat_skips;     /* (node, tile) items k_pull skipped as saturated since reset (pull_sat) */
    uint32_t pull_sat;           /* 1: the last tick's k_pull kept saturation bits (option pull_sat) */
    uint32_t pad0;
    uint64_t window_early_retires; /* allocations that first retired tiles from the last tick's
                                      liveness (the window near its capacity) since creation */
    uint64_t young_list_lines;   /* seen-list lines k_pull_young read and wrote [128 B] since reset */
    uint64_t pull_items;         /* k_pull work items (node, pass) since reset */
    uint64_t pull_gather_items;  /* of those, items that gathered some peer row since reset */
    uint64_t dense_fused_launches; /* DENSE ticks run as one k_dense_fused launch (contraction + dedup +
                                      transposed F_next) since creation; the others ran k_transpose,
                                      k_dense_bits and k_dense_dedup (option dense_fused)       */
    uint32_t young_grid;         /* blocks of the last k_pull_young launch (option young_grid resolved) */
    uint32_t young_skip_ticks;   /* k_pull_young launches that read only stamped slots (young_skip) since reset */
    /* push marks (option pull_push) since reset: (tile, tick) pairs k_pull skipped at unmarked nodes,
       (tile, tick) pairs whose rows marked their writers' peers, and marks set (8-B atomics) */
    uint64_t pull_push_tiles;
    uint64_t pull_pushw_tiles;
    uint64_t pull_marks;
    uint64_t young_idle_ticks;   /* k_pull_young launches that skipped their idle nodes' walks (young_idle) */
} gossip_counters;
int gossip_engine_get_counters(gossip_engine* e, gossip_counters* c);
/* Option rehearse_rows = R: per row block r < R, summed since the last reset_timing -- pull time,
 * pack time, unpack time (ms, HIP events) and message bytes; *ticks = ticks rehearsed. */
int gossip_engine_get_rehearsal(gossip_engine* e, uint32_t ranges, double* pull_ms, double* pack_ms,
                                double* unpack_ms, uint64_t* msg_bytes, uint64_t* ticks);
/* The same rehearsal: per row block, the largest message of one tick (bytes) since reset_timing --
 * what a rank's exchange buffers must hold, where get_rehearsal's sums give the mean. */
int gossip_engine_get_rehearsal_peak(gossip_engine* e, uint32_t ranges, uint64_t* msg_bytes_max);
int gossip_engine_reset_timing(gossip_engine* e);

/* First-contact trace (GOSSIP_F_TRACE): one record per (node, shareId) whose first
 * contact happened in a simulated tick; via_recv=1 for ReceiveShare, 0 for own
 * generation; hop = ticks since the winning source's generation. */
uint64_t gossip_engine_trace_size(const gossip_engine* e);
int gossip_engine_get_trace(const gossip_engine* e, uint32_t* node, uint32_t* share_id,
                            int64_t* tick, uint32_t* hop, uint8_t* via_recv);

void gossip_engine_destroy(gossip_engine* e);

/* ------------------------------------------------------------------------------------
 * Event log: the reference's per-event NS_LOG_INFO lines (p2pnode.cc:88,122,143-144,160-161,
 * 184,191-192) rendered from a first-contact trace (gossip_engine_get_trace, or ORACLE A's)
 * plus the topology's peer lists, for events in [t_start, t_cut).  ev: the run's generation
 * events with their real times, unique ids.  Lines of one nanosecond come in a canonical
 * order (node, first contact before duplicates, share); with_time != 0 prefixes each line
 * with "<t_ns>\t".  ns_per_byte/header_bytes/send_defer_ns: the link timing of the run
 * (0, 0, 0 = ideal hop).  Writes into buf like gossip_format_statistics; returns the full
 * length or a negative status.  Cost and size O(edge events): small runs only.
 * ---------------------------------------------------------------------------------- */
int64_t gossip_format_event_log(const gossip_topology* t, uint64_t num_events,
                                const gossip_gen_event* ev, uint64_t num_trace,
                                const uint32_t* tr_node, const uint32_t* tr_share_id,
                                const uint32_t* tr_hop, const uint8_t* tr_via_recv,
                                int64_t latency_ns, int64_t t_start_ns, int64_t t_cut_ns,
                                int64_t ns_per_byte, uint32_t header_bytes,
                                int64_t send_defer_ns, int with_time, char* buf,
                                uint64_t buf_len);
/* NetAnim XML of SetupNetAnim (p2pnetwork.cc:153-190): the node grid, descriptions, colours
 * and links, plus -- packets != 0, EnablePacketMetadata(true) at :187 -- one <p> record per
 * gossip Send (p2pnode.cc:140) derived from a run's first-contact trace as in the event log
 * (fbTx/lbTx/fbRx/lbRx in seconds from the link model: latency, send deferral and
 * (len(message) + header_bytes) x ns_per_byte; meta-info = the Share::ToString() payload).  Needs
 * unique share ids.  TCP handshake, ACK and REGISTER segments are not recorded.  Writes into
 * buf (NUL-terminated) and returns the full length; buf=NULL sizes it. */
int64_t gossip_format_netanim(const gossip_topology* t, uint64_t num_events, const gossip_gen_event* ev,
                              uint64_t num_trace, const uint32_t* tr_node, const uint32_t* tr_share_id,
                              const uint32_t* tr_hop, int64_t latency_ns, int64_t t_cut_ns,
                              int64_t ns_per_byte, uint32_t header_bytes, int64_t send_defer_ns,
                              int packets, char* buf, uint64_t buf_len);

/* ------------------------------------------------------------------------------------
 * Report: the exact NS_LOG_INFO lines of PrintStatistics (p2pnetwork.cc:255-284) and
 * PrintPeriodicStats (:233-249), uint32 accumulators included.  Writes into buf
 * (NUL-terminated) and returns the full length; call with buf=NULL to size it.
 * ---------------------------------------------------------------------------------- */
int64_t gossip_format_statistics(uint32_t num_nodes, const uint32_t* gen, const uint32_t* recv,
                                 const uint32_t* fwd, const uint64_t* sent,
                                 const uint32_t* processed, const uint32_t* peers,
                                 const uint32_t* sockets, char* buf, uint64_t buf_len);
int64_t gossip_format_periodic(double t_seconds, uint32_t num_nodes, uint64_t total_gen,
                               uint64_t total_processed, uint64_t total_sockets, char* buf,
                               uint64_t buf_len);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_H */
