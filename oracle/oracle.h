/*
 * oracle.h -- C API of ORACLE A, the CPU event-driven restatement of the reference's
 * P2PNode gossip logic (no NS-3 socket stack, ideal hop delay = --Latency).
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so.  The product path (libgossip.so, gossip_sim)
 * never links or calls it.
 *
 * Parity status: UNPINNED against NS-3.  The reference ships no tests, fixtures or
 * golden logs, and cannot be built here (NS-3 is absent; a stub-header build is not
 * allowed).  The oracle is pinned only by known-answer tests of the libstdc++
 * primitives it shares with the reference (mt19937, generate_canonical,
 * uniform_real_distribution, std::hash<uint64_t>) and by the hand-derived small
 * cases in tests/.  See DESIGN.md "Oracle".
 */
#ifndef GOSSIP_ORACLE_H
#define GOSSIP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_sim oracle_sim;

/* Reference-mode parameters: p2pnetwork.cc:294-306 (CLI) + seeds that replace
 * std::random_device (p2pnetwork.cc:65, p2pnode.cc:41). */
typedef struct oracle_params {
    uint32_t num_nodes;        /* --numNodes        (default 10)  */
    double connection_prob;    /* --connectionProb  (default 0.3) */
    double sim_time_s;         /* --simTime         (default 60)  */
    double latency_ms;         /* --Latency         (default 5)   */
    uint32_t topo_seed;        /* replaces rd() at p2pnetwork.cc:66            */
    uint32_t node_seed;        /* replaces rd() at p2pnode.cc:41 (seed+id)     */
    uint32_t id_mask;          /* test knob: shareId &= id_mask (0 => no mask) */
    int64_t register_delay_ns; /* 0 = ideal: REGISTER handled at t=5 s         */
    int64_t est_delay_ns;      /* handshake model: shares a connector sends before
                                  t=5 s + est_delay are lost (0 = ideal)        */
} oracle_params;

/* Build topology + per-node RNGs literally as the reference does. */
int oracle_create_reference(const oracle_params* p, oracle_sim** out);

/* Replay mode: an external link list (key order (a,b), as in the std::map at
 * p2pnetwork.cc:30) and a list of COUNTED generation events (ns, node, shareId).
 * t_cut_ns = time of PrintStatistics; use INT64_MAX to run floods to completion. */
int oracle_create_replay(uint32_t num_nodes, int64_t latency_ns, int64_t t_start_ns,
                         int64_t t_cut_ns, uint64_t num_links, const uint32_t* link_a,
                         const uint32_t* link_b, uint64_t num_events, const int64_t* ev_ns,
                         const uint32_t* ev_node, const uint32_t* ev_id, oracle_sim** out);

/* Handshake model for either mode: shares sent before t_start +
 * est_delay_ns ride the REGISTER segment and are lost; REGISTER appends the acceptor-side
 * peer at t_start + register_delay_ns (before any other event of that ns).  Call before
 * oracle_run. */
int oracle_set_handshake(oracle_sim* s, int64_t est_delay_ns, int64_t register_delay_ns);

/* NS-3 link timing for either mode: a Send at time t is delivered at
 *     t + latency + send_defer_ns + (len(Share::ToString()) + header_bytes) * ns_per_byte
 * (TcpSocketBase's one-TimeStep SendPendingData deferral, then the PointToPoint device's
 * serialisation at the link DataRate, then the channel delay).  5 Mbps links
 * (p2pnetwork.cc:113): ns_per_byte = 1600, header_bytes = 54, send_defer_ns = 1.  Not
 * modelled: device queueing behind other segments and ACKs, and the coalescing of the two
 * sends to a duplicate peer into one segment.  Call before oracle_run. */
int oracle_set_link_timing(oracle_sim* s, int64_t ns_per_byte, uint32_t header_bytes,
                           int64_t send_defer_ns);

/* Record the NS_LOG_INFO lines of the gossip path (p2pnode.cc:88,110,122,143-144,160-161,
 * 184,191-192) in event order, each as "<t_ns>\t<line>\n" (small runs only).
 * oracle_get_log copies them into buf (NUL-terminated) and returns the full length. */
int oracle_enable_log(oracle_sim* s);
int64_t oracle_get_log(const oracle_sim* s, char* buf, uint64_t buf_len);

/* Enable the per-(node, shareId) first-contact trace (small runs only). */
int oracle_enable_trace(oracle_sim* s);

/* Run the discrete-event loop until PrintStatistics (t_cut) or the queue drains. */
int oracle_run(oracle_sim* s);

/* Per-node statistics as printed by PrintStatistics (p2pnetwork.cc:271-277). Any
 * pointer may be NULL. */
int oracle_get_stats(const oracle_sim* s, uint32_t* gen, uint32_t* recv, uint32_t* fwd,
                     uint64_t* sent, uint32_t* processed, uint32_t* peers, uint32_t* sockets);

/* Totals: edge events (= sum of sends), events processed, wall seconds of the event loop
 * after makeconnections. */
int oracle_get_counters(const oracle_sim* s, uint64_t* edge_events, uint64_t* events,
                        double* wall_s);

/* The link list built in reference mode (key order).  Call with NULL to get count. */
uint64_t oracle_get_links(const oracle_sim* s, uint32_t* a, uint32_t* b);

/* The counted generation events (ns, node, shareId), in execution order. */
uint64_t oracle_get_gen_events(const oracle_sim* s, int64_t* ns, uint32_t* node, uint32_t* id);

/* Periodic stats (p2pnetwork.cc:231-250): one record per stats time. */
uint64_t oracle_get_periodic(const oracle_sim* s, int64_t* t_ns, uint32_t* total_gen,
                             uint32_t* total_processed, uint32_t* total_sockets);

/* First-contact trace: one record per (node, shareId) inserted into processedShares
 * before t_cut: time, hop count (0 = own generation), via_recv (1 = ReceiveShare). */
uint64_t oracle_get_trace(const oracle_sim* s, uint32_t* node, uint32_t* id, int64_t* t_ns,
                          uint32_t* hop, uint8_t* via_recv);

/* Time conversions used by the oracle (ns-3 int64x64 exact rounding). */
int64_t oracle_seconds_to_ns(double s);
int64_t oracle_milliseconds_to_ns(double ms);

const char* oracle_last_error(void);
void oracle_destroy(oracle_sim* s);

/* ORACLE B (oracle_b.cpp): a bit-sliced, level-synchronous restatement of the same path for
 * schedules whose share ids are all distinct (each share is then an independent flood; ideal
 * hop).  Same link keys and counted-generation events as oracle_create_replay; arrivals count
 * iff t + hop * latency < t_cut_ns.  Multi-threaded (num_threads); for sizes ORACLE A's event
 * loop cannot reach.  Fails (-1, oracle_b_last_error) if two events share an id. */
int oracle_b_run(uint32_t n, int64_t latency_ns, int64_t t_cut_ns, uint64_t num_links,
                 const uint32_t* la, const uint32_t* lb, uint64_t num_events, const int64_t* ev_ns,
                 const uint32_t* ev_node, const uint32_t* ev_id, int num_threads, uint32_t* gen,
                 uint32_t* recv, uint32_t* fwd, uint64_t* sent, uint32_t* processed,
                 uint32_t* peers, uint32_t* sockets, uint64_t* edge_events);
const char* oracle_b_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
