// oracle.cpp -- ORACLE A: event-driven CPU restatement of the reference's gossip path.
//
// TEST INFRASTRUCTURE ONLY (see oracle.h).  Nothing in the product links this file.
//
// What it restates, literally and single-threaded like the NS-3 simulator:
//   * topology      CreateRandomTopology            p2pnetwork.cc:62-96  (+ConnectNodes :110-130)
//   * peer lists    makeconnections/ConnectPeerSockets p2pnetwork.cc:99-107,133-150,
//                   P2PNode::AddPeer p2pnode.cc:77-83, REGISTER branch p2pnode.cc:178-188
//   * node RNG      P2PNode::P2PNode               p2pnode.cc:33-43  (rd() -> node_seed)
//   * generation    ScheduleNextShare/GenerateAndGossipShare p2pnode.cc:97-125
//   * share id      GenerateUniqueShareId           p2pnode.cc:201-209
//   * hot path      GossipShareToPeers              p2pnode.cc:127-153
//                   HandleRead (seen-set check)      p2pnode.cc:167-199
//                   ReceiveShare                     p2pnode.cc:155-165
//   * reporting     PrintStatistics                  p2pnetwork.cc:253-285
//                   PrintPeriodicStats               p2pnetwork.cc:231-250
//   * run window    Start                            p2pnetwork.cc:193-218
//
// The NS-3 transport is replaced by an ideal hop: a Send at time t is delivered (HandleRead)
// at t + Latency.  Events at equal time run in scheduling order (NS-3's (ts, uid) order).
// Time conversion follows ns-3's int64x64 path: Seconds(x) = round-half-up(x * 1e9) computed
// exactly (not through a double product).  This is an assumption about the (unpinned) ns-3
// version; see DESIGN.md.
#include "oracle.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <queue>
#include <random>
#include <sstream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(const std::string& m) {
    g_err = m;
    return -1;
}

// ns-3 int64x64: Seconds(double) -> From(int64x64_t(value), S) -> Time(v.Round()).
// The double converts exactly into 64.64 fixed point; the product with 10^k is exact;
// Round() is half away from zero.
int64_t exact_scale_round(double x, uint64_t factor) {
    if (x == 0.0) return 0;
    const bool neg = x < 0;
    double ax = neg ? -x : x;
    int e2 = 0;
    double m = std::frexp(ax, &e2);                          // ax = m * 2^e2, m in [0.5,1)
    const uint64_t M = (uint64_t)std::ldexp(m, 53);           // exact 53-bit mantissa
    const int sh = e2 - 53;                                    // ax = M * 2^sh
    unsigned __int128 P = (unsigned __int128)M * factor;
    unsigned __int128 q;
    if (sh >= 0) {
        q = P << sh;
    } else {
        const int s = -sh;
        if (s >= 127) {
            q = 0;
        } else {
            q = P >> s;
            const unsigned __int128 rem = P - (q << s);
            const unsigned __int128 half = (unsigned __int128)1 << (s - 1);
            if (rem >= half) q += 1;
        }
    }
    int64_t r = (int64_t)q;
    return neg ? -r : r;
}

struct Share {
    uint32_t origin;
    uint32_t id;
    int64_t ts;
    int64_t hop_ns;  // delivery delay of every Send of this share
};

// Set of uint32 keys with the semantics of the reference's std::unordered_set<uint32_t>
// processedShares / the key set of std::unordered_map<uint32_t, Ptr<Socket>> peersockets
// (p2pnode.h:38-39): insert, find, size.  Open addressing in one allocation, so a 10M-node
// replay (C4) builds and frees its 20M sets in seconds instead of minutes.
class KeySet {
  public:
    // returns true if the key was not present
    bool insert(uint32_t k) {
        if (k == kEmpty) {
            const bool fresh = !has_empty_key_;
            has_empty_key_ = true;
            size_ += fresh;
            return fresh;
        }
        if ((used_ + 1) * 4 > slots_.size() * 3) rehash(slots_.empty() ? 8 : slots_.size() * 2);
        size_t i = hash(k) & (slots_.size() - 1);
        while (slots_[i] != kEmpty) {
            if (slots_[i] == k) return false;
            i = (i + 1) & (slots_.size() - 1);
        }
        slots_[i] = k;
        used_++;
        size_++;
        return true;
    }
    bool contains(uint32_t k) const {
        if (k == kEmpty) return has_empty_key_;
        if (slots_.empty()) return false;
        size_t i = hash(k) & (slots_.size() - 1);
        while (slots_[i] != kEmpty) {
            if (slots_[i] == k) return true;
            i = (i + 1) & (slots_.size() - 1);
        }
        return false;
    }
    size_t size() const { return size_; }
    void reserve(size_t k) {
        size_t cap = 8;
        while (cap * 3 < (k + 1) * 4) cap *= 2;
        if (cap > slots_.size()) rehash(cap);
    }
    void clear() {
        std::vector<uint32_t>().swap(slots_);
        used_ = size_ = 0;
        has_empty_key_ = false;
    }

  private:
    static constexpr uint32_t kEmpty = 0xffffffffu;
    static size_t hash(uint32_t k) { return (size_t)((k * 0x9E3779B1u) ^ (k >> 16)); }
    void rehash(size_t cap) {
        std::vector<uint32_t> old;
        old.swap(slots_);
        slots_.assign(cap, kEmpty);
        used_ = 0;
        for (uint32_t k : old)
            if (k != kEmpty) {
                size_t i = hash(k) & (cap - 1);
                while (slots_[i] != kEmpty) i = (i + 1) & (cap - 1);
                slots_[i] = k;
                used_++;
            }
    }
    std::vector<uint32_t> slots_;
    size_t used_ = 0, size_ = 0;
    bool has_empty_key_ = false;
};

struct Node {
    uint32_t id = 0;
    std::vector<uint32_t> peers;                  // p2pnode.h:32
    KeySet peersockets;                           // p2pnode.h:39 (keys only)
    KeySet processed;                             // p2pnode.h:38
    bool running = false;                         // p2pnode.h:36
    uint32_t sent = 0, recv = 0, gen = 0, fwd = 0;  // p2pnode.h:40-43
    uint64_t sent64 = 0;
};

enum EvType : uint32_t { EV_CONNECT, EV_GEN, EV_ARRIVE, EV_REGISTER, EV_PERIODIC, EV_STATS };

struct Event {
    int64_t t;
    uint64_t seq;
    uint32_t type;
    uint32_t node;
    uint32_t arg;  // share index (ARRIVE), peer id (REGISTER), replay-event index (GEN)
    uint32_t hop;
};
struct EvLater {
    bool operator()(const Event& a, const Event& b) const {
        if (a.t != b.t) return a.t > b.t;
        // a REGISTER runs before any other event of its nanosecond (handshake model only)
        const int pa = a.type == EV_REGISTER ? 0 : 1, pb = b.type == EV_REGISTER ? 0 : 1;
        return pa != pb ? pa > pb : a.seq > b.seq;
    }
};

struct TraceRec {
    uint32_t node, id;
    int64_t t;
    uint32_t hop;
    uint8_t via_recv;
};

}  // namespace

struct oracle_sim {
    bool replay = false;
    uint32_t n = 0;
    int64_t L = 0;            // hop delay (ns)
    int64_t t_start = 0;      // makeconnections time (5 s)
    int64_t t_cut = 0;        // PrintStatistics time (simTime - 0.1)
    int64_t register_delay = 0;
    int64_t est_delay = 0;    // handshake model: connector sends before t_start+est are lost
    bool link_timing = false; // serialisation model (oracle_set_link_timing)
    int64_t link_npb = 0, link_defer = 0;
    uint32_t link_hdr = 0;
    uint32_t id_mask = 0;
    std::vector<Node> nodes;
    std::vector<std::mt19937> rngs;  // p2pnode.h:34 (reference mode only)
    // Keys of the `connections` map (p2pnetwork.cc:30) in map order: reference mode builds the
    // std::map literally and flattens it; replay mode sorts and de-duplicates the given keys.
    std::vector<std::pair<uint32_t, uint32_t>> links;
    std::vector<Share> shares;
    std::priority_queue<Event, std::vector<Event>, EvLater> q;
    uint64_t seq = 0;
    // replay inputs
    std::vector<int64_t> rp_ns;
    std::vector<uint32_t> rp_node, rp_id;
    // outputs
    std::vector<int64_t> gen_ns;
    std::vector<uint32_t> gen_node, gen_id;
    std::vector<int64_t> per_t;
    std::vector<uint32_t> per_gen, per_proc, per_sock;
    bool trace = false;
    std::vector<TraceRec> tr;
    bool log = false;
    std::string lg;  // "<t_ns>\t<NS_LOG_INFO line>\n" in event order
    // snapshot at PrintStatistics
    bool have_stats = false;
    std::vector<uint32_t> s_gen, s_recv, s_fwd, s_proc, s_peers, s_sock;
    std::vector<uint64_t> s_sent;
    uint64_t edge_events = 0, events = 0;
    double wall = 0.0;

    template <class F>
    void log_line(int64_t t, F&& body) {
        if (!log) return;
        std::ostringstream os;
        os << t << '\t';
        body(os);
        os << '\n';
        lg += os.str();
    }

    void schedule(int64_t t, uint32_t type, uint32_t node, uint32_t arg, uint32_t hop) {
        q.push(Event{t, seq++, type, node, arg, hop});
    }

    // P2PNode::AddPeer (p2pnode.cc:77-83): de-duplicated.
    static void add_peer(Node& nd, uint32_t peer) {
        if (std::find(nd.peers.begin(), nd.peers.end(), peer) == nd.peers.end())
            nd.peers.push_back(peer);
    }

    // ScheduleNextShare (p2pnode.cc:97-104): U(2,5) s via libstdc++ generate_canonical.
    void schedule_next_share(Node& nd, int64_t now) {
        std::uniform_real_distribution<double> dist(2.0, 5.0);
        const double next = dist(rngs[nd.id]);
        schedule(now + exact_scale_round(next, 1000000000ull), EV_GEN, nd.id, 0, 0);
    }

    // GenerateUniqueShareId (p2pnode.cc:201-209); std::hash<uint64_t> is the identity.
    uint32_t unique_share_id(const Node& nd, int64_t now) const {
        const uint64_t seed = (uint64_t)nd.id * 1000000ull + (uint64_t)nd.gen * 1000ull +
                              (uint64_t)(now % 1000);
        uint32_t id = (uint32_t)std::hash<uint64_t>{}(seed);
        if (id_mask) id &= id_mask;
        return id;
    }

    // GossipShareToPeers (p2pnode.cc:127-153).  Send never fails at these loads.
    // Handshake model: before t_start + est_delay only connector-side peers exist and their
    // sockets are not ESTABLISHED; the share is buffered behind "REGISTER:", which HandleRead
    // parses as a registration only (p2pnode.cc:178): counted as sent, never delivered.
    void gossip(Node& nd, uint32_t share_idx, int64_t now, uint32_t hop) {
        const bool lost = est_delay != 0 && now < t_start + est_delay;
        for (uint32_t peer : nd.peers) {
            if (!nd.peersockets.contains(peer)) continue;  // :131-135
            nd.sent++;
            nd.sent64++;
            edge_events++;
            const Share& sh = shares[share_idx];
            log_line(now, [&](std::ostream& os) {  // :143-144
                os << "Node " << nd.id << " sending share " << sh.origin << ":" << sh.id
                   << " to peer " << peer;
            });
            if (!lost) schedule(now + shares[share_idx].hop_ns, EV_ARRIVE, peer, share_idx, hop + 1);
        }
    }

    void record(uint32_t node, uint32_t id, int64_t t, uint32_t hop, uint8_t via) {
        if (trace) tr.push_back(TraceRec{node, id, t, hop, via});
    }

    // GenerateAndGossipShare (p2pnode.cc:106-125).
    void on_gen(const Event& e) {
        Node& nd = nodes[e.node];
        if (nd.peers.empty()) {                  // :108-113
            log_line(e.t, [&](std::ostream& os) { os << "Node " << nd.id << " has no peers to send shares to"; });
            if (!replay) schedule_next_share(nd, e.t);
            return;
        }
        if (!nd.running) return;                 // :114
        Share sh;
        sh.origin = nd.id;
        sh.id = replay ? rp_id[e.arg] : unique_share_id(nd, e.t);
        nd.gen++;
        sh.ts = e.t;
        sh.hop_ns = L;
        if (link_timing) {
            // Share::ToString (p2pnode.cc:6-11) with timestamp = Now().GetSeconds() (:119); a
            // receiver re-serialises the parsed fields (:177,138), so every hop carries this string
            std::ostringstream ss;
            ss << "SHARE:" << sh.origin << ":" << sh.id << ":" << (double)e.t / 1e9;
            sh.hop_ns += link_defer + ((int64_t)ss.str().size() + link_hdr) * link_npb;
        }
        const bool was_seen = !nd.processed.insert(sh.id);
        shares.push_back(sh);
        gen_ns.push_back(e.t);
        gen_node.push_back(nd.id);
        gen_id.push_back(sh.id);
        if (!was_seen) record(nd.id, sh.id, e.t, 0, 0);
        log_line(e.t, [&](std::ostream& os) { os << "Node " << nd.id << " generating new share " << sh.id; });  // :122
        gossip(nd, (uint32_t)(shares.size() - 1), e.t, 0);
        if (!replay) schedule_next_share(nd, e.t);
    }

    // HandleRead (p2pnode.cc:167-199) for one SHARE message, then ReceiveShare (:155-165).
    void on_arrive(const Event& e) {
        Node& nd = nodes[e.node];
        const Share& sh = shares[e.arg];
        if (nd.processed.contains(sh.id)) {                           // :189-193 duplicate
            log_line(e.t, [&](std::ostream& os) {
                os << "Node " << nd.id << " already processed share " << sh.origin << ":" << sh.id;
            });
            return;
        }
        nd.recv++;                                                   // ReceiveShare :157
        nd.processed.insert(sh.id);                                  // :158
        nd.fwd++;                                                    // :163
        record(nd.id, sh.id, e.t, e.hop, 1);
        log_line(e.t, [&](std::ostream& os) {  // :160-161, timestamp streamed as a double
            os << "Node " << nd.id << " received new share " << sh.origin << ":" << sh.id << ":"
               << (double)sh.ts / 1e9 << " from origin " << sh.origin;
        });
        gossip(nd, e.arg, e.t, e.hop);                               // :164
    }

    // makeconnections (p2pnetwork.cc:99-107) -> ConnectPeerSockets (:133-150).
    void on_connect(const Event& e) {
        {   // capacity only (a 10M-node replay): no effect on the sets' contents
            std::vector<uint32_t> cnt(n, 0);
            for (const auto& kv : links) {
                cnt[kv.first]++;
                cnt[kv.second]++;
            }
            for (uint32_t v = 0; v < n; v++) {
                nodes[v].peers.reserve(cnt[v]);
                nodes[v].peersockets.reserve(cnt[v]);
            }
        }
        for (const auto& kv : links) {
            const uint32_t i = kv.first, j = kv.second;
            nodes[i].peersockets.insert(j);  // AddPeerSocket :144
            log_line(e.t, [&](std::ostream& os) { os << "Node " << i << " added socket connection to peer " << j; });  // p2pnode.cc:88
            add_peer(nodes[i], j);           // AddPeer :145
            if (register_delay != 0) schedule(e.t + register_delay, EV_REGISTER, j, i, 0);
        }
        // "REGISTER:i" reaches node j in a later event (after every AddPeer of this loop has
        // run); HandleRead :178-188 then appends i WITHOUT de-duplication.  The ideal model
        // delivers them at t = 5 s, still after the whole makeconnections loop.
        if (register_delay == 0)
            for (const auto& kv : links) {
                const uint32_t i = kv.first, j = kv.second;
                nodes[j].peersockets.insert(i);
                nodes[j].peers.push_back(i);
                log_line(e.t, [&](std::ostream& os) { os << "Node " << j << " received registration from peer " << i; });  // p2pnode.cc:184
            }
    }

    void on_register(const Event& e) {
        log_line(e.t, [&](std::ostream& os) { os << "Node " << e.node << " received registration from peer " << e.arg; });
        nodes[e.node].peersockets.insert(e.arg);
        nodes[e.node].peers.push_back(e.arg);
    }

    // PrintPeriodicStats (p2pnetwork.cc:231-250): uint32 accumulators.
    void on_periodic(const Event& e) {
        uint32_t total_shares = 0, total_gen = 0, total_sock = 0;
        for (const Node& nd : nodes) {
            total_shares += (uint32_t)nd.processed.size();
            total_gen += nd.gen;
            total_sock += (uint32_t)nd.peersockets.size();
        }
        per_t.push_back(e.t);
        per_gen.push_back(total_gen);
        per_proc.push_back(total_shares);
        per_sock.push_back(total_sock);
    }

    void on_stats() {
        have_stats = true;
        s_gen.resize(n); s_recv.resize(n); s_fwd.resize(n); s_proc.resize(n);
        s_peers.resize(n); s_sock.resize(n); s_sent.resize(n);
        for (uint32_t i = 0; i < n; i++) {
            const Node& nd = nodes[i];
            s_gen[i] = nd.gen; s_recv[i] = nd.recv; s_fwd[i] = nd.fwd;
            s_sent[i] = nd.sent64; s_proc[i] = (uint32_t)nd.processed.size();
            s_peers[i] = (uint32_t)nd.peers.size(); s_sock[i] = (uint32_t)nd.peersockets.size();
        }
    }
};

extern "C" {

int64_t oracle_seconds_to_ns(double s) { return exact_scale_round(s, 1000000000ull); }
int64_t oracle_milliseconds_to_ns(double ms) { return exact_scale_round(ms, 1000000ull); }

const char* oracle_last_error(void) { return g_err.c_str(); }

int oracle_create_reference(const oracle_params* p, oracle_sim** out) {
    if (!p || !out) return fail("null argument");
    if (p->num_nodes < 2)
        return fail("numNodes < 2: the reference indexes nodes.Get(1) (p2pnetwork.cc:82)");
    if (!(p->sim_time_s > 0.1)) return fail("simTime must exceed 0.1 s (p2pnetwork.cc:206)");
    auto s = std::make_unique<oracle_sim>();
    s->n = p->num_nodes;
    s->L = exact_scale_round(p->latency_ms, 1000000ull);     // MilliSeconds(latencyMs) :114
    s->t_start = exact_scale_round(5.0, 1000000000ull);      // Seconds(5) :93
    s->t_cut = exact_scale_round(p->sim_time_s - 0.1, 1000000000ull);  // :206
    s->register_delay = p->register_delay_ns;
    s->est_delay = p->est_delay_ns;
    s->id_mask = p->id_mask;
    s->nodes.resize(s->n);
    s->rngs.resize(s->n);
    // P2PNode::P2PNode (p2pnode.cc:33-43): rng.seed(rd() + id).
    for (uint32_t i = 0; i < s->n; i++) {
        s->nodes[i].id = i;
        s->rngs[i].seed((uint32_t)(p->node_seed + i));
    }
    // CreateRandomTopology (p2pnetwork.cc:62-96); ConnectNodes (:110-130) keys the map.
    {
        std::map<std::pair<uint32_t, uint32_t>, int> connections;  // p2pnetwork.cc:30
        std::mt19937 rng(p->topo_seed);
        std::uniform_real_distribution<double> dist(0.0, 1.0);
        const uint32_t n = s->n;
        for (uint32_t i = 0; i < n; i++) {
            bool connected = false;
            for (uint32_t j = i + 1; j < n; j++) {
                if (dist(rng) < p->connection_prob) {
                    connected = true;
                    connections[std::make_pair(i, j)] = 1;
                }
            }
            if (!connected) {
                if (i == 0) connections[std::make_pair(0u, 1u)] = 1;
                else connections[std::make_pair(i, i - 1)] = 1;
            }
        }
        s->links.reserve(connections.size());
        for (const auto& kv : connections) s->links.push_back(kv.first);
    }
    // Event order mirrors the uids the reference hands out: makeconnections is scheduled
    // in CreateRandomTopology (:93), then Start() schedules the first share of every node
    // (:196-199), the periodic stats (:201-204), then PrintStatistics (:206).
    s->schedule(s->t_start, EV_CONNECT, 0, 0, 0);
    for (auto& nd : s->nodes) {
        nd.running = true;                     // StartGeneratingShares p2pnode.cc:91-95
        s->schedule_next_share(nd, 0);
    }
    for (double t = 10.0; t < p->sim_time_s; t += 10.0)
        s->schedule(exact_scale_round(t, 1000000000ull), EV_PERIODIC, 0, 0, 0);
    s->schedule(s->t_cut, EV_STATS, 0, 0, 0);
    *out = s.release();
    return 0;
}

int oracle_create_replay(uint32_t num_nodes, int64_t latency_ns, int64_t t_start_ns,
                         int64_t t_cut_ns, uint64_t num_links, const uint32_t* link_a,
                         const uint32_t* link_b, uint64_t num_events, const int64_t* ev_ns,
                         const uint32_t* ev_node, const uint32_t* ev_id, oracle_sim** out) {
    if (!out) return fail("null argument");
    if (num_nodes < 1) return fail("num_nodes must be >= 1");
    if (latency_ns <= 0) return fail("latency must be positive");
    auto s = std::make_unique<oracle_sim>();
    s->replay = true;
    s->n = num_nodes;
    s->L = latency_ns;
    s->t_start = t_start_ns;
    s->t_cut = t_cut_ns;
    s->nodes.resize(num_nodes);
    for (uint32_t i = 0; i < num_nodes; i++) {
        s->nodes[i].id = i;
        s->nodes[i].running = true;
    }
    s->links.resize(num_links);
    for (uint64_t k = 0; k < num_links; k++) {
        if (link_a[k] >= num_nodes || link_b[k] >= num_nodes) return fail("link out of range");
        s->links[k] = std::make_pair(link_a[k], link_b[k]);
    }
    // std::map semantics: ordered keys, a repeated key is one entry (p2pnetwork.cc:129).
    std::sort(s->links.begin(), s->links.end());
    s->links.erase(std::unique(s->links.begin(), s->links.end()), s->links.end());
    s->rp_ns.assign(ev_ns, ev_ns + num_events);
    s->rp_node.assign(ev_node, ev_node + num_events);
    s->rp_id.assign(ev_id, ev_id + num_events);
    s->schedule(s->t_start, EV_CONNECT, 0, 0, 0);
    // Replay events carry the uids of generation events: earlier than any arrival.
    std::vector<uint64_t> order(num_events);
    for (uint64_t k = 0; k < num_events; k++) order[k] = k;
    std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) {
        return s->rp_ns[a] != s->rp_ns[b] ? s->rp_ns[a] < s->rp_ns[b]
                                          : s->rp_node[a] < s->rp_node[b];
    });
    for (uint64_t k : order) {
        if (s->rp_node[k] >= num_nodes) return fail("event node out of range");
        if (s->rp_ns[k] < t_start_ns) return fail("replay event before t_start");
        s->schedule(s->rp_ns[k], EV_GEN, s->rp_node[k], (uint32_t)k, 0);
    }
    if (t_cut_ns != std::numeric_limits<int64_t>::max())
        s->schedule(t_cut_ns, EV_STATS, 0, 0, 0);
    *out = s.release();
    return 0;
}

int oracle_set_handshake(oracle_sim* s, int64_t est_delay_ns, int64_t register_delay_ns) {
    if (!s) return fail("null sim");
    if (est_delay_ns < 0 || register_delay_ns < 0) return fail("negative delay");
    if (s->events) return fail("set the handshake model before oracle_run");
    s->est_delay = est_delay_ns;
    s->register_delay = register_delay_ns;
    return 0;
}

int oracle_set_link_timing(oracle_sim* s, int64_t ns_per_byte, uint32_t header_bytes,
                           int64_t send_defer_ns) {
    if (!s) return fail("null sim");
    if (ns_per_byte < 0 || send_defer_ns < 0) return fail("negative link timing");
    if (s->events) return fail("set link timing before oracle_run");
    s->link_timing = true;
    s->link_npb = ns_per_byte;
    s->link_hdr = header_bytes;
    s->link_defer = send_defer_ns;
    return 0;
}

int oracle_enable_log(oracle_sim* s) {
    if (!s) return fail("null sim");
    s->log = true;
    return 0;
}

int64_t oracle_get_log(const oracle_sim* s, char* buf, uint64_t buf_len) {
    if (!s) return fail("null sim");
    if (buf && buf_len) {
        const uint64_t k = std::min<uint64_t>(s->lg.size(), buf_len - 1);
        std::memcpy(buf, s->lg.data(), k);
        buf[k] = 0;
    }
    return (int64_t)s->lg.size();
}

int oracle_enable_trace(oracle_sim* s) {
    if (!s) return fail("null sim");
    s->trace = true;
    return 0;
}

int oracle_run(oracle_sim* s) {
    if (!s) return fail("null sim");
    auto t0 = std::chrono::steady_clock::now();
    while (!s->q.empty()) {
        const Event e = s->q.top();
        s->q.pop();
        s->events++;
        switch (e.type) {
            case EV_CONNECT:
                s->on_connect(e);
                t0 = std::chrono::steady_clock::now();  // time the gossip, not the peer setup
                break;
            case EV_GEN: s->on_gen(e); break;
            case EV_ARRIVE: s->on_arrive(e); break;
            case EV_REGISTER: s->on_register(e); break;
            case EV_PERIODIC: s->on_periodic(e); break;
            case EV_STATS: break;
        }
        if (e.type == EV_STATS) {
            // StopAllNodes (same time, scheduled after PrintStatistics) stops generation and
            // closes every socket (p2pnode.cc:55-69: peersockets.clear()).  Only periodic
            // stats scheduled in (t_cut, simTime) can still print; they see the counters
            // frozen at t_cut and zero socket connections (arrivals at closed sockets are
            // not delivered to HandleRead).
            s->on_stats();
            s->wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            while (!s->q.empty()) {
                const Event r = s->q.top();
                s->q.pop();
                if (r.type != EV_PERIODIC) continue;
                uint32_t tg = 0, tp = 0;
                for (const Node& nd : s->nodes) {
                    tg += nd.gen;
                    tp += (uint32_t)nd.processed.size();
                }
                s->per_t.push_back(r.t);
                s->per_gen.push_back(tg);
                s->per_proc.push_back(tp);
                s->per_sock.push_back(0);
            }
            break;
        }
    }
    if (!s->have_stats) {
        s->on_stats();
        s->wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    return 0;
}

int oracle_get_stats(const oracle_sim* s, uint32_t* gen, uint32_t* recv, uint32_t* fwd,
                     uint64_t* sent, uint32_t* processed, uint32_t* peers, uint32_t* sockets) {
    if (!s || !s->have_stats) return fail("no stats: run first");
    const size_t n = s->n;
    if (gen) std::memcpy(gen, s->s_gen.data(), n * 4);
    if (recv) std::memcpy(recv, s->s_recv.data(), n * 4);
    if (fwd) std::memcpy(fwd, s->s_fwd.data(), n * 4);
    if (sent) std::memcpy(sent, s->s_sent.data(), n * 8);
    if (processed) std::memcpy(processed, s->s_proc.data(), n * 4);
    if (peers) std::memcpy(peers, s->s_peers.data(), n * 4);
    if (sockets) std::memcpy(sockets, s->s_sock.data(), n * 4);
    return 0;
}

int oracle_get_counters(const oracle_sim* s, uint64_t* edge_events, uint64_t* events,
                        double* wall_s) {
    if (!s) return fail("null sim");
    if (edge_events) *edge_events = s->edge_events;
    if (events) *events = s->events;
    if (wall_s) *wall_s = s->wall;
    return 0;
}

uint64_t oracle_get_links(const oracle_sim* s, uint32_t* a, uint32_t* b) {
    if (!s) return 0;
    uint64_t k = 0;
    for (const auto& kv : s->links) {
        if (a) a[k] = kv.first;
        if (b) b[k] = kv.second;
        k++;
    }
    return k;
}

uint64_t oracle_get_gen_events(const oracle_sim* s, int64_t* ns, uint32_t* node, uint32_t* id) {
    if (!s) return 0;
    const uint64_t m = s->gen_ns.size();
    for (uint64_t k = 0; k < m; k++) {
        if (ns) ns[k] = s->gen_ns[k];
        if (node) node[k] = s->gen_node[k];
        if (id) id[k] = s->gen_id[k];
    }
    return m;
}

uint64_t oracle_get_periodic(const oracle_sim* s, int64_t* t_ns, uint32_t* total_gen,
                             uint32_t* total_processed, uint32_t* total_sockets) {
    if (!s) return 0;
    const uint64_t m = s->per_t.size();
    for (uint64_t k = 0; k < m; k++) {
        if (t_ns) t_ns[k] = s->per_t[k];
        if (total_gen) total_gen[k] = s->per_gen[k];
        if (total_processed) total_processed[k] = s->per_proc[k];
        if (total_sockets) total_sockets[k] = s->per_sock[k];
    }
    return m;
}

uint64_t oracle_get_trace(const oracle_sim* s, uint32_t* node, uint32_t* id, int64_t* t_ns,
                          uint32_t* hop, uint8_t* via_recv) {
    if (!s) return 0;
    const uint64_t m = s->tr.size();
    for (uint64_t k = 0; k < m; k++) {
        const TraceRec& r = s->tr[k];
        if (node) node[k] = r.node;
        if (id) id[k] = r.id;
        if (t_ns) t_ns[k] = r.t;
        if (hop) hop[k] = r.hop;
        if (via_recv) via_recv[k] = r.via_recv;
    }
    return m;
}

void oracle_destroy(oracle_sim* s) { delete s; }

}  // extern "C"
