// eventlog.cpp -- the reference's per-event NS_LOG_INFO stream, rendered from a run's
// first-contact trace.
//
// The engine never moves individual messages: a tick ORs whole frontier rows.  Every
// NS_LOG_INFO line of the gossip path is still determined by what the trace holds -- who first
// saw which share, at which hop -- plus the peer lists:
//
//   GenerateAndGossipShare  "Node u generating new share ID"                p2pnode.cc:122
//   GossipShareToPeers      "Node u sending share O:ID to peer p", per entry  p2pnode.cc:143-144
//   ReceiveShare            "Node v received new share O:ID:TS from origin O" p2pnode.cc:160-161
//   HandleRead, duplicate   "Node v already processed share O:ID"            p2pnode.cc:191-192
//   HandleRead, REGISTER    "Node b received registration from peer a"       p2pnode.cc:184
//   AddPeerSocket           "Node a added socket connection to peer b"       p2pnode.cc:88
//
// A node that first sees a share at time t emits one message per entry of peers(node) (sender
// and duplicates included, p2pnode.cc:129), each arriving one hop delay later.  Of the k
// messages that reach v at its first-contact time, one is the "received new share" (its
// sender does not appear in the line), the other k-1 and every later one are "already
// processed".  Lines sharing a nanosecond are written in a canonical order (node, then
// first-contact block before duplicates, then share): NS-3 orders them by TCP event
// scheduling, which the reference does not pin.
//
// The window is the engine's: events at t_start <= t < t_cut (PrintStatistics runs first at
// t_cut, p2pnetwork.cc:206).  Not rendered: lines of the NS-3 socket layer that carry an IP
// address (HandleAccept, p2pnode.cc:73) and the "has no peers" lines of generations before
// t_start (p2pnode.cc:110), which are not in a counted schedule.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.h"

using namespace gossip;

namespace {

enum Kind : uint8_t { K_SOCKET = 0, K_REGISTER = 1, K_NOPEERS = 2, K_GEN = 3, K_RECV = 4, K_DUP = 5 };

struct Rec {
    int64_t t;
    uint32_t node;
    uint8_t kind;
    uint32_t arg;  // share index (GEN/RECV/DUP/NOPEERS: event index), peer (SOCKET/REGISTER)
};

}  // namespace

extern "C" int64_t gossip_format_event_log(const gossip_topology* t, uint64_t m,
                                           const gossip_gen_event* ev, uint64_t nt,
                                           const uint32_t* tr_node, const uint32_t* tr_id,
                                           const uint32_t* tr_hop, const uint8_t* tr_via,
                                           int64_t latency_ns, int64_t t_start_ns,
                                           int64_t t_cut_ns, int64_t ns_per_byte,
                                           uint32_t header_bytes, int64_t send_defer_ns,
                                           int with_time, char* buf, uint64_t buf_len) {
    if (!t || (m && !ev) || (nt && (!tr_node || !tr_id || !tr_hop || !tr_via)))
        return set_error(GOSSIP_EINVAL, "NULL argument");
    if (latency_ns <= 0) return set_error(GOSSIP_EINVAL, "latency must be positive");
    try {
        const uint32_t n = t->n;
        // peers(v) in the reference's order: connector-side AddPeer in map-key order at
        // makeconnections (p2pnetwork.cc:101-106, 144-145), then the REGISTER appends in the
        // order the keys sent them (p2pnode.cc:185-186, not de-duplicated).
        std::vector<std::vector<uint32_t>> peers(n);
        for (size_t k = 0; k < t->la.size(); k++) {
            auto& p = peers[t->la[k]];
            if (std::find(p.begin(), p.end(), t->lb[k]) == p.end()) p.push_back(t->lb[k]);
        }
        for (size_t k = 0; k < t->la.size(); k++) peers[t->lb[k]].push_back(t->la[k]);

        // share id -> event (unique ids: the trace names shares by id only)
        std::unordered_map<uint32_t, uint32_t> by_id;
        by_id.reserve(m * 2 + 1);
        for (uint64_t k = 0; k < m; k++) {
            if (ev[k].node >= n) return set_error(GOSSIP_EINVAL, "event node out of range");
            if (!by_id.emplace(ev[k].share_id, (uint32_t)k).second)
                return set_error(GOSSIP_EINVAL, "event log needs unique share ids (n <= 128,849)");
        }
        std::vector<int64_t> hop_ns(m, latency_ns);
        if (ns_per_byte || send_defer_ns)
            for (uint64_t k = 0; k < m; k++)
                hop_ns[k] += send_defer_ns +
                             ((int64_t)gossip_share_message_length(ev[k].node, ev[k].share_id, ev[k].ns) +
                              header_bytes) * ns_per_byte;

        std::vector<Rec> recs;
        if (t_start_ns < t_cut_ns)
            for (size_t k = 0; k < t->la.size(); k++) {
                recs.push_back(Rec{t_start_ns, t->la[k], K_SOCKET, t->lb[k]});
                recs.push_back(Rec{t_start_ns, t->lb[k], K_REGISTER, t->la[k]});
            }
        for (uint64_t k = 0; k < m; k++)
            if (peers[ev[k].node].empty() && ev[k].ns >= t_start_ns && ev[k].ns < t_cut_ns)
                recs.push_back(Rec{ev[k].ns, ev[k].node, K_NOPEERS, (uint32_t)k});
        // first contacts: (node, share) -> time; "claimed" once its first message is matched
        std::unordered_map<uint64_t, int64_t> first;
        first.reserve(nt * 2 + 1);
        std::vector<std::pair<uint32_t, uint32_t>> contacts;  // (node, share), trace order
        contacts.reserve(nt);
        for (uint64_t i = 0; i < nt; i++) {
            const auto it = by_id.find(tr_id[i]);
            if (it == by_id.end()) return set_error(GOSSIP_EINVAL, "trace names an unknown share id");
            const uint32_t s = it->second;
            if (tr_node[i] >= n) return set_error(GOSSIP_EINVAL, "trace node out of range");
            const int64_t tv = ev[s].ns + (int64_t)tr_hop[i] * hop_ns[s];
            if (tv >= t_cut_ns) continue;
            first[(uint64_t)tr_node[i] << 32 | s] = tr_via[i] ? tv : -1 - tv;  // <0: own generation
            recs.push_back(Rec{tv, tr_node[i], tr_via[i] ? K_RECV : K_GEN, s});
            contacts.emplace_back(tr_node[i], s);
        }
        std::unordered_map<uint64_t, uint32_t> claimed;
        for (const auto& c : contacts) {
            const uint32_t u = c.first, s = c.second;
            const int64_t fu = first[(uint64_t)u << 32 | s];
            const int64_t ta = (fu < 0 ? -1 - fu : fu) + hop_ns[s];
            if (ta >= t_cut_ns) continue;
            for (uint32_t p : peers[u]) {
                const uint64_t key = (uint64_t)p << 32 | s;
                const auto f = first.find(key);
                if (f != first.end() && f->second == ta && !claimed[key]++) continue;  // the "new" one
                recs.push_back(Rec{ta, p, K_DUP, s});
            }
        }
        std::stable_sort(recs.begin(), recs.end(), [](const Rec& a, const Rec& b) {
            if (a.t != b.t) return a.t < b.t;
            if (a.node != b.node) return a.node < b.node;
            if (a.kind != b.kind) return a.kind < b.kind;
            return a.arg < b.arg;
        });

        std::ostringstream os;
        auto stamp = [&](int64_t tt) {
            if (with_time) os << tt << '\t';
        };
        auto sends = [&](const Rec& r) {
            const gossip_gen_event& e = ev[r.arg];
            for (uint32_t p : peers[r.node]) {
                stamp(r.t);
                os << "Node " << r.node << " sending share " << e.node << ":" << e.share_id
                   << " to peer " << p << "\n";
            }
        };
        for (const Rec& r : recs) {
            stamp(r.t);
            switch (r.kind) {
            case K_SOCKET:
                os << "Node " << r.node << " added socket connection to peer " << r.arg << "\n";
                break;
            case K_REGISTER:
                os << "Node " << r.node << " received registration from peer " << r.arg << "\n";
                break;
            case K_NOPEERS:
                os << "Node " << r.node << " has no peers to send shares to\n";
                break;
            case K_GEN:
                os << "Node " << r.node << " generating new share " << ev[r.arg].share_id << "\n";
                sends(r);
                break;
            case K_RECV: {
                const gossip_gen_event& e = ev[r.arg];
                // Share::timestamp streamed as a double (p2pnode.cc:119,161)
                os << "Node " << r.node << " received new share " << e.node << ":" << e.share_id
                   << ":" << (double)e.ns / 1e9 << " from origin " << e.node << "\n";
                sends(r);
                break;
            }
            default:
                os << "Node " << r.node << " already processed share " << ev[r.arg].node << ":"
                   << ev[r.arg].share_id << "\n";
            }
        }
        const std::string s = os.str();
        if (buf && buf_len) {
            const uint64_t k = std::min<uint64_t>(s.size(), buf_len - 1);
            std::memcpy(buf, s.data(), k);
            buf[k] = 0;
        }
        return (int64_t)s.size();
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
}

// NetAnim XML (SetupNetAnim, p2pnetwork.cc:153-190), with the packet records that
// EnablePacketMetadata(true) (:187) asks for.  Topology part: nodes on a ceil(sqrt(n)) grid 100
// units apart, "Node i" descriptions, colours by |peers| when SetupNetAnim runs -- Start() calls it
// before makeconnections, so every node still has 0 peers and is blue (the reference's own
// behaviour) -- and one link per connection key.  Packet part (packets != 0): one <p> record per
// gossip Send (p2pnode.cc:140), from the first-contact trace exactly as the event log derives its
// "sending share" lines: first byte on the wire fbTx = first contact + send deferral, last byte
// lbTx = fbTx + (len(message) + header bytes) x ns_per_byte, fbRx / lbRx = + latency, times in
// seconds; meta-info = the application payload Share::ToString() (p2pnode.cc:6-11).  Not recorded:
// the TCP handshake, ACKs and REGISTER segments.  Element layout after ns-3's AnimationInterface;
// no NS-3 run is available to pin the exact attribute formatting (visual parity).
extern "C" int64_t gossip_format_netanim(const gossip_topology* t, uint64_t m, const gossip_gen_event* ev,
                                         uint64_t nt, const uint32_t* tr_node, const uint32_t* tr_id,
                                         const uint32_t* tr_hop, int64_t latency_ns, int64_t t_cut_ns,
                                         int64_t ns_per_byte, uint32_t header_bytes, int64_t send_defer_ns,
                                         int packets, char* buf, uint64_t buf_len) {
    if (!t || (m && !ev) || (nt && (!tr_node || !tr_id || !tr_hop))) return set_error(GOSSIP_EINVAL, "NULL argument");
    if (latency_ns <= 0) return set_error(GOSSIP_EINVAL, "latency must be positive");
    try {
        const uint32_t n = t->n;
        std::ostringstream os;
        const uint32_t grid = (uint32_t)std::ceil(std::sqrt((double)n));
        const uint32_t rows = grid ? (n + grid - 1) / grid : 0;
        os << "<anim ver=\"netanim-3.108\" filetype=\"animation\" >\n";
        os << "<topology minX = \"0\" minY = \"0\" maxX = \"" << (grid ? 100u * (grid - 1) : 0u)
           << "\" maxY = \"" << (rows ? 100u * (rows - 1) : 0u) << "\">\n";
        for (uint32_t i = 0; i < n; i++)
            os << "<node id=\"" << i << "\" sysId=\"0\" locX=\"" << 100u * (i % grid) << "\" locY=\""
               << 100u * (i / grid) << "\" />\n";
        for (uint32_t i = 0; i < n; i++) {
            os << "<nu p=\"c\" t=\"0\" id=\"" << i << "\" r=\"0\" g=\"0\" b=\"255\" />\n";
            os << "<nu p=\"d\" t=\"0\" id=\"" << i << "\" descr=\"Node " << i << "\" />\n";
        }
        for (size_t k = 0; k < t->la.size(); k++)
            os << "<link fromId=\"" << t->la[k] << "\" toId=\"" << t->lb[k] << "\" fd=\"\" td=\"\" ld=\"\" />\n";
        os << "</topology>\n";
        if (packets && nt) {
            std::vector<std::vector<uint32_t>> peers(n);  // the reference's order (see above)
            for (size_t k = 0; k < t->la.size(); k++) {
                auto& p = peers[t->la[k]];
                if (std::find(p.begin(), p.end(), t->lb[k]) == p.end()) p.push_back(t->lb[k]);
            }
            for (size_t k = 0; k < t->la.size(); k++) peers[t->lb[k]].push_back(t->la[k]);
            std::unordered_map<uint32_t, uint32_t> by_id;
            by_id.reserve(m * 2 + 1);
            for (uint64_t k = 0; k < m; k++) {
                if (ev[k].node >= n) return set_error(GOSSIP_EINVAL, "event node out of range");
                if (!by_id.emplace(ev[k].share_id, (uint32_t)k).second)
                    return set_error(GOSSIP_EINVAL, "NetAnim packets need unique share ids (n <= 128,849)");
            }
            struct Pkt {
                int64_t t;
                uint32_t from, to, s;
            };
            std::vector<Pkt> pk;
            std::vector<int64_t> wire(m, 0);  // serialisation of one message of share k
            std::vector<std::string> msg(m);
            for (uint64_t i = 0; i < nt; i++) {
                const auto it = by_id.find(tr_id[i]);
                if (it == by_id.end()) return set_error(GOSSIP_EINVAL, "trace names an unknown share id");
                const uint32_t s = it->second;
                if (tr_node[i] >= n) return set_error(GOSSIP_EINVAL, "trace node out of range");
                if (msg[s].empty()) {
                    std::ostringstream ms;
                    ms << "SHARE:" << ev[s].node << ":" << ev[s].share_id << ":" << (double)ev[s].ns / 1e9;
                    msg[s] = ms.str();
                    wire[s] = ((int64_t)msg[s].size() + header_bytes) * ns_per_byte;
                }
                const int64_t tf = ev[s].ns + (int64_t)tr_hop[i] * (latency_ns + send_defer_ns + wire[s]);
                if (tf >= t_cut_ns) continue;
                for (uint32_t p : peers[tr_node[i]]) pk.push_back(Pkt{tf, tr_node[i], p, s});
            }
            std::stable_sort(pk.begin(), pk.end(), [](const Pkt& a, const Pkt& b) {
                if (a.t != b.t) return a.t < b.t;
                if (a.from != b.from) return a.from < b.from;
                return a.s < b.s;
            });
            os.precision(9);
            os << std::fixed;
            for (const Pkt& q : pk) {
                const int64_t fb = q.t + send_defer_ns, lb = fb + wire[q.s];
                os << "<p fId=\"" << q.from << "\" fbTx=\"" << fb / 1e9 << "\" lbTx=\"" << lb / 1e9
                   << "\" meta-info=\"" << msg[q.s] << "\" tId=\"" << q.to << "\" fbRx=\""
                   << (fb + latency_ns) / 1e9 << "\" lbRx=\"" << (lb + latency_ns) / 1e9 << "\" />\n";
            }
        }
        os << "</anim>\n";
        const std::string out = os.str();
        if (buf && buf_len) {
            const uint64_t k = std::min<uint64_t>(out.size(), buf_len - 1);
            std::memcpy(buf, out.data(), k);
            buf[k] = 0;
        }
        return (int64_t)out.size();
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
}
