// gossip_sim.cpp -- command-line driver: the drop-in replacement for the reference's main()
// (p2pnetwork.cc:289-313) and P2PGossipNetworkSimulation (p2pnetwork.cc:15-286), with the
// NS-3 event loop replaced by the MI355X engine of libgossip.so.
//
//   gossip_sim --numNodes=10 --connectionProb=0.3 --simTime=60 --Latency=5
//
// Same four flags and defaults as the reference (p2pnetwork.cc:294-306, ns3::CommandLine
// syntax --name=value; "--name value" is accepted too).  std::random_device is replaced by
// explicit seeds (--seed for the topology, --nodeSeed for the per-node share RNGs), printed
// so that a run can be reproduced.  The report is the reference's NS_LOG_INFO text.
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gossip.h"

namespace {

struct Options {
    uint32_t numNodes = 10;            // p2pnetwork.cc:294
    double connectionProb = 0.3;       // :295
    double simTime = 60.0;             // :296
    double latencyMs = 5.0;            // :297
    uint32_t seed = 1;                 // replaces rd() at p2pnetwork.cc:65
    uint32_t nodeSeed = 1000;          // replaces rd() at p2pnode.cc:41
    std::string topology = "auto";     // exact | skip | auto
    int device = 0;
    int threads = 8;
    uint32_t maxWords = 0;
    bool quiet = false;                // totals only (no per-node lines)
    bool periodic = true;
    bool timing = false;
    bool handshake = false;            // NS-3 handshake window (GOSSIP_F_HANDSHAKE)
    bool hopBatch = false;             // hop-batched run (GOSSIP_F_HOP_BATCH)
    bool linkTiming = false;           // 5 Mbps serialisation per hop (implies --hopBatch)
    std::string mode = "auto";         // auto | csr | dense
    std::string dumpLinks, dumpEvents, linksIn, eventsIn, dumpTrace, netanim;
    std::string log;  // per-event NS_LOG_INFO lines ("-" = stderr, where NS_LOG writes)
};

void usage() {
    std::fprintf(stderr,
                 "usage: gossip_sim [--numNodes=N] [--connectionProb=P] [--simTime=S] "
                 "[--Latency=MS]\n"
                 "                  [--seed=S] [--nodeSeed=S] [--topology=auto|exact|skip]\n"
                 "                  [--device=D] [--threads=T] [--maxWords=W] [--quiet]\n"
                 "                  [--noPeriodic] [--timing] [--handshake] [--hopBatch] [--linkTiming]\n"
                 "                  [--mode=auto|csr|dense] [--dumpLinks=F] [--dumpEvents=F]\n"
                 "                  [--links=F] [--events=F] [--dumpTrace=F] [--netanim=F]\n"
                 "                  [--log=F|-]\n");
}

bool parse(int argc, char** argv, Options& o) {
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--help" || a == "-h") return false;
        if (a.rfind("--", 0) != 0) {
            std::fprintf(stderr, "unexpected argument '%s'\n", a.c_str());
            return false;
        }
        std::string key = a.substr(2), val;
        const size_t eq = key.find('=');
        bool has_val = eq != std::string::npos;
        if (has_val) {
            val = key.substr(eq + 1);
            key = key.substr(0, eq);
        }
        auto need = [&]() -> bool {
            if (has_val) return true;
            if (i + 1 < argc) {
                val = argv[++i];
                return true;
            }
            std::fprintf(stderr, "missing value for --%s\n", key.c_str());
            return false;
        };
        auto num = [&](double& d) -> bool {
            if (!need()) return false;
            char* end = nullptr;
            errno = 0;
            d = std::strtod(val.c_str(), &end);
            if (errno || end == val.c_str() || *end) {
                std::fprintf(stderr, "invalid value '%s' for --%s\n", val.c_str(), key.c_str());
                return false;
            }
            return true;
        };
        double d = 0;
        if (key == "numNodes") { if (!num(d) || d < 0 || d > 4294967295.0) return false; o.numNodes = (uint32_t)d; }
        else if (key == "connectionProb") { if (!num(o.connectionProb)) return false; }
        else if (key == "simTime") { if (!num(o.simTime)) return false; }
        else if (key == "Latency") { if (!num(o.latencyMs)) return false; }
        else if (key == "seed") { if (!num(d)) return false; o.seed = (uint32_t)d; }
        else if (key == "nodeSeed") { if (!num(d)) return false; o.nodeSeed = (uint32_t)d; }
        else if (key == "device") { if (!num(d)) return false; o.device = (int)d; }
        else if (key == "threads") { if (!num(d)) return false; o.threads = (int)d; }
        else if (key == "maxWords") { if (!num(d)) return false; o.maxWords = (uint32_t)d; }
        else if (key == "topology") { if (!need()) return false; o.topology = val; }
        else if (key == "quiet") o.quiet = true;
        else if (key == "noPeriodic") o.periodic = false;
        else if (key == "timing") o.timing = true;
        else if (key == "handshake") o.handshake = true;
        else if (key == "hopBatch") o.hopBatch = true;
        else if (key == "linkTiming") o.linkTiming = o.hopBatch = true;
        else if (key == "mode") { if (!need()) return false; o.mode = val; }
        else if (key == "dumpLinks") { if (!need()) return false; o.dumpLinks = val; }
        else if (key == "dumpEvents") { if (!need()) return false; o.dumpEvents = val; }
        else if (key == "links") { if (!need()) return false; o.linksIn = val; }
        else if (key == "events") { if (!need()) return false; o.eventsIn = val; }
        else if (key == "dumpTrace") { if (!need()) return false; o.dumpTrace = val; }
        else if (key == "log") { if (!need()) return false; o.log = val; }
        else if (key == "netanim") { if (!need()) return false; o.netanim = val; }
        else {
            std::fprintf(stderr, "unknown option --%s\n", key.c_str());
            return false;
        }
    }
    return true;
}

// SetupNetAnim (p2pnetwork.cc:153-190) as a NetAnim XML file: nodes on a ceil(sqrt(n)) grid
// 100 units apart, "Node i" descriptions, colours by |peers| at the time SetupNetAnim runs --
// Start() calls it before makeconnections, so every node still has 0 peers and is blue
// (the reference's own behaviour) -- and one link per connection key.  The element layout
// follows ns-3's AnimationInterface output; packet records (EnablePacketMetadata) are not
// written.  Visual parity only: no NS-3 run is available to pin the format.
bool write_netanim(const std::string& path, uint32_t n, const std::vector<uint32_t>& a,
                   const std::vector<uint32_t>& b) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return false;
    const uint32_t grid = (uint32_t)std::ceil(std::sqrt((double)n));
    const uint32_t rows = grid ? (n + grid - 1) / grid : 0;
    std::fprintf(f, "<anim ver=\"netanim-3.108\" filetype=\"animation\" >\n");
    std::fprintf(f, "<topology minX = \"0\" minY = \"0\" maxX = \"%u\" maxY = \"%u\">\n",
                 grid ? 100u * (grid - 1) : 0u, rows ? 100u * (rows - 1) : 0u);
    for (uint32_t i = 0; i < n; i++)
        std::fprintf(f, "<node id=\"%u\" sysId=\"0\" locX=\"%u\" locY=\"%u\" />\n", i,
                     100u * (i % grid), 100u * (i / grid));
    for (uint32_t i = 0; i < n; i++) {
        std::fprintf(f, "<nu p=\"c\" t=\"0\" id=\"%u\" r=\"0\" g=\"0\" b=\"255\" />\n", i);
        std::fprintf(f, "<nu p=\"d\" t=\"0\" id=\"%u\" descr=\"Node %u\" />\n", i, i);
    }
    for (size_t k = 0; k < a.size(); k++)
        std::fprintf(f, "<link fromId=\"%u\" toId=\"%u\" fd=\"\" td=\"\" ld=\"\" />\n", a[k], b[k]);
    std::fprintf(f, "</topology>\n</anim>\n");
    return std::fclose(f) == 0;
}

int die(const char* what) {
    std::fprintf(stderr, "gossip_sim: %s failed: %s\n", what, gossip_last_error());
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    if (!parse(argc, argv, o)) {
        usage();
        return 2;
    }
    const int64_t L = gossip_milliseconds_to_ns(o.latencyMs);          // p2pnetwork.cc:114
    const int64_t t_start = gossip_seconds_to_ns(5.0);                 // :93
    const int64_t t_cut = gossip_seconds_to_ns(o.simTime - 0.1);       // :206
    if (!(o.simTime > 0.1)) {
        std::fprintf(stderr, "gossip_sim: --simTime must exceed 0.1 s\n");
        return 2;
    }

    // ---- CreateRandomTopology (p2pnetwork.cc:62-96) ----
    gossip_topology* topo = nullptr;
    if (!o.linksIn.empty()) {
        FILE* f = std::fopen(o.linksIn.c_str(), "r");
        if (!f) { std::perror(o.linksIn.c_str()); return 1; }
        std::vector<uint32_t> a, b;
        unsigned x, y;
        while (std::fscanf(f, "%u %u", &x, &y) == 2) { a.push_back(x); b.push_back(y); }
        std::fclose(f);
        if (gossip_topology_from_links(o.numNodes, a.size(), a.data(), b.data(), &topo)) return die("topology import");
    } else {
        int kind = GOSSIP_TOPO_EXACT;
        if (o.topology == "skip" || (o.topology == "auto" && o.numNodes > 16384)) kind = GOSSIP_TOPO_SKIP;
        else if (o.topology != "exact" && o.topology != "auto") { usage(); return 2; }
        if (gossip_topology_create(o.numNodes, o.connectionProb, o.seed, kind, o.threads, &topo))
            return die("topology");
    }
    const uint32_t n = gossip_topology_num_nodes(topo);

    // ---- share schedule (P2PNode RNGs, p2pnode.cc:33-43, 91-125) ----
    gossip_schedule* sched = nullptr;
    if (!o.eventsIn.empty()) {
        FILE* f = std::fopen(o.eventsIn.c_str(), "r");
        if (!f) { std::perror(o.eventsIn.c_str()); return 1; }
        std::vector<gossip_gen_event> ev;
        long long ns;
        unsigned node, id;
        while (std::fscanf(f, "%lld %u %u", &ns, &node, &id) == 3) ev.push_back({ns, node, id});
        std::fclose(f);
        if (gossip_schedule_from_events(ev.size(), ev.data(), &sched)) return die("schedule import");
    } else if (gossip_schedule_create(n, o.nodeSeed, t_start, t_cut, 0, 0, o.threads, &sched)) {
        return die("schedule");
    }
    if (!o.dumpLinks.empty()) {
        std::vector<uint32_t> a(gossip_topology_num_links(topo)), b(a.size());
        gossip_topology_get_links(topo, a.data(), b.data());
        FILE* f = std::fopen(o.dumpLinks.c_str(), "w");
        for (size_t k = 0; f && k < a.size(); k++) std::fprintf(f, "%u %u\n", a[k], b[k]);
        if (f) std::fclose(f);
    }
    if (!o.netanim.empty()) {
        std::vector<uint32_t> a(gossip_topology_num_links(topo)), b(a.size());
        gossip_topology_get_links(topo, a.data(), b.data());
        if (!write_netanim(o.netanim, n, a, b)) { std::perror(o.netanim.c_str()); return 1; }
        std::printf("NetAnim configured to save in %s\n", o.netanim.c_str());  // p2pnetwork.cc:189
    }
    if (!o.dumpEvents.empty()) {
        std::vector<gossip_gen_event> ev(gossip_schedule_size(sched));
        gossip_schedule_get(sched, ev.data());
        FILE* f = std::fopen(o.dumpEvents.c_str(), "w");
        for (size_t k = 0; f && k < ev.size(); k++)
            std::fprintf(f, "%lld %u %u\n", (long long)ev[k].ns, ev[k].node, ev[k].share_id);
        if (f) std::fclose(f);
    }

    // ---- engine ----
    gossip_config cfg{};
    cfg.num_nodes = n;
    cfg.latency_ns = L;
    cfg.t_start_ns = t_start;
    cfg.t_cut_ns = t_cut;
    cfg.device = o.device;
    if (o.mode == "csr") cfg.mode = GOSSIP_MODE_CSR;
    else if (o.mode == "dense") cfg.mode = GOSSIP_MODE_DENSE;
    else if (o.mode == "auto") cfg.mode = GOSSIP_MODE_AUTO;
    else { usage(); return 2; }
    cfg.max_words = o.maxWords;
    cfg.flags = (o.timing ? GOSSIP_F_TIMING : 0u) | (o.handshake ? GOSSIP_F_HANDSHAKE : 0u) |
                (o.hopBatch ? GOSSIP_F_HOP_BATCH : 0u) | (o.dumpTrace.empty() && o.log.empty() ? 0u : GOSSIP_F_TRACE);
    if (!o.log.empty() && o.handshake) {
        std::fprintf(stderr, "gossip_sim: --log renders the ideal / --linkTiming models, not --handshake\n");
        return 2;
    }
    gossip_engine* eng = nullptr;
    if (gossip_engine_create(&cfg, &eng)) return die("engine create");
    if (gossip_engine_set_topology(eng, topo)) return die("engine graph");
    // NS-3 link timing: 5 Mbps DataRate (p2pnetwork.cc:113) = 1600 ns/byte, 54 header bytes
    // (PPP + IPv4 + TCP with timestamps), 1 ns TcpSocketBase send deferral (gossip.h)
    if (o.linkTiming && gossip_engine_set_link_timing(eng, 1600, 54, 1)) return die("link timing");
    std::vector<double> per_t;
    if (o.periodic)
        for (double t = 10.0; t < o.simTime; t += 10.0) {  // Start(): p2pnetwork.cc:201-204
            if (gossip_engine_add_snapshot(eng, gossip_seconds_to_ns(t))) return die("snapshot");
            per_t.push_back(t);
        }
    if (gossip_engine_set_schedule_obj(eng, sched)) return die("engine schedule");

    std::printf("Starting gossip network simulation for %g seconds\n", o.simTime);
    if (o.hopBatch)
        std::printf("seeds: topology %u, nodes %u; latency %lld ns; hop-batched from tick %lld\n", o.seed,
                    o.nodeSeed, (long long)L, (long long)gossip_engine_first_tick(eng));
    else
        std::printf("seeds: topology %u, nodes %u; latency %lld ns; ticks [%lld, %lld)\n", o.seed,
                    o.nodeSeed, (long long)L, (long long)gossip_engine_first_tick(eng),
                    (long long)gossip_engine_end_tick(eng));
    auto w0 = std::chrono::steady_clock::now();
    if (gossip_engine_run(eng, gossip_engine_end_tick(eng))) return die("engine run");
    if (gossip_engine_sync(eng)) return die("engine sync");
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();

    std::vector<uint32_t> gen(n), recv(n), fwd(n), proc(n), peers(n), sock(n);
    std::vector<uint64_t> sent(n);
    if (gossip_engine_get_stats(eng, gen.data(), recv.data(), fwd.data(), sent.data(), proc.data(),
                                peers.data(), sock.data()))
        return die("stats");
    uint64_t total_sock = 0;
    for (uint32_t v = 0; v < n; v++) total_sock += sock[v];
    for (size_t k = 0; k < per_t.size(); k++) {
        int64_t tns;
        uint64_t tg, tp;
        if (gossip_engine_get_snapshot(eng, (uint32_t)k, &tns, &tg, &tp)) return die("snapshot read");
        // sockets exist from makeconnections (t_start) until StopAllNodes (t_cut)
        const uint64_t sockets_now = (tns >= t_start && tns <= t_cut) ? total_sock : 0;
        std::string buf((size_t)gossip_format_periodic(per_t[k], n, tg, tp, sockets_now, nullptr, 0) + 1, '\0');
        gossip_format_periodic(per_t[k], n, tg, tp, sockets_now, &buf[0], buf.size());
        std::fputs(buf.c_str(), stdout);
    }
    if (t_cut < t_start)  // PrintStatistics before makeconnections: no peers, no sockets yet
        for (uint32_t v = 0; v < n; v++) peers[v] = sock[v] = 0;
    if (o.quiet) {
        uint32_t tg = 0, tr = 0, tf = 0, ts = 0, tc = 0;
        for (uint32_t v = 0; v < n; v++) {
            tg += gen[v]; tr += recv[v]; tf += fwd[v]; ts += (uint32_t)sent[v]; tc += sock[v];
        }
        std::printf("=== P2P Gossip Network Simulation Statistics ===\n");
        std::printf("Total shares generated: %u\nTotal shares received: %u\nTotal shares forwarded: %u\n"
                    "Total shares sent: %u\nTotal socket connections: %u\n", tg, tr, tf, ts, tc);
    } else {
        const int64_t len = gossip_format_statistics(n, gen.data(), recv.data(), fwd.data(), sent.data(),
                                                     proc.data(), peers.data(), sock.data(), nullptr, 0);
        if (len < 0) return die("format");
        std::string buf((size_t)len + 1, '\0');
        gossip_format_statistics(n, gen.data(), recv.data(), fwd.data(), sent.data(), proc.data(),
                                 peers.data(), sock.data(), &buf[0], buf.size());
        std::fputs(buf.c_str(), stdout);
    }
    std::printf("All nodes stopped.\n");
    const uint64_t m_tr = o.dumpTrace.empty() && o.log.empty() ? 0 : gossip_engine_trace_size(eng);
    std::vector<uint32_t> tn(m_tr), ti(m_tr), th(m_tr);
    std::vector<int64_t> tt(m_tr);
    std::vector<uint8_t> tv(m_tr);
    if (m_tr && gossip_engine_get_trace(eng, tn.data(), ti.data(), tt.data(), th.data(), tv.data()))
        return die("trace");
    if (!o.log.empty()) {  // NS_LOG_INFO lines of the gossip path, rendered from the trace
        std::vector<gossip_gen_event> ev(gossip_schedule_size(sched));
        if (!ev.empty()) gossip_schedule_get(sched, ev.data());
        const int64_t npb = o.linkTiming ? 1600 : 0, dfr = o.linkTiming ? 1 : 0;
        const uint32_t hdr = o.linkTiming ? 54u : 0u;
        const int64_t len = gossip_format_event_log(topo, ev.size(), ev.data(), m_tr, tn.data(), ti.data(),
                                                    th.data(), tv.data(), L, t_start, t_cut, npb, hdr, dfr,
                                                    0, nullptr, 0);
        if (len < 0) return die("event log");
        std::string buf((size_t)len + 1, '\0');
        gossip_format_event_log(topo, ev.size(), ev.data(), m_tr, tn.data(), ti.data(), th.data(), tv.data(),
                                L, t_start, t_cut, npb, hdr, dfr, 0, &buf[0], buf.size());
        FILE* f = o.log == "-" ? stderr : std::fopen(o.log.c_str(), "w");
        if (!f) { std::perror(o.log.c_str()); return 1; }
        std::fwrite(buf.data(), 1, (size_t)len, f);
        if (f != stderr) std::fclose(f);
    }
    if (!o.dumpTrace.empty()) {  // first contact per (node, shareId): tick, hop, via ReceiveShare
        const uint64_t m = m_tr;
        FILE* f = std::fopen(o.dumpTrace.c_str(), "w");
        if (!f) { std::perror(o.dumpTrace.c_str()); return 1; }
        for (uint64_t k = 0; k < m; k++)
            std::fprintf(f, "%u %u %lld %u %u\n", tn[k], ti[k], (long long)tt[k], th[k], (unsigned)tv[k]);
        std::fclose(f);
    }
    gossip_counters c{};
    gossip_engine_get_counters(eng, &c);
    std::fprintf(stderr,
                 "[engine] %llu ticks, %llu edge events in %.3f s wall (%.3e edge events/s), "
                 "window %u/%u words%s\n",
                 (unsigned long long)c.ticks, (unsigned long long)c.edge_events, wall,
                 wall > 0 ? (double)c.edge_events / wall : 0.0, c.words_hw, c.words_cap,
                 o.timing ? "" : "");
    if (o.timing && c.pull_ms > 0)
        std::fprintf(stderr, "[engine] pull kernel %.3f ms over %llu launches, %.1f GB/s algorithmic\n",
                     c.pull_ms, (unsigned long long)c.pull_launches, c.pull_bytes / (c.pull_ms * 1e6));
    gossip_engine_destroy(eng);
    gossip_schedule_destroy(sched);
    gossip_topology_destroy(topo);
    return 0;
}
