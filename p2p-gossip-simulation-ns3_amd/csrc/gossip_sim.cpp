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
//
// Multi-GPU (--gpus=N, one host thread per device): --layout=shards (default) runs the share
// instances in S >= N independent shards (gossip_shard_events; no exchange, counters summed on
// the host), doubling S on its own when a shard's live window does not fit a device
// (GOSSIP_ECAPACITY / GOSSIP_ENOMEM); --layout=rows runs the north star's row partition, one
// rank per device, with the per-tick frontier exchange over RCCL (gossip_engine_connect_rccl).
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
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
    bool noPackets = false;            // --netanim without packet records
    std::string mode = "auto";         // auto | csr | dense
    std::string dumpLinks, dumpEvents, linksIn, eventsIn, dumpTrace, netanim;
    std::string log;  // per-event NS_LOG_INFO lines ("-" = stderr, where NS_LOG writes)
    int gpus = 1;                      // devices device .. device+gpus-1, one thread each
    uint32_t shards = 0;               // share shards (0: gpus); doubled on capacity errors
    std::string layout = "shards";     // shards | rows
    double memLimitMB = 0;             // device memory budget per engine (0: the device's)
    std::string schedule = "exact";    // exact (the reference's mt19937 stream) | philox (GPU)
};

void usage() {
    std::fprintf(stderr,
                 "usage: gossip_sim [--numNodes=N] [--connectionProb=P] [--simTime=S] "
                 "[--Latency=MS]\n"
                 "                  [--seed=S] [--nodeSeed=S] [--topology=auto|exact|skip]\n"
                 "                  [--device=D] [--threads=T] [--maxWords=W] [--quiet]\n"
                 "                  [--noPeriodic] [--timing] [--handshake] [--hopBatch] [--linkTiming]\n"
                 "                  [--mode=auto|csr|dense] [--dumpLinks=F] [--dumpEvents=F]\n"
                 "                  [--links=F] [--events=F] [--dumpTrace=F] [--netanim=F] [--noPackets]\n"
                 "                  [--log=F|-] [--gpus=N] [--shards=S] [--layout=shards|rows]\n"
                 "                  [--memLimitMB=M] [--schedule=exact|philox]\n");
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
        else if (key == "noPackets") o.noPackets = true;
        else if (key == "gpus") { if (!num(d) || d < 1 || d > 64) return false; o.gpus = (int)d; }
        else if (key == "shards") { if (!num(d) || d < 0 || d > 4096) return false; o.shards = (uint32_t)d; }
        else if (key == "layout") { if (!need()) return false; o.layout = val; }
        else if (key == "memLimitMB") { if (!num(o.memLimitMB) || o.memLimitMB < 0) return false; }
        else if (key == "schedule") { if (!need()) return false; o.schedule = val; }
        else {
            std::fprintf(stderr, "unknown option --%s\n", key.c_str());
            return false;
        }
    }
    return true;
}

int die(const char* what) {
    std::fprintf(stderr, "gossip_sim: %s failed: %s\n", what, gossip_last_error());
    return 1;
}

// What every engine of a run contributes (summed over shards / row ranks on the host).
struct Part {
    std::vector<uint32_t> gen, recv, fwd, proc, peers, sock;
    std::vector<uint64_t> sent;
    std::vector<int64_t> snap_t;
    std::vector<uint64_t> snap_gen, snap_proc;
    std::vector<uint32_t> tn, ti, th;
    std::vector<int64_t> tt;
    std::vector<uint8_t> tv;
    gossip_counters c{};
    int64_t first_tick = 0, end_tick = 0;
    int rc = 0;
    std::string err;
};

// The ranks of a row partition (--layout=rows) fail together.  Each rank's set-up (device,
// memory budget, graph, schedule) can fail on that rank alone; the ranks therefore meet here
// before ncclCommInitRank, which would otherwise wait forever for a rank that has given up.  A
// rank that fails later, inside the run, aborts the other ranks' communicators
// (gossip_engine_abort), so that they leave their collectives with an error instead of hanging.
struct RowGroup {
    std::mutex m;
    std::condition_variable cv;
    uint32_t count = 0, arrived = 0;
    bool failed = false;
    std::vector<gossip_engine*> live;  // engines that may be inside a collective (guarded by m)

    // Every rank calls this exactly once, with its set-up status; true = all ranks are ready.
    bool ready(uint32_t rank, gossip_engine* e, bool ok) {
        std::unique_lock<std::mutex> lk(m);
        if (!ok) failed = true;
        else live[rank] = e;
        arrived++;
        cv.notify_all();
        cv.wait(lk, [&] { return arrived == count; });
        if (failed) live[rank] = nullptr;
        return !failed;
    }
    // Rank `rank` failed (or finished): take its engine out, and on failure abort the others.
    void leave(uint32_t rank, bool failure) {
        std::lock_guard<std::mutex> lk(m);
        live[rank] = nullptr;
        if (!failure) return;
        failed = true;
        for (gossip_engine* e : live)
            if (e) gossip_engine_abort(e);
    }
};

// One engine, start to finish: shard `rank` of `count` (share sharding) or row rank `rank` of
// `count` (layout rows, exchange over RCCL with the shared communicator id `uid`; `group` is the
// partition's rendezvous).
void run_engine(const gossip_config& base, int device, bool rows, uint32_t rank, uint32_t count,
                const uint8_t* uid, RowGroup* group, const gossip_topology* topo, const gossip_schedule* sched,
                const std::vector<double>& per_t, bool link_timing, bool want_trace, double mem_limit_mb,
                Part& out) {
    gossip_config cfg = base;
    cfg.device = device;
    if (!rows && count > 1) {
        cfg.shard_rank = rank;
        cfg.shard_count = count;
    }
    gossip_engine* eng = nullptr;
    bool met = group == nullptr;  // a row rank has passed the rendezvous
    auto fail = [&](const char* what, int rc) {
        out.rc = rc;
        out.err = std::string(what) + ": " + gossip_last_error();
        if (!met) group->ready(rank, nullptr, false);  // (never leave the other ranks waiting)
        else if (group) group->leave(rank, true);
        if (eng) gossip_engine_destroy(eng);
    };
    int rc = gossip_engine_create(&cfg, &eng);
    if (rc) return fail("engine create", rc);
    if (rows && count > 1 && (rc = gossip_engine_set_row_partition(eng, rank, count))) return fail("row partition", rc);
    if (mem_limit_mb > 0 && (rc = gossip_engine_set_option(eng, "mem_limit", (int64_t)(mem_limit_mb * 1048576.0))))
        return fail("mem limit", rc);
    if ((rc = gossip_engine_set_topology(eng, topo))) return fail("engine graph", rc);
    // NS-3 link timing: 5 Mbps DataRate (p2pnetwork.cc:113) = 1600 ns/byte, 54 header bytes
    // (PPP + IPv4 + TCP with timestamps), 1 ns TcpSocketBase send deferral (gossip.h)
    if (link_timing && (rc = gossip_engine_set_link_timing(eng, 1600, 54, 1))) return fail("link timing", rc);
    for (double t : per_t)  // Start(): p2pnetwork.cc:201-204
        if ((rc = gossip_engine_add_snapshot(eng, gossip_seconds_to_ns(t)))) return fail("snapshot", rc);
    if ((rc = gossip_engine_set_schedule_obj(eng, sched))) return fail("engine schedule", rc);
    if (group) {
        met = true;
        if (!group->ready(rank, eng, true)) {
            out.rc = GOSSIP_ESTATE;
            out.err = "another row rank failed during set-up";
            gossip_engine_destroy(eng);
            return;
        }
        if ((rc = gossip_engine_connect_rccl(eng, uid, 128))) return fail("rccl connect", rc);
    }
    out.first_tick = gossip_engine_first_tick(eng);
    out.end_tick = gossip_engine_end_tick(eng);
    if ((rc = gossip_engine_run(eng, gossip_engine_end_tick(eng)))) return fail("engine run", rc);
    if ((rc = gossip_engine_sync(eng))) return fail("engine sync", rc);
    if (group) group->leave(rank, false);  // (no collective after this point)
    const uint32_t n = base.num_nodes;
    out.gen.assign(n, 0); out.recv.assign(n, 0); out.fwd.assign(n, 0); out.proc.assign(n, 0);
    out.peers.assign(n, 0); out.sock.assign(n, 0); out.sent.assign(n, 0);
    if ((rc = gossip_engine_get_stats(eng, out.gen.data(), out.recv.data(), out.fwd.data(), out.sent.data(),
                                      out.proc.data(), out.peers.data(), out.sock.data())))
        return fail("stats", rc);
    for (size_t k = 0; k < per_t.size(); k++) {
        int64_t tns;
        uint64_t tg, tp;
        if ((rc = gossip_engine_get_snapshot(eng, (uint32_t)k, &tns, &tg, &tp))) return fail("snapshot read", rc);
        out.snap_t.push_back(tns);
        out.snap_gen.push_back(tg);
        out.snap_proc.push_back(tp);
    }
    const uint64_t m = want_trace ? gossip_engine_trace_size(eng) : 0;
    out.tn.resize(m); out.ti.resize(m); out.th.resize(m); out.tt.resize(m); out.tv.resize(m);
    if (m && (rc = gossip_engine_get_trace(eng, out.tn.data(), out.ti.data(), out.tt.data(), out.th.data(),
                                           out.tv.data())))
        return fail("trace", rc);
    gossip_engine_get_counters(eng, &out.c);
    gossip_engine_destroy(eng);
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
        if (gossip_topology_load_links(o.numNodes, o.linksIn.c_str(), &topo)) return die("topology import");
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
        if (gossip_schedule_load_events(n, o.eventsIn.c_str(), &sched)) return die("schedule import");
    } else if (o.schedule == "philox") {  // synthetic: per-node Philox streams, generated on the GPU
        if (gossip_schedule_create_philox(n, o.nodeSeed, t_start, t_cut, 0, o.device, &sched))
            return die("philox schedule");
    } else if (o.schedule != "exact") {
        usage();
        return 2;
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
    if (!o.netanim.empty())  // (the file is written after the run: it holds the run's packets)
        std::printf("NetAnim configured to save in %s\n", o.netanim.c_str());  // p2pnetwork.cc:189
    if (!o.dumpEvents.empty()) {
        std::vector<gossip_gen_event> ev(gossip_schedule_size(sched));
        gossip_schedule_get(sched, ev.data());
        FILE* f = std::fopen(o.dumpEvents.c_str(), "w");
        for (size_t k = 0; f && k < ev.size(); k++)
            std::fprintf(f, "%lld %u %u\n", (long long)ev[k].ns, ev[k].node, ev[k].share_id);
        if (f) std::fclose(f);
    }

    // ---- engines (one per shard / row rank; one host thread per device) ----
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
    if (o.layout != "shards" && o.layout != "rows") { usage(); return 2; }
    const bool rows = o.layout == "rows";
    cfg.max_words = o.maxWords;
    // (NetAnim packet records need the trace and unique ids: small runs, n <= 128,849)
    const bool anim_packets = !o.netanim.empty() && n <= 128849u && !o.noPackets;
    const bool want_trace = !(o.dumpTrace.empty() && o.log.empty()) || anim_packets;
    cfg.flags = (o.timing ? GOSSIP_F_TIMING : 0u) | (o.handshake ? GOSSIP_F_HANDSHAKE : 0u) |
                (o.hopBatch ? GOSSIP_F_HOP_BATCH : 0u) | (want_trace ? GOSSIP_F_TRACE : 0u);
    if (!o.log.empty() && o.handshake) {
        std::fprintf(stderr, "gossip_sim: --log renders the ideal / --linkTiming models, not --handshake\n");
        return 2;
    }
    std::vector<double> per_t;
    if (o.periodic)
        for (double t = 10.0; t < o.simTime; t += 10.0) per_t.push_back(t);  // p2pnetwork.cc:201-204

    std::printf("Starting gossip network simulation for %g seconds\n", o.simTime);
    uint32_t count = rows ? (uint32_t)o.gpus : std::max<uint32_t>(o.shards ? o.shards : 1u, (uint32_t)o.gpus);
    std::vector<Part> parts;
    double wall = 0.0;
    for (;;) {
        parts.assign(count, Part{});
        std::vector<uint8_t> uid(128, 0);
        if (rows && count > 1 && gossip_rccl_unique_id(uid.data(), 128)) return die("rccl unique id");
        RowGroup group;
        group.count = count;
        group.live.assign(count, nullptr);
        RowGroup* gp = rows && count > 1 ? &group : nullptr;
        auto w0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        const uint32_t ng = (uint32_t)o.gpus;
        for (uint32_t g = 0; g < std::min(ng, count); g++)
            th.emplace_back([&, g] {
                // device g runs shards g, g + N, ... (rows: exactly rank g)
                for (uint32_t r = g; r < count; r += ng)
                    run_engine(cfg, o.device + (int)g, rows, r, count, uid.data(), gp, topo, sched, per_t,
                               o.linkTiming, want_trace, o.memLimitMB, parts[r]);
            });
        for (auto& t : th) t.join();
        wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
        int worst = 0;
        std::string err;
        for (const Part& p : parts)  // (report a rank's own failure over the ranks it stopped)
            if (p.rc && (!worst || err.rfind("another row rank", 0) == 0)) { worst = p.rc; err = p.err; }
        if (!worst) break;
        if (!rows && (worst == GOSSIP_ECAPACITY || worst == GOSSIP_ENOMEM) && count < 4096) {
            std::fprintf(stderr, "gossip_sim: %u share shard(s) do not fit (%s); retrying with %u\n", count,
                         err.c_str(), 2 * count);
            count *= 2;
            continue;
        }
        std::fprintf(stderr, "gossip_sim: %s\n", err.c_str());
        return 1;
    }
    if (o.hopBatch)
        std::printf("seeds: topology %u, nodes %u; latency %lld ns; hop-batched from tick %lld\n", o.seed,
                    o.nodeSeed, (long long)L, (long long)parts[0].first_tick);
    else
        std::printf("seeds: topology %u, nodes %u; latency %lld ns; ticks [%lld, %lld)\n", o.seed,
                    o.nodeSeed, (long long)L, (long long)parts[0].first_tick, (long long)parts[0].end_tick);
    if (count > 1)
        std::printf("engines: %u %s on %d GPU(s)\n", count, rows ? "row ranks (RCCL exchange)" : "share shards",
                    o.gpus);
    std::vector<uint32_t> gen(n, 0), recv(n, 0), fwd(n, 0), proc(n, 0), peers = parts[0].peers, sock = parts[0].sock;
    std::vector<uint64_t> sent(n, 0);
    for (const Part& p : parts)  // counters add exactly over shards and row ranks
        for (uint32_t v = 0; v < n; v++) {
            gen[v] += p.gen[v]; recv[v] += p.recv[v]; fwd[v] += p.fwd[v]; proc[v] += p.proc[v];
            sent[v] += p.sent[v];
        }
    uint64_t total_sock = 0;
    for (uint32_t v = 0; v < n; v++) total_sock += sock[v];
    for (size_t k = 0; k < per_t.size(); k++) {
        const int64_t tns = parts[0].snap_t[k];
        uint64_t tg = 0, tp = 0;
        for (const Part& p : parts) {
            // row ranks report the global generation total each; shards their own
            tg = rows ? p.snap_gen[k] : tg + p.snap_gen[k];
            tp += p.snap_proc[k];
        }
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
    std::vector<uint32_t> tn, ti, th;
    std::vector<int64_t> tt;
    std::vector<uint8_t> tv;
    for (const Part& p : parts) {  // every first contact happened on exactly one engine
        tn.insert(tn.end(), p.tn.begin(), p.tn.end());
        ti.insert(ti.end(), p.ti.begin(), p.ti.end());
        th.insert(th.end(), p.th.begin(), p.th.end());
        tt.insert(tt.end(), p.tt.begin(), p.tt.end());
        tv.insert(tv.end(), p.tv.begin(), p.tv.end());
    }
    const uint64_t m_tr = tn.size();
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
    if (!o.netanim.empty()) {  // SetupNetAnim + EnablePacketMetadata (p2pnetwork.cc:153-190)
        std::vector<gossip_gen_event> ev(gossip_schedule_size(sched));
        if (!ev.empty()) gossip_schedule_get(sched, ev.data());
        const int64_t npb = o.linkTiming ? 1600 : 0, dfr = o.linkTiming ? 1 : 0;
        const uint32_t hdr = o.linkTiming ? 54u : 0u;
        const int pk = anim_packets ? 1 : 0;
        const int64_t len = gossip_format_netanim(topo, ev.size(), ev.data(), m_tr, tn.data(), ti.data(), th.data(),
                                                  L, t_cut, npb, hdr, dfr, pk, nullptr, 0);
        if (len < 0) return die("netanim");
        std::string buf((size_t)len + 1, '\0');
        gossip_format_netanim(topo, ev.size(), ev.data(), m_tr, tn.data(), ti.data(), th.data(), L, t_cut, npb, hdr,
                              dfr, pk, &buf[0], buf.size());
        FILE* f = std::fopen(o.netanim.c_str(), "w");
        if (!f) { std::perror(o.netanim.c_str()); return 1; }
        std::fwrite(buf.data(), 1, (size_t)len, f);
        std::fclose(f);
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
    for (const Part& p : parts) {
        c.ticks = std::max(c.ticks, p.c.ticks);
        c.edge_events += p.c.edge_events;
        c.pull_ms += p.c.pull_ms;
        c.pull_launches += p.c.pull_launches;
        c.pull_bytes += p.c.pull_bytes;
        c.words_hw = std::max(c.words_hw, p.c.words_hw);
        c.words_cap = std::max(c.words_cap, p.c.words_cap);
    }
    std::fprintf(stderr,
                 "[engine] %llu ticks, %llu edge events in %.3f s wall (%.3e edge events/s), "
                 "window %u/%u words%s\n",
                 (unsigned long long)c.ticks, (unsigned long long)c.edge_events, wall,
                 wall > 0 ? (double)c.edge_events / wall : 0.0, c.words_hw, c.words_cap,
                 o.timing ? "" : "");
    if (o.timing && c.pull_ms > 0)
        std::fprintf(stderr, "[engine] pull kernel %.3f ms over %llu launches, %.1f GB/s algorithmic\n",
                     c.pull_ms, (unsigned long long)c.pull_launches, c.pull_bytes / (c.pull_ms * 1e6));
    gossip_schedule_destroy(sched);
    gossip_topology_destroy(topo);
    return 0;
}
