// asan_driver.cpp -- CPU sanitizer run (AddressSanitizer + UndefinedBehaviorSanitizer) of the
// host-side C++ of libgossip.so (host.cpp: topology, schedule, CSR, shard rule, dump loaders,
// report; eventlog.cpp: event log + NetAnim) and of both oracles (oracle.cpp, oracle_b.cpp).
// Built and run by `make -C tests/asan` (tests/test_asan.py, CPU suite).  No GPU code is linked:
// the engine (engine.hip) is not part of this build.
//
// Every check prints "ok <name>" or aborts with "FAIL <name>: ..."; any sanitizer report aborts
// the process (-fno-sanitize-recover), so a clean exit status means no report.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gossip.h"
#include "oracle.h"

static int g_checks = 0;

#define CHECK(name, cond)                                                                   \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            std::fprintf(stderr, "FAIL %s: %s (last error: %s)\n", name, #cond, gossip_last_error()); \
            std::exit(1);                                                                   \
        }                                                                                   \
        g_checks++;                                                                         \
    } while (0)

static std::string g_dir;

static std::string write_file(const char* name, const std::string& text) {
    const std::string p = g_dir + "/" + name;
    FILE* f = std::fopen(p.c_str(), "wb");
    if (!f) {
        std::perror(p.c_str());
        std::exit(1);
    }
    std::fwrite(text.data(), 1, text.size(), f);
    std::fclose(f);
    return p;
}

// Every malformed key list must be GOSSIP_EINVAL with *out NULL; the good ones must load.
static void links_dumps() {
    struct Case {
        const char* text;
        bool ok;
    } cases[] = {
        {"0 1\n1 2\n", true},
        {"0 1\r\n1 2\r\n\n\n", true},          // CRLF and blank lines
        {"0\t1\n  2   3  \n", true},            // tabs, padding
        {"", true},                             // no keys at all
        {"0 1\n1\n", false},                    // truncated line
        {"0 1 2\n", false},                     // extra field
        {"0 -1\n", false},                      // sign
        {"0 1x\n", false},                      // trailing garbage in a field
        {"0 0x1\n", false},                     // hex
        {"0 4294967296\n", false},              // u32 overflow
        {"0 99999999999999999999999\n", false}, // u64 overflow
        {"0 10\n", false},                      // node beyond --numNodes (10)
        {"3 3\n", false},                       // self-loop
        {"a b\n", false},                       // not numbers
        {"0 1\n\x01\x02\n", false},             // binary junk
    };
    int k = 0;
    for (const Case& c : cases) {
        char name[64];
        std::snprintf(name, sizeof name, "links_%d.txt", k++);
        const std::string p = write_file(name, c.text);
        gossip_topology* t = reinterpret_cast<gossip_topology*>(0x1);
        const int rc = gossip_topology_load_links(10, p.c_str(), &t);
        if (c.ok) {
            CHECK("links ok", rc == GOSSIP_OK && t != nullptr);
            gossip_topology_destroy(t);
        } else {
            CHECK("links malformed -> EINVAL", rc == GOSSIP_EINVAL && t == nullptr);
            CHECK("links error names the line", std::strstr(gossip_last_error(), "line ") != nullptr);
        }
    }
    gossip_topology* t = nullptr;
    CHECK("links missing file", gossip_topology_load_links(10, (g_dir + "/nope").c_str(), &t) == GOSSIP_EINVAL);
    std::printf("ok links dumps (%d cases)\n", k);
}

static void events_dumps() {
    struct Case {
        const char* text;
        bool ok;
    } cases[] = {
        {"5000000000 1 7\n5000000001 2 8\n", true},
        {"9223372036854775807 0 0\n", true},   // INT64_MAX ns
        {"9223372036854775808 0 0\n", false},  // > INT64_MAX
        {"5000000000 1\n", false},
        {"5000000000 1 7 9\n", false},
        {"-5 1 7\n", false},
        {"5e9 1 7\n", false},
        {"5000000000 10 7\n", false},          // node beyond n
        {"5000000000 1 4294967296\n", false},  // id overflow
    };
    int k = 0;
    for (const Case& c : cases) {
        char name[64];
        std::snprintf(name, sizeof name, "events_%d.txt", k++);
        const std::string p = write_file(name, c.text);
        gossip_schedule* s = reinterpret_cast<gossip_schedule*>(0x1);
        const int rc = gossip_schedule_load_events(10, p.c_str(), &s);
        if (c.ok) {
            CHECK("events ok", rc == GOSSIP_OK && s != nullptr);
            gossip_schedule_destroy(s);
        } else {
            CHECK("events malformed -> EINVAL", rc == GOSSIP_EINVAL && s == nullptr);
        }
    }
    // from_events: negative ns refused; a sparse span (0 .. INT64_MAX) sorts without a giant table
    gossip_gen_event bad[2] = {{-1, 0, 1}, {5, 0, 2}};
    gossip_schedule* s = nullptr;
    CHECK("from_events negative ns", gossip_schedule_from_events(2, bad, &s) == GOSSIP_EINVAL && !s);
    gossip_gen_event wide[3] = {{INT64_MAX, 2, 1}, {0, 1, 2}, {INT64_MAX, 1, 3}};
    CHECK("from_events wide span", gossip_schedule_from_events(3, wide, &s) == GOSSIP_OK);
    gossip_gen_event got[3];
    gossip_schedule_get(s, got);
    CHECK("from_events order", got[0].ns == 0 && got[1].node == 1 && got[2].node == 2);
    gossip_schedule_destroy(s);
    std::printf("ok events dumps (%d cases)\n", k);
}

static void topology_and_schedule() {
    // exact stream vs ORACLE A's reference-mode links (p2pnetwork.cc:62-96)
    const uint32_t n = 60;
    gossip_topology* t = nullptr;
    CHECK("topo exact", gossip_topology_create(n, 0.3, 7, GOSSIP_TOPO_EXACT, 3, &t) == GOSSIP_OK);
    oracle_params p{};
    p.num_nodes = n; p.connection_prob = 0.3; p.sim_time_s = 12.0; p.latency_ms = 5.0;
    p.topo_seed = 7; p.node_seed = 1000;
    oracle_sim* o = nullptr;
    CHECK("oracle create", oracle_create_reference(&p, &o) == 0);
    const uint64_t nl = oracle_get_links(o, nullptr, nullptr);
    std::vector<uint32_t> oa(nl), ob(nl), ga(nl), gb(nl);
    oracle_get_links(o, oa.data(), ob.data());
    CHECK("links count", gossip_topology_num_links(t) == nl);
    gossip_topology_get_links(t, ga.data(), gb.data());
    CHECK("links equal", ga == oa && gb == ob);
    CHECK("oracle trace", oracle_enable_trace(o) == 0 && oracle_enable_log(o) == 0);
    CHECK("oracle run", oracle_run(o) == 0);
    std::vector<uint32_t> gen(n), recv(n), fwd(n), proc(n), peers(n), sock(n);
    std::vector<uint64_t> sent(n);
    oracle_get_stats(o, gen.data(), recv.data(), fwd.data(), sent.data(), proc.data(), peers.data(), sock.data());
    const int64_t loglen = oracle_get_log(o, nullptr, 0);
    std::string olog((size_t)loglen + 1, '\0');
    oracle_get_log(o, &olog[0], olog.size());

    // schedule (p2pnode.cc:33-43, 97-125) vs the oracle's counted generations
    gossip_schedule* s = nullptr;
    const int64_t t0 = gossip_seconds_to_ns(5.0), tc = gossip_seconds_to_ns(12.0 - 0.1);
    CHECK("schedule", gossip_schedule_create(n, 1000, t0, tc, 0, 0, 4, &s) == GOSSIP_OK);
    const uint64_t m = gossip_schedule_size(s);
    std::vector<gossip_gen_event> ev(m);
    gossip_schedule_get(s, ev.data());
    std::vector<int64_t> ons(m + 1);
    std::vector<uint32_t> onode(m + 1), oid(m + 1);
    CHECK("schedule size", oracle_get_gen_events(o, nullptr, nullptr, nullptr) == m);
    oracle_get_gen_events(o, ons.data(), onode.data(), oid.data());
    for (uint64_t k = 0; k < m; k++)
        CHECK("schedule event", ev[k].ns == ons[k] && ev[k].node == onode[k] && ev[k].share_id == oid[k]);

    // event log from the oracle's trace (eventlog.cpp), NetAnim, shard rule
    const uint64_t mt = oracle_get_trace(o, nullptr, nullptr, nullptr, nullptr, nullptr);
    std::vector<uint32_t> tn(mt), ti(mt), th(mt);
    std::vector<int64_t> tt(mt);
    std::vector<uint8_t> tv(mt);
    oracle_get_trace(o, tn.data(), ti.data(), tt.data(), th.data(), tv.data());
    const int64_t L = gossip_milliseconds_to_ns(5.0);
    const int64_t len = gossip_format_event_log(t, m, ev.data(), mt, tn.data(), ti.data(), th.data(), tv.data(), L,
                                                t0, tc, 0, 0, 0, 1, nullptr, 0);
    CHECK("event log size", len > 0);
    std::string buf((size_t)len + 1, '\0');
    gossip_format_event_log(t, m, ev.data(), mt, tn.data(), ti.data(), th.data(), tv.data(), L, t0, tc, 0, 0, 0, 1,
                            &buf[0], buf.size());
    char tiny[7];  // truncated output stays NUL-terminated inside the buffer
    CHECK("event log truncated", gossip_format_event_log(t, m, ev.data(), mt, tn.data(), ti.data(), th.data(),
                                                         tv.data(), L, t0, tc, 0, 0, 0, 1, tiny, sizeof tiny) == len &&
                                     std::strlen(tiny) == sizeof tiny - 1);
    const int64_t alen = gossip_format_netanim(t, m, ev.data(), mt, tn.data(), ti.data(), th.data(), L, tc, 1600, 54,
                                               1, 1, nullptr, 0);
    CHECK("netanim", alen > 0);
    std::string anim((size_t)alen + 1, '\0');
    gossip_format_netanim(t, m, ev.data(), mt, tn.data(), ti.data(), th.data(), L, tc, 1600, 54, 1, 1, &anim[0],
                          anim.size());
    std::vector<uint32_t> owner(m);
    CHECK("shard rule", gossip_shard_events(t, m, ev.data(), 3, owner.data()) == GOSSIP_OK);
    for (uint32_t w : owner) CHECK("shard range", w < 3);
    // the birth-tick rule, its collision branch too: ids folded to 6 bits collide
    // across nodes, and every (id, component) instance must stay on one shard
    {
        std::vector<gossip_gen_event> cev(ev.begin(), ev.end());
        for (auto& x : cev) x.share_id &= 0x3fu;
        std::vector<uint32_t> own8(m);
        CHECK("shard by tick", gossip_shard_events_by_tick(t, m, cev.data(), 8, L, own8.data()) == GOSSIP_OK);
        bool whole = true;
        for (uint64_t i = 0; i < m; i++) {
            CHECK("shard by tick range", own8[i] < 8);
            for (uint64_t j = i + 1; j < m; j++)  // (n = 60 is one component: same id, same shard)
                if (cev[i].share_id == cev[j].share_id && own8[i] != own8[j]) whole = false;
        }
        CHECK("shard by tick keeps instances whole", whole);
        CHECK("shard by tick bad latency", gossip_shard_events_by_tick(t, m, cev.data(), 8, 0, own8.data()) != GOSSIP_OK);
    }

    // the report (p2pnetwork.cc:253-285) with full and truncated buffers
    const int64_t rl = gossip_format_statistics(n, gen.data(), recv.data(), fwd.data(), sent.data(), proc.data(),
                                                peers.data(), sock.data(), nullptr, 0);
    std::string rep((size_t)rl + 1, '\0');
    gossip_format_statistics(n, gen.data(), recv.data(), fwd.data(), sent.data(), proc.data(), peers.data(),
                             sock.data(), &rep[0], rep.size());
    CHECK("report text", rep.find("Total shares sent") != std::string::npos);
    char one[1];
    gossip_format_statistics(n, gen.data(), recv.data(), fwd.data(), sent.data(), proc.data(), peers.data(),
                             sock.data(), one, 1);
    CHECK("report 1-byte buffer", one[0] == 0);
    char per[256];
    CHECK("periodic", gossip_format_periodic(10.0, n, 5, 7, 9, per, sizeof per) > 0);

    // ORACLE B on the same replay (distinct ids at n = 60) equals ORACLE A
    std::vector<int64_t> ens(m);
    std::vector<uint32_t> enode(m), eid(m);
    for (uint64_t k = 0; k < m; k++) { ens[k] = ev[k].ns; enode[k] = ev[k].node; eid[k] = ev[k].share_id; }
    std::vector<uint32_t> bgen(n), brecv(n), bfwd(n), bproc(n), bpeers(n), bsock(n);
    std::vector<uint64_t> bsent(n);
    uint64_t bee = 0;
    CHECK("oracle b", oracle_b_run(n, L, tc, nl, oa.data(), ob.data(), m, ens.data(), enode.data(), eid.data(), 3,
                                   bgen.data(), brecv.data(), bfwd.data(), bsent.data(), bproc.data(), bpeers.data(),
                                   bsock.data(), &bee) == 0);
    CHECK("oracle b == a", bgen == gen && brecv == recv && bsent == sent && bproc == proc && bpeers == peers);

    // the replay mode of ORACLE A on a colliding-id schedule (id_mask), with link timing
    std::vector<uint32_t> mid(m);
    for (uint64_t k = 0; k < m; k++) mid[k] = eid[k] & 0x3f;
    oracle_sim* r = nullptr;
    CHECK("replay", oracle_create_replay(n, L, t0, tc, nl, oa.data(), ob.data(), m, ens.data(), enode.data(),
                                         mid.data(), &r) == 0);
    CHECK("replay timing", oracle_set_link_timing(r, 1600, 54, 1) == 0 && oracle_run(r) == 0);
    oracle_destroy(r);
    oracle_destroy(o);
    gossip_schedule_destroy(s);
    gossip_topology_destroy(t);

    // the skip generator (Philox rows) on several threads, and error paths
    CHECK("topo skip", gossip_topology_create(20000, 16.0 / 19999, 3, GOSSIP_TOPO_SKIP, 8, &t) == GOSSIP_OK);
    const uint64_t nnz = gossip_topology_num_entries(t);
    std::vector<int64_t> rp(20001);
    std::vector<int32_t> col(nnz);
    std::vector<uint8_t> mult(nnz);
    gossip_topology_get_csr(t, rp.data(), col.data(), mult.data());
    CHECK("csr", rp[20000] == (int64_t)nnz);
    gossip_topology_destroy(t);
    uint32_t la[2] = {0, 5}, lb[2] = {1, 5};
    t = reinterpret_cast<gossip_topology*>(0x1);
    CHECK("from_links self-loop", gossip_topology_from_links(6, 2, la, lb, &t) == GOSSIP_EINVAL && t == nullptr);
    std::printf("ok topology, schedule, report, event log, NetAnim, oracles (n=%u, %" PRIu64 " events)\n", n, m);
}

int main(int argc, char** argv) {
    g_dir = argc > 1 ? argv[1] : "/tmp";
    links_dumps();
    events_dumps();
    topology_and_schedule();
    std::printf("asan_driver: %d checks passed\n", g_checks);
    return 0;
}
