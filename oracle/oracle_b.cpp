// oracle_b.cpp -- ORACLE B: bit-sliced, level-synchronous CPU restatement of the gossip path
// for schedules whose share ids are all distinct (n <= 128,849 at simTime ~ 60 s; SURVEY.md
// A.5).  TEST INFRASTRUCTURE ONLY (see oracle.h): it checks the HIP engine at sizes where
// ORACLE A's event loop is too slow (a 65,536-node p = 0.3 flood is ~1.3e9 edge events per
// share).
//
// Why a level-synchronous BFS restates the reference exactly when ids are distinct:
//   * the seen-set is keyed by shareId (p2pnode.cc:189), so with distinct ids every share is an
//     independent flood; no share can suppress another;
//   * a node first reaches share s through the first arrival of any copy (HandleRead at
//     p2pnode.cc:189-197 inserts on the first, drops the rest), i.e. at BFS distance h from the
//     origin, at time t_s + h * Latency (ideal hop, ORACLE A's transport);
//   * ReceiveShare (p2pnode.cc:155-165) counts received / forwarded once and forwards to every
//     entry of peers (multiplicity included, sender included): sent += |peers|;
//   * GenerateAndGossipShare (p2pnode.cc:106-125): gen++, sent += |peers|; a generation at a
//     node with no peers is not counted (p2pnode.cc:108-113);
//   * PrintStatistics runs at t_cut before any same-time arrival (p2pnetwork.cc:206), so hop h
//     counts iff t_s + h * Latency < t_cut; a later hop never counts once an earlier one did not.
// Peer lists come from the link keys exactly as ORACLE A builds them: key (a,b) puts b in
// peers(a) de-duplicated (AddPeer, p2pnode.cc:77-83) and a in peers(b) without de-duplication
// (REGISTER branch, p2pnode.cc:178-188).
//
// Work: 64 shares per 64-bit word; per hop, inc[v] = OR over distinct peers u of F[u].
#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "oracle.h"

namespace {

thread_local std::string g_err_b;
thread_local double g_wall_b = 0.0;  // seconds of the last run's level-synchronous propagation

int fail_b(const std::string& m) {
    g_err_b = m;
    return -1;
}

template <class F>
void par_for(uint64_t n, int threads, F&& f) {
    if (threads <= 1 || n < 1024) {
        f(0, n);
        return;
    }
    std::vector<std::thread> ts;
    const uint64_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        const uint64_t lo = std::min<uint64_t>(n, (uint64_t)t * chunk), hi = std::min<uint64_t>(n, lo + chunk);
        if (lo < hi) ts.emplace_back([&, lo, hi] { f(lo, hi); });
    }
    for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

const char* oracle_b_last_error(void) { return g_err_b.c_str(); }
// wall time of the last oracle_b_run's propagation (the bit-sliced BFS levels), without the
// CSR construction: what a timed CPU baseline of the hot path measures
double oracle_b_last_wall_s(void) { return g_wall_b; }

int oracle_b_run(uint32_t n, int64_t latency_ns, int64_t t_cut_ns, uint64_t num_links,
                 const uint32_t* la, const uint32_t* lb, uint64_t num_events, const int64_t* ev_ns,
                 const uint32_t* ev_node, const uint32_t* ev_id, int num_threads, uint32_t* gen,
                 uint32_t* recv, uint32_t* fwd, uint64_t* sent, uint32_t* processed,
                 uint32_t* peers_out, uint32_t* sockets_out, uint64_t* edge_events) {
    if (n == 0 || latency_ns <= 0) return fail_b("bad n / latency");
    {
        std::vector<uint32_t> ids(ev_id, ev_id + num_events);
        std::sort(ids.begin(), ids.end());
        if (std::adjacent_find(ids.begin(), ids.end()) != ids.end())
            return fail_b("ORACLE B needs distinct share ids (use ORACLE A for collisions)");
    }
    // Keys in std::map order, one entry per key (p2pnetwork.cc:30,129).
    std::vector<std::pair<uint32_t, uint32_t>> keys(num_links);
    for (uint64_t k = 0; k < num_links; k++) {
        if (la[k] >= n || lb[k] >= n) return fail_b("link out of range");
        keys[k] = {la[k], lb[k]};
    }
    if (!std::is_sorted(keys.begin(), keys.end())) std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    const int th = std::max(1, num_threads);
    // |peers| (duplicates counted) and the distinct-neighbour adjacency.  peers(a) gains b once
    // per distinct key (a,b) -- AddPeer's find() only matters for a repeated key, which the map
    // already merged -- and peers(b) gains a per key (a,b).  So |peers(v)| = #keys touching v
    // and the distinct neighbours are the union of both directions.
    std::vector<uint32_t> deg(n, 0);
    std::vector<uint64_t> rp((size_t)n + 1, 0);
    for (const auto& kv : keys) {
        deg[kv.first]++;
        deg[kv.second]++;
        rp[kv.first + 1]++;
        rp[kv.second + 1]++;
    }
    for (uint32_t v = 0; v < n; v++) rp[v + 1] += rp[v];
    std::vector<uint32_t> adj(rp[n]);
    {
        std::vector<uint64_t> pos(rp.begin(), rp.end() - 1);
        for (const auto& kv : keys) {
            adj[pos[kv.first]++] = kv.second;
            adj[pos[kv.second]++] = kv.first;
        }
    }
    // de-duplicate each row (a parallel link pair (i,i-1) + (i-1,i) lists the neighbour twice)
    std::vector<uint64_t> rp2((size_t)n + 1, 0);
    std::vector<uint32_t> sock(n, 0);
    par_for(n, th, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t v = lo; v < hi; v++) {
            uint32_t* b = adj.data() + rp[v];
            uint32_t* e = adj.data() + rp[v + 1];
            std::sort(b, e);
            sock[v] = (uint32_t)(std::unique(b, e) - b);
        }
    });
    for (uint32_t v = 0; v < n; v++) rp2[v + 1] = rp2[v] + sock[v];
    std::vector<uint32_t> col(rp2[n]);
    par_for(n, th, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t v = lo; v < hi; v++)
            std::memcpy(col.data() + rp2[v], adj.data() + rp[v], sock[v] * 4ull);
    });
    std::vector<uint64_t>().swap(rp);
    std::vector<uint32_t>().swap(adj);

    std::vector<uint32_t> g(n, 0), r(n, 0);
    std::vector<uint64_t> s(n, 0);
    // Counted generations: nodes with peers only (p2pnode.cc:108-113).
    std::vector<uint64_t> live_ev;
    for (uint64_t k = 0; k < num_events; k++) {
        if (ev_node[k] >= n) return fail_b("event node out of range");
        if (ev_ns[k] >= t_cut_ns) continue;  // after PrintStatistics
        if (deg[ev_node[k]] == 0) continue;
        live_ev.push_back(k);
        g[ev_node[k]]++;
        s[ev_node[k]] += deg[ev_node[k]];
    }
    std::vector<uint64_t> F(n), Fn(n), seen(n);
    const auto w0 = std::chrono::steady_clock::now();
    for (size_t b0 = 0; b0 < live_ev.size(); b0 += 64) {
        const size_t nb = std::min<size_t>(64, live_ev.size() - b0);
        std::fill(F.begin(), F.end(), 0ull);
        std::fill(seen.begin(), seen.end(), 0ull);
        for (size_t q = 0; q < nb; q++) {
            const uint32_t o = ev_node[live_ev[b0 + q]];
            F[o] |= 1ull << q;
            seen[o] |= 1ull << q;
        }
        for (int64_t h = 1;; h++) {
            // shares whose hop-h arrivals precede PrintStatistics
            uint64_t keep = 0ull;
            for (size_t q = 0; q < nb; q++) {
                const int64_t t = ev_ns[live_ev[b0 + q]];
                if (t_cut_ns - t > h * latency_ns) keep |= 1ull << q;  // t + h L < t_cut, no overflow
            }
            if (!keep) break;
            std::atomic<uint64_t> any{0};
            par_for(n, th, [&](uint64_t lo, uint64_t hi) {
                uint64_t a = 0;
                for (uint64_t v = lo; v < hi; v++) {
                    uint64_t inc = 0;
                    for (uint64_t j = rp2[v]; j < rp2[v + 1]; j++) inc |= F[col[j]];
                    const uint64_t nw = inc & ~seen[v] & keep;
                    Fn[v] = nw;
                    if (nw) {
                        seen[v] |= nw;
                        const uint32_t c = (uint32_t)__builtin_popcountll(nw);
                        r[v] += c;
                        s[v] += (uint64_t)c * deg[v];
                        a |= nw;
                    }
                }
                if (a) any.fetch_or(a);
            });
            F.swap(Fn);
            if (!any.load()) break;
        }
    }
    g_wall_b = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();
    uint64_t ee = 0;
    for (uint32_t v = 0; v < n; v++) ee += s[v];
    if (gen) std::memcpy(gen, g.data(), n * 4ull);
    if (recv) std::memcpy(recv, r.data(), n * 4ull);
    if (fwd) std::memcpy(fwd, r.data(), n * 4ull);  // sharesForwarded++ beside sharesReceived++
    if (sent) std::memcpy(sent, s.data(), n * 8ull);
    if (processed)
        for (uint32_t v = 0; v < n; v++) processed[v] = g[v] + r[v];  // distinct ids
    if (peers_out) std::memcpy(peers_out, deg.data(), n * 4ull);
    if (sockets_out) std::memcpy(sockets_out, sock.data(), n * 4ull);
    if (edge_events) *edge_events = ee;
    return 0;
}

}  // extern "C"
