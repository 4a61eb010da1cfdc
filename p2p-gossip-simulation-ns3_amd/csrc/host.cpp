// host.cpp -- host C++ core of libgossip.so: ns-3 time conversion, the reference's G(n,p)
// topology with its fix-up, per-node share schedules, and the statistics report.
//
// Reference behaviour restated here (see SURVEY.md Appendix A for the quirks):
//   CreateRandomTopology      p2pnetwork.cc:62-96   (one mt19937, 2 draws per pair,
//                                                    "no forward link => (i,i-1)" fix-up)
//   makeconnections/REGISTER  p2pnetwork.cc:99-150, p2pnode.cc:77-89,178-188
//   P2PNode RNG seeding       p2pnode.cc:33-43
//   ScheduleNextShare etc.    p2pnode.cc:91-125
//   GenerateUniqueShareId     p2pnode.cc:201-209
//   PrintStatistics           p2pnetwork.cc:253-285
//   PrintPeriodicStats        p2pnetwork.cc:231-250
#include <algorithm>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <new>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "internal.h"

namespace gossip {

thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int64_t exact_scale_round(double x, uint64_t factor) {
    if (x == 0.0 || !std::isfinite(x)) return 0;
    const bool neg = x < 0;
    const double ax = neg ? -x : x;
    int e2 = 0;
    const double m = std::frexp(ax, &e2);
    const uint64_t M = (uint64_t)std::ldexp(m, 53);
    const int sh = e2 - 53;
    const unsigned __int128 P = (unsigned __int128)M * factor;
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
            if (rem >= ((unsigned __int128)1 << (s - 1))) q += 1;
        }
    }
    const int64_t r = (int64_t)q;
    return neg ? -r : r;
}

// ---------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11): counter-based, so every topology row draws from its
// own stream and rows can be generated on any number of threads with identical output.
// ---------------------------------------------------------------------------------------
struct Philox {
    static inline void round(uint32_t c[4], const uint32_t k[2]) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k[0];
        const uint32_t n2 = hi0 ^ c[3] ^ k[1];
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    }
    static inline void block(uint32_t ctr[4], uint32_t key0, uint32_t key1, uint32_t out[4]) {
        uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
        uint32_t k[2] = {key0, key1};
        for (int r = 0; r < 10; r++) {
            round(c, k);
            k[0] += 0x9E3779B9u;
            k[1] += 0xBB67AE85u;
        }
        out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
    }
};

// Uniform (0,1] doubles from a Philox stream keyed by (seed, row).
struct RowStream {
    uint32_t seed, row, ctr = 0, idx = 4;
    uint32_t buf[4];
    RowStream(uint32_t s, uint32_t r) : seed(s), row(r) {}
    uint32_t next32() {
        if (idx == 4) {
            uint32_t c[4] = {row, ctr++, 0x6f737369u /* "ossi" */, 0x70676f73u};
            Philox::block(c, seed, 0x47535350u, buf);
            idx = 0;
        }
        return buf[idx++];
    }
    double open_closed() {  // (0,1]
        const uint64_t hi = next32() >> 5, lo = next32() >> 6;  // 27 + 26 = 53 bits
        return ((double)((hi << 26) | lo) + 1.0) * (1.0 / 9007199254740992.0);
    }
};

int build_csr(gossip_topology* t, int threads) {
    const uint32_t n = t->n;
    const uint64_t nl = t->la.size();
    std::vector<int64_t> cnt((size_t)n + 1, 0);
    for (uint64_t k = 0; k < nl; k++) {
        cnt[t->la[k] + 1]++;
        cnt[t->lb[k] + 1]++;
    }
    for (uint32_t v = 0; v < n; v++) cnt[v + 1] += cnt[v];
    std::vector<int32_t> raw((size_t)cnt[n]);
    {
        std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
        for (uint64_t k = 0; k < nl; k++) {
            const uint32_t a = t->la[k], b = t->lb[k];
            raw[pos[a]++] = (int32_t)b;  // key (a,b): b in peers(a)  (AddPeer)
            raw[pos[b]++] = (int32_t)a;  // key (a,b): a in peers(b)  (REGISTER)
        }
    }
    // Per row: sort, then merge duplicates into multiplicity.
    std::vector<uint32_t> distinct(n, 0);
    parallel_for(n, threads, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t v = lo; v < hi; v++) {
            int32_t* b = raw.data() + cnt[v];
            int32_t* e = raw.data() + cnt[v + 1];
            std::sort(b, e);
            uint32_t d = 0;
            for (int32_t* p = b; p != e; ++p)
                if (p == b || *p != *(p - 1)) d++;
            distinct[v] = d;
        }
    });
    t->row_ptr.assign((size_t)n + 1, 0);
    for (uint32_t v = 0; v < n; v++) t->row_ptr[v + 1] = t->row_ptr[v] + distinct[v];
    const uint64_t nnz = (uint64_t)t->row_ptr[n];
    t->col.resize(nnz);
    t->mult.resize(nnz);
    t->peers.resize(n);
    t->sockets.resize(n);
    parallel_for(n, threads, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t v = lo; v < hi; v++) {
            const int32_t* b = raw.data() + cnt[v];
            const int32_t* e = raw.data() + cnt[v + 1];
            int64_t o = t->row_ptr[v] - 1;
            for (const int32_t* p = b; p != e; ++p) {
                if (p == b || *p != *(p - 1)) {
                    ++o;
                    t->col[o] = *p;
                    t->mult[o] = 1;
                } else {
                    t->mult[o]++;
                }
            }
            t->peers[v] = (uint32_t)(cnt[v + 1] - cnt[v]);
            t->sockets[v] = distinct[v];
        }
    });
    return 0;
}

std::vector<uint32_t> components(uint32_t n, const int64_t* row_ptr, const int32_t* col) {
    std::vector<uint32_t> comp(n);
    for (uint32_t v = 0; v < n; v++) comp[v] = v;
    auto find = [&](uint32_t x) {
        while (comp[x] != x) {
            comp[x] = comp[comp[x]];
            x = comp[x];
        }
        return x;
    };
    for (uint32_t v = 0; v < n; v++)
        for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; j++) {
            const uint32_t a = find(v), b = find((uint32_t)col[j]);
            if (a != b) comp[std::max(a, b)] = std::min(a, b);
        }
    for (uint32_t v = 0; v < n; v++) comp[v] = find(v);
    return comp;
}

static std::mutex g_comp_mu;

const std::vector<uint32_t>& topology_components(const gossip_topology* t) {
    std::lock_guard<std::mutex> g(g_comp_mu);
    if (t->comp.empty() && t->n) t->comp = components(t->n, t->row_ptr.data(), t->col.data());
    return t->comp;
}

bool cached_topology_components(const gossip_topology* t, std::vector<uint32_t>* out) {
    std::lock_guard<std::mutex> g(g_comp_mu);
    if (t->comp.empty()) return false;
    *out = t->comp;
    return true;
}

uint64_t instance_hash(uint32_t share_id, uint32_t node_or_comp, bool lone) {
    uint64_t x = ((uint64_t)share_id << 32) ^ node_or_comp ^ (lone ? 0x9e3779b97f4a7c15ull : 0ull);
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

bool any_id_collision(uint64_t m, const gossip_gen_event* ev) {
    std::vector<uint32_t> ids(m);
    for (uint64_t k = 0; k < m; k++) ids[k] = ev[k].share_id;
    std::sort(ids.begin(), ids.end());
    for (uint64_t k = 1; k < m; k++)
        if (ids[k] == ids[k - 1]) return true;
    return false;
}

}  // namespace gossip

using namespace gossip;

// latency_ns > 0: the birth-tick rule (gossip_shard_events_by_tick), else the hash rule
static int shard_events_rule(const gossip_topology* t, uint64_t m, const gossip_gen_event* ev,
                             uint32_t shard_count, int64_t latency_ns, uint32_t* owner) {
    if (!t || (m && (!ev || !owner))) return set_error(GOSSIP_EINVAL, "NULL argument");
    if (shard_count == 0) return set_error(GOSSIP_EINVAL, "shard_count must be >= 1");
    if (m >= (1ull << 32)) return set_error(GOSSIP_EINVAL, "more than 2^32 - 1 events");
    try {
        for (uint64_t k = 0; k < m; k++)
            if (ev[k].node >= t->n) return set_error(GOSSIP_EINVAL, "event node out of range");
        // one sort of (id, event index): runs of equal ids give both the collision test and
        // every event's lone flag
        std::vector<uint64_t> key(m);
        for (uint64_t k = 0; k < m; k++) key[k] = ((uint64_t)ev[k].share_id << 32) | k;
        std::sort(key.begin(), key.end());
        std::vector<uint8_t> lone(m, 1);
        bool collision = false;
        for (uint64_t k = 1; k < m; k++)
            if ((key[k] >> 32) == (key[k - 1] >> 32)) {
                lone[(uint32_t)key[k]] = lone[(uint32_t)key[k - 1]] = 0;
                collision = true;
            }
        key = std::vector<uint64_t>();
        if (collision) topology_components(t);
        if (latency_ns > 0) {
            // birth-tick rule: the first generation of the instance (lone: the event itself)
            std::unordered_map<uint64_t, int64_t> first;  // (id, component) -> earliest ns
            if (collision)
                for (uint64_t k = 0; k < m; k++)
                    if (!lone[k]) {
                        const uint64_t ik = ((uint64_t)ev[k].share_id << 32) | t->comp[ev[k].node];
                        auto it = first.find(ik);
                        if (it == first.end() || ev[k].ns < it->second) first[ik] = ev[k].ns;
                    }
            for (uint64_t k = 0; k < m; k++) {
                const int64_t ns = lone[k] ? ev[k].ns : first[((uint64_t)ev[k].share_id << 32) | t->comp[ev[k].node]];
                owner[k] = (uint32_t)((uint64_t)(ns / latency_ns) % shard_count);
            }
            return GOSSIP_OK;
        }
        for (uint64_t k = 0; k < m; k++) {
            const uint64_t h = lone[k] ? instance_hash(ev[k].share_id, ev[k].node, true)
                                       : instance_hash(ev[k].share_id, t->comp[ev[k].node], false);
            owner[k] = (uint32_t)(h % shard_count);
        }
        return GOSSIP_OK;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
}

extern "C" int gossip_shard_events(const gossip_topology* t, uint64_t m, const gossip_gen_event* ev,
                                   uint32_t shard_count, uint32_t* owner) {
    return shard_events_rule(t, m, ev, shard_count, 0, owner);
}

extern "C" int gossip_shard_events_by_tick(const gossip_topology* t, uint64_t m, const gossip_gen_event* ev,
                                           uint32_t shard_count, int64_t latency_ns, uint32_t* owner) {
    if (latency_ns <= 0) return set_error(GOSSIP_EINVAL, "latency_ns must be > 0");
    return shard_events_rule(t, m, ev, shard_count, latency_ns, owner);
}

extern "C" {

const char* gossip_last_error(void) { return g_last_error.c_str(); }
const char* gossip_version(void) { return "gossip-mi355x 0.1.0"; }

int64_t gossip_seconds_to_ns(double seconds) { return exact_scale_round(seconds, 1000000000ull); }

// len(Share::ToString()) (p2pnode.cc:6-11): the same ostream formatting of the same fields.
// timestamp = Simulator::Now().GetSeconds() (p2pnode.cc:119), taken here as ns / 1e9 in double
// (ns-3 divides in int64x64 first: the two can differ by one ulp, which moves the 6-digit
// rendering only on an exact decimal tie -- unpinned).
uint32_t gossip_share_message_length(uint32_t origin, uint32_t share_id, int64_t t_ns) {
    std::ostringstream ss;
    ss << "SHARE:" << origin << ":" << share_id << ":" << (double)t_ns / 1e9;
    return (uint32_t)ss.str().size();
}
int64_t gossip_milliseconds_to_ns(double ms) { return exact_scale_round(ms, 1000000ull); }

// ---------------------------------------------------------------------------------------
// Topology
// ---------------------------------------------------------------------------------------
int gossip_topology_create(uint32_t num_nodes, double p, uint32_t seed, int kind,
                           int num_threads, gossip_topology** out) {
    if (!out) return set_error(GOSSIP_EINVAL, "out is NULL");
    *out = nullptr;
    if (num_nodes < 2)
        return set_error(GOSSIP_EINVAL,
                         "numNodes < 2: the reference's fix-up indexes nodes.Get(1) "
                         "(p2pnetwork.cc:82) and aborts");
    if (!(p == p)) return set_error(GOSSIP_EINVAL, "connectionProb is NaN");
    try {
        auto t = std::make_unique<gossip_topology>();
        t->n = num_nodes;
        const uint32_t n = num_nodes;
        if (kind == GOSSIP_TOPO_EXACT) {
            // p2pnetwork.cc:64-85, literally: one engine, row-major i<j, two 32-bit draws
            // per pair (generate_canonical<double,53>), fix-up when no j>i link was made.
            // Keys come out in std::map order: row i emits (i, j>i) ascending, or the single
            // fix-up key (i, i-1) / (0, 1).
            std::mt19937 rng(seed);
            std::uniform_real_distribution<double> dist(0.0, 1.0);
            for (uint32_t i = 0; i < n; i++) {
                bool connected = false;
                for (uint32_t j = i + 1; j < n; j++) {
                    if (dist(rng) < p) {
                        connected = true;
                        t->la.push_back(i);
                        t->lb.push_back(j);
                    }
                }
                if (!connected) {
                    t->la.push_back(i);
                    t->lb.push_back(i == 0 ? 1u : i - 1);
                }
            }
        } else if (kind == GOSSIP_TOPO_SKIP) {
            // Same G(n,p) law and the same fix-up, sampled by geometric skipping with a
            // per-row Philox stream: O(links) work, rows on any number of threads.
            const int T = std::max(1, num_threads);
            const uint64_t chunks = std::min<uint64_t>(n, (uint64_t)T * 16);
            std::vector<std::vector<uint32_t>> ca(chunks), cb(chunks);
            const double lq = (p > 0.0 && p < 1.0) ? std::log1p(-p) : 0.0;
            parallel_for(chunks, T, [&](uint64_t c0, uint64_t c1) {
                for (uint64_t c = c0; c < c1; c++) {
                    const uint32_t lo = (uint32_t)((uint64_t)n * c / chunks);
                    const uint32_t hi = (uint32_t)((uint64_t)n * (c + 1) / chunks);
                    auto& A = ca[c];
                    auto& B = cb[c];
                    for (uint32_t i = lo; i < hi; i++) {
                        bool connected = false;
                        if (p >= 1.0) {
                            for (uint32_t j = i + 1; j < n; j++) {
                                A.push_back(i); B.push_back(j); connected = true;
                            }
                        } else if (p > 0.0) {
                            RowStream rs(seed, i);
                            int64_t j = i;
                            for (;;) {
                                const double u = rs.open_closed();
                                const double skip = std::floor(std::log(u) / lq);
                                if (skip >= (double)n) break;
                                j += (int64_t)skip + 1;
                                if (j >= (int64_t)n) break;
                                A.push_back(i); B.push_back((uint32_t)j);
                                connected = true;
                            }
                        }
                        if (!connected) {
                            A.push_back(i);
                            B.push_back(i == 0 ? 1u : i - 1);
                        }
                    }
                }
            });
            uint64_t total = 0;
            for (auto& v : ca) total += v.size();
            t->la.reserve(total);
            t->lb.reserve(total);
            for (uint64_t c = 0; c < chunks; c++) {
                t->la.insert(t->la.end(), ca[c].begin(), ca[c].end());
                t->lb.insert(t->lb.end(), cb[c].begin(), cb[c].end());
                std::vector<uint32_t>().swap(ca[c]);
                std::vector<uint32_t>().swap(cb[c]);
            }
        } else {
            return set_error(GOSSIP_EINVAL, "unknown topology kind");
        }
        build_csr(t.get(), std::max(1, num_threads));
        *out = t.release();
        return GOSSIP_OK;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed building topology");
    }
}

int gossip_topology_from_links(uint32_t num_nodes, uint64_t num_links, const uint32_t* a,
                               const uint32_t* b, gossip_topology** out) {
    if (!out || (num_links && (!a || !b))) return set_error(GOSSIP_EINVAL, "NULL argument");
    *out = nullptr;
    try {
        auto t = std::make_unique<gossip_topology>();
        t->n = num_nodes;
        std::vector<std::pair<uint32_t, uint32_t>> keys(num_links);
        for (uint64_t k = 0; k < num_links; k++) {
            if (a[k] >= num_nodes || b[k] >= num_nodes || a[k] == b[k])
                return set_error(GOSSIP_EINVAL, "link endpoint out of range or self-loop");
            keys[k] = {a[k], b[k]};
        }
        // std::map semantics: ordered, duplicate keys collapse (p2pnetwork.cc:129).
        std::sort(keys.begin(), keys.end());
        keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
        for (auto& kv : keys) {
            t->la.push_back(kv.first);
            t->lb.push_back(kv.second);
        }
        build_csr(t.get(), 1);
        *out = t.release();
        return GOSSIP_OK;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
}

uint32_t gossip_topology_num_nodes(const gossip_topology* t) { return t ? t->n : 0; }
uint64_t gossip_topology_num_links(const gossip_topology* t) { return t ? t->la.size() : 0; }

int gossip_topology_get_links(const gossip_topology* t, uint32_t* a, uint32_t* b) {
    if (!t) return set_error(GOSSIP_EINVAL, "NULL topology");
    if (a) std::memcpy(a, t->la.data(), t->la.size() * 4);
    if (b) std::memcpy(b, t->lb.data(), t->lb.size() * 4);
    return GOSSIP_OK;
}

uint64_t gossip_topology_num_entries(const gossip_topology* t) { return t ? t->col.size() : 0; }

int gossip_topology_get_csr(const gossip_topology* t, int64_t* row_ptr, int32_t* col,
                            uint8_t* mult) {
    if (!t) return set_error(GOSSIP_EINVAL, "NULL topology");
    if (row_ptr) std::memcpy(row_ptr, t->row_ptr.data(), t->row_ptr.size() * 8);
    if (col) std::memcpy(col, t->col.data(), t->col.size() * 4);
    if (mult) std::memcpy(mult, t->mult.data(), t->mult.size());
    return GOSSIP_OK;
}

int gossip_topology_get_degrees(const gossip_topology* t, uint32_t* peers, uint32_t* sockets) {
    if (!t) return set_error(GOSSIP_EINVAL, "NULL topology");
    if (peers) std::memcpy(peers, t->peers.data(), t->peers.size() * 4);
    if (sockets) std::memcpy(sockets, t->sockets.data(), t->sockets.size() * 4);
    return GOSSIP_OK;
}

void gossip_topology_destroy(gossip_topology* t) { delete t; }

// ---------------------------------------------------------------------------------------
// Schedule
// ---------------------------------------------------------------------------------------
static void sort_events(std::vector<gossip_gen_event>& ev, int threads) {
    if (ev.empty()) return;
    // Bucket by ~1 ms of ns, then sort buckets in parallel: O(m) + small sorts.
    int64_t lo = ev[0].ns, hi = ev[0].ns;
    for (const auto& e : ev) {
        lo = std::min(lo, e.ns);
        hi = std::max(hi, e.ns);
    }
    const int shift = 20;
    const uint64_t nb = (uint64_t)((hi - lo) >> shift) + 1;
    std::vector<uint64_t> off(nb + 1, 0);
    for (const auto& e : ev) off[((e.ns - lo) >> shift) + 1]++;
    for (uint64_t k = 0; k < nb; k++) off[k + 1] += off[k];
    std::vector<gossip_gen_event> out(ev.size());
    {
        std::vector<uint64_t> pos(off.begin(), off.end() - 1);
        for (const auto& e : ev) out[pos[(e.ns - lo) >> shift]++] = e;
    }
    parallel_for(nb, threads, [&](uint64_t b0, uint64_t b1) {
        for (uint64_t k = b0; k < b1; k++)
            std::sort(out.begin() + off[k], out.begin() + off[k + 1],
                      [](const gossip_gen_event& a, const gossip_gen_event& b) {
                          return a.ns != b.ns ? a.ns < b.ns : a.node < b.node;
                      });
    });
    ev.swap(out);
}

int gossip_schedule_create(uint32_t num_nodes, uint32_t node_seed, int64_t t_start_ns,
                           int64_t t_cut_ns, int64_t t_gen_end_ns, uint32_t id_mask,
                           int num_threads, gossip_schedule** out) {
    if (!out) return set_error(GOSSIP_EINVAL, "out is NULL");
    *out = nullptr;
    if (t_gen_end_ns <= 0 || t_gen_end_ns > t_cut_ns) t_gen_end_ns = t_cut_ns;
    try {
        const int T = std::max(1, num_threads);
        const uint64_t chunks = std::min<uint64_t>(std::max<uint32_t>(num_nodes, 1), (uint64_t)T * 8);
        std::vector<std::vector<gossip_gen_event>> parts(chunks);
        parallel_for(chunks, T, [&](uint64_t c0, uint64_t c1) {
            for (uint64_t c = c0; c < c1; c++) {
                const uint32_t lo = (uint32_t)((uint64_t)num_nodes * c / chunks);
                const uint32_t hi = (uint32_t)((uint64_t)num_nodes * (c + 1) / chunks);
                auto& P = parts[c];
                std::mt19937 rng;
                for (uint32_t v = lo; v < hi; v++) {
                    rng.seed((uint32_t)(node_seed + v));  // p2pnode.cc:41 rng.seed(rd() + id)
                    std::uniform_real_distribution<double> dist(2.0, 5.0);  // :99
                    int64_t t = 0;                        // StartGeneratingShares at t = 0
                    uint32_t g = 0;                       // sharesGenerated
                    for (;;) {
                        t += exact_scale_round(dist(rng), 1000000000ull);  // Schedule(Seconds(x))
                        if (t >= t_gen_end_ns) break;     // after PrintStatistics/StopAllNodes
                        if (t < t_start_ns) continue;     // peers.empty() branch :108-113
                        // GenerateUniqueShareId :203-208; std::hash<uint64_t> is identity.
                        const uint64_t seed = (uint64_t)v * 1000000ull + (uint64_t)g * 1000ull +
                                              (uint64_t)(t % 1000);
                        uint32_t id = (uint32_t)seed;
                        if (id_mask) id &= id_mask;
                        P.push_back(gossip_gen_event{t, v, id});
                        g++;
                    }
                }
            }
        });
        auto s = std::make_unique<gossip_schedule>();
        uint64_t total = 0;
        for (auto& p : parts) total += p.size();
        s->ev.reserve(total);
        for (auto& p : parts) {
            s->ev.insert(s->ev.end(), p.begin(), p.end());
            std::vector<gossip_gen_event>().swap(p);
        }
        sort_events(s->ev, T);
        *out = s.release();
        return GOSSIP_OK;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed building schedule");
    }
}

int gossip_schedule_from_events(uint64_t num_events, const gossip_gen_event* ev,
                                gossip_schedule** out) {
    if (!out || (num_events && !ev)) return set_error(GOSSIP_EINVAL, "NULL argument");
    *out = nullptr;
    for (uint64_t k = 0; k < num_events; k++)  // (a negative ns would also overflow hi - lo below)
        if (ev[k].ns < 0)
            return set_error(GOSSIP_EINVAL, "generation event " + std::to_string(k) + " has a negative time");
    try {
        auto s = std::make_unique<gossip_schedule>();
        s->ev.assign(ev, ev + num_events);
        int64_t lo = INT64_MAX, hi = 0;
        for (const auto& e : s->ev) {
            lo = std::min(lo, e.ns);
            hi = std::max(hi, e.ns);
        }
        if (num_events && (uint64_t)((hi - lo) >> 20) > 4 * num_events + 1024)
            std::sort(s->ev.begin(), s->ev.end(), [](const gossip_gen_event& a, const gossip_gen_event& b) {
                return a.ns != b.ns ? a.ns < b.ns : a.node < b.node;
            });  // a sparse span: the bucket sort's table would dwarf the events
        else
            sort_events(s->ev, 1);
        *out = s.release();
        return GOSSIP_OK;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
}

// ---------------------------------------------------------------------------------------
// Dump files (gossip_sim --dumpLinks / --dumpEvents), read strictly.  The reference parses its
// messages with an unchecked getline/stoul chain (Share::FromString, p2pnode.cc:13-30) that
// leaves fields uninitialised on malformed input; here every malformed line is GOSSIP_EINVAL.
// ---------------------------------------------------------------------------------------
static bool read_file(const char* path, std::string& text) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, k);
    const bool ok = !std::ferror(f);
    std::fclose(f);
    return ok;
}

// Splits `text` into lines of exactly `nf` unsigned decimal fields (<= max[i] each), separated
// by spaces or tabs; blank lines are skipped, a trailing '\r' is allowed.  Calls row(fields) for
// every line; returns "" or the error text naming the line.
static std::string parse_rows(const std::string& text, int nf, const uint64_t* max,
                              const std::function<std::string(const uint64_t*)>& row) {
    uint64_t vals[4];
    size_t pos = 0, line = 0;
    while (pos < text.size()) {
        size_t end = text.find('\n', pos);
        if (end == std::string::npos) end = text.size();
        line++;
        size_t i = pos, stop = end;
        if (stop > i && text[stop - 1] == '\r') stop--;
        int got = 0;
        for (;;) {
            while (i < stop && (text[i] == ' ' || text[i] == '\t')) i++;
            if (i >= stop) break;
            if (got == nf) return "line " + std::to_string(line) + ": more than " + std::to_string(nf) + " fields";
            uint64_t v = 0;
            const size_t d0 = i;
            while (i < stop && text[i] >= '0' && text[i] <= '9') {
                const uint64_t dig = (uint64_t)(text[i] - '0');
                if (v > (max[got] - dig) / 10) return "line " + std::to_string(line) + ": field " +
                                                       std::to_string(got + 1) + " out of range";
                v = v * 10 + dig;
                i++;
            }
            if (i == d0 || (i < stop && text[i] != ' ' && text[i] != '\t'))
                return "line " + std::to_string(line) + ": field " + std::to_string(got + 1) +
                       " is not an unsigned decimal integer";
            vals[got++] = v;
        }
        if (got != 0 && got != nf)
            return "line " + std::to_string(line) + ": " + std::to_string(got) + " field(s), expected " +
                   std::to_string(nf);
        if (got) {
            std::string e = row(vals);
            if (!e.empty()) return "line " + std::to_string(line) + ": " + e;
        }
        pos = end + 1;
    }
    return "";
}

int gossip_topology_load_links(uint32_t num_nodes, const char* path, gossip_topology** out) {
    if (!out || !path) return set_error(GOSSIP_EINVAL, "NULL argument");
    *out = nullptr;
    try {
        std::string text;
        if (!read_file(path, text)) return set_error(GOSSIP_EINVAL, std::string("cannot read ") + path);
        std::vector<uint32_t> a, b;
        const uint64_t mx[2] = {0xffffffffull, 0xffffffffull};
        const std::string err = parse_rows(text, 2, mx, [&](const uint64_t* v) -> std::string {
            if (v[0] >= num_nodes || v[1] >= num_nodes) return "node id beyond --numNodes";
            if (v[0] == v[1]) return "self-loop";
            a.push_back((uint32_t)v[0]);
            b.push_back((uint32_t)v[1]);
            return "";
        });
        if (!err.empty()) return set_error(GOSSIP_EINVAL, std::string(path) + ": " + err);
        return gossip_topology_from_links(num_nodes, a.size(), a.data(), b.data(), out);
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed reading links");
    }
}

int gossip_schedule_load_events(uint32_t num_nodes, const char* path, gossip_schedule** out) {
    if (!out || !path) return set_error(GOSSIP_EINVAL, "NULL argument");
    *out = nullptr;
    try {
        std::string text;
        if (!read_file(path, text)) return set_error(GOSSIP_EINVAL, std::string("cannot read ") + path);
        std::vector<gossip_gen_event> ev;
        const uint64_t mx[3] = {(uint64_t)INT64_MAX, 0xffffffffull, 0xffffffffull};
        const std::string err = parse_rows(text, 3, mx, [&](const uint64_t* v) -> std::string {
            if (num_nodes && v[1] >= num_nodes) return "node id beyond --numNodes";
            ev.push_back(gossip_gen_event{(int64_t)v[0], (uint32_t)v[1], (uint32_t)v[2]});
            return "";
        });
        if (!err.empty()) return set_error(GOSSIP_EINVAL, std::string(path) + ": " + err);
        return gossip_schedule_from_events(ev.size(), ev.data(), out);
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed reading events");
    }
}

uint64_t gossip_schedule_size(const gossip_schedule* s) { return s ? s->ev.size() : 0; }

int gossip_schedule_get(const gossip_schedule* s, gossip_gen_event* out) {
    if (!s || !out) return set_error(GOSSIP_EINVAL, "NULL argument");
    std::memcpy(out, s->ev.data(), s->ev.size() * sizeof(gossip_gen_event));
    return GOSSIP_OK;
}

void gossip_schedule_destroy(gossip_schedule* s) { delete s; }

// ---------------------------------------------------------------------------------------
// Report (NS_LOG_INFO text of PrintStatistics / PrintPeriodicStats)
// ---------------------------------------------------------------------------------------
static int64_t emit(const std::string& s, char* buf, uint64_t len) {
    if (buf && len) {
        const uint64_t k = std::min<uint64_t>(s.size(), len - 1);
        std::memcpy(buf, s.data(), k);
        buf[k] = 0;
    }
    return (int64_t)s.size();
}

int64_t gossip_format_statistics(uint32_t n, const uint32_t* gen, const uint32_t* recv,
                                 const uint32_t* fwd, const uint64_t* sent,
                                 const uint32_t* processed, const uint32_t* peers,
                                 const uint32_t* sockets, char* buf, uint64_t buf_len) {
    if (!gen || !recv || !fwd || !sent || !processed || !peers || !sockets)
        return set_error(GOSSIP_EINVAL, "NULL stats array");
    std::ostringstream os;
    os << "=== P2P Gossip Network Simulation Statistics ===\n";
    // uint32_t accumulators, as at p2pnetwork.cc:257-261.
    uint32_t tr = 0, tg = 0, tf = 0, ts = 0, tc = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t s32 = (uint32_t)sent[i];  // sharesSent is uint32_t (p2pnode.h:40)
        tr += recv[i]; tg += gen[i]; tf += fwd[i]; ts += s32; tc += sockets[i];
        os << "Node " << i << ": Generated " << gen[i] << ", Received " << recv[i]
           << ", Forwarded " << fwd[i] << ", Total sent " << s32 << ", Total processed "
           << processed[i] << ", Peer count " << peers[i] << ", Socket connections "
           << sockets[i] << "\n";
    }
    os << "Total shares generated: " << tg << "\n";
    os << "Total shares received: " << tr << "\n";
    os << "Total shares forwarded: " << tf << "\n";
    os << "Total shares sent: " << ts << "\n";
    os << "Total socket connections: " << tc << "\n";
    return emit(os.str(), buf, buf_len);
}

int64_t gossip_format_periodic(double t_seconds, uint32_t n, uint64_t total_gen,
                               uint64_t total_processed, uint64_t total_sockets, char* buf,
                               uint64_t buf_len) {
    std::ostringstream os;
    os << "=== Periodic Stats at " << t_seconds << "s ===\n";
    const uint32_t tg = (uint32_t)total_gen, tp = (uint32_t)total_processed,
                   tc = (uint32_t)total_sockets;
    os << "Total shares generated: " << tg << "\n";
    os << "Average shares per node: " << (n ? (uint64_t)tp / (uint64_t)n : 0) << "\n";
    os << "Total socket connections: " << tc << "\n";
    return emit(os.str(), buf, buf_len);
}

}  // extern "C"
