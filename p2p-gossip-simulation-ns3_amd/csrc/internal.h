// internal.h -- shared host-side types of libgossip.so (not part of the C ABI).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "gossip.h"

namespace gossip {

// Sets the thread-local error text returned by gossip_last_error(); returns `code`.
int set_error(int code, const std::string& msg);

// ns-3 int64x64 conversion: round-half-up(x * factor) computed exactly.
int64_t exact_scale_round(double x, uint64_t factor);

// Run f(lo, hi) over [0, n) split across `threads` std::threads (threads <= 1: inline).
template <class F>
void parallel_for(uint64_t n, int threads, F&& f);

}  // namespace gossip

// Opaque ABI objects (definitions shared by host.cpp and engine.hip).
struct gossip_topology {
    uint32_t n = 0;
    std::vector<uint32_t> la, lb;  // map keys (a,b) in std::map order
    std::vector<int64_t> row_ptr;  // CSR over distinct neighbours
    std::vector<int32_t> col;
    std::vector<uint8_t> mult;     // multiplicity of col in peers(row): 1 or 2
    std::vector<uint32_t> peers;   // |peers(v)| including duplicates
    std::vector<uint32_t> sockets; // |peersockets(v)| = distinct peers
    // connected-component labels, built on first use by gossip_shard_events (guarded there)
    mutable std::vector<uint32_t> comp;
};

struct gossip_schedule {
    std::vector<gossip_gen_event> ev;  // sorted by (ns, node)
};

namespace gossip {
// Builds row_ptr/col/mult/peers/sockets from la/lb.
int build_csr(gossip_topology* t, int threads);

// Connected-component label (smallest node id of the component) of every node.
std::vector<uint32_t> components(uint32_t n, const int64_t* row_ptr, const int32_t* col);

// Share-instance key -> 64-bit hash used for multi-GPU sharding.  An instance is one
// shareId inside one connected component; a lone generation of an id is keyed by
// (id, node) so that no component labelling is needed when no id collides.
uint64_t instance_hash(uint32_t share_id, uint32_t node_or_comp, bool lone);
// The topology's component labels, built once and cached on it (thread-safe).
const std::vector<uint32_t>& topology_components(const gossip_topology* t);
// Copies the cached labels into *out when an earlier call built them.
bool cached_topology_components(const gossip_topology* t, std::vector<uint32_t>* out);

// True if any two events share an id.
bool any_id_collision(uint64_t m, const gossip_gen_event* ev);
}

#include <thread>
namespace gossip {
template <class F>
void parallel_for(uint64_t n, int threads, F&& f) {
    if (threads <= 1 || n < 2) {
        f((uint64_t)0, n);
        return;
    }
    if ((uint64_t)threads > n) threads = (int)n;
    std::vector<std::thread> pool;
    pool.reserve(threads);
    for (int k = 0; k < threads; k++) {
        const uint64_t lo = n * (uint64_t)k / (uint64_t)threads;
        const uint64_t hi = n * (uint64_t)(k + 1) / (uint64_t)threads;
        pool.emplace_back([&f, lo, hi] { f(lo, hi); });
    }
    for (auto& t : pool) t.join();
}
}  // namespace gossip
