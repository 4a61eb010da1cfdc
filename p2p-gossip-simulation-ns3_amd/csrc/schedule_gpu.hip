// schedule_gpu.hip -- synthetic share-generation schedules generated on the GPU with a
// counter-based Philox4x32-10 stream per node (the north star's "Philox-counter share generation
// seeded per node"; gossip.h gossip_schedule_create_philox).
//
// Same rules as the reference's schedule (p2pnode.cc:91-125, 201-209), different random stream:
//   * every node's first generation event is at Now() = 0 + interval, then every interval after
//     the previous one (ScheduleNextShare, p2pnode.cc:97-104), interval = U(2,5) s;
//   * U(2,5): 2 + 3 u with u = (x0 + x1 * 2^32) / 2^64 from two 32-bit draws -- the structure of
//     libstdc++'s generate_canonical<double,53> over a 32-bit engine (with its u < 1 clamp) and
//     uniform_real_distribution -- where the reference draws x0, x1 from mt19937(seed + id)
//     (p2pnode.cc:41) and this generator draws them from Philox4x32-10 keyed by (seed, node),
//     counter = (node, block index), so any node's stream is computed independently;
//   * Seconds(interval) rounds exactly (ns-3 int64x64 half-up, like gossip_seconds_to_ns);
//   * an event is a counted generation iff t_start <= t < t_cut (and t < t_gen_end): before
//     t_start a node has no peers (p2pnode.cc:108-113), after t_cut PrintStatistics has run;
//   * shareId = (uint32)(node * 10^6 + g * 10^3 + t mod 1000), g = counted generations so far
//     (GenerateUniqueShareId, p2pnode.cc:201-209, std::hash<uint64_t> = identity).
// One thread per node counts its events, an exclusive scan gives each node its output range,
// a second pass writes (ns, node, id), and a stable radix sort on ns yields (ns, node) order.
// The mt19937 exact-stream schedule (gossip_schedule_create) stays the default everywhere;
// this one serves synthetic runs at sizes where the host stream is the setup bottleneck.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "internal.h"

using gossip::set_error;

namespace {

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            return set_error(GOSSIP_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

constexpr uint32_t kKey1 = 0x53484152u;  // "SHAR": second key word of the schedule stream

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = (uint32_t)p1;
        c[2] = n2;
        c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// ns-3 Seconds(x): round-half-up(x * 1e9) computed exactly (host twin: exact_scale_round).
__device__ int64_t seconds_to_ns_exact(double x) {
    if (x == 0.0) return 0;
    int e2 = 0;
    const double m = frexp(x, &e2);
    const uint64_t M = (uint64_t)ldexp(m, 53);
    const int sh = e2 - 53;
    const unsigned __int128 P = (unsigned __int128)M * 1000000000ull;
    unsigned __int128 q;
    if (sh >= 0) {
        q = P << sh;
    } else {
        const int s = -sh;
        if (s >= 127) return 0;
        q = P >> s;
        const unsigned __int128 rem = P - (q << s);
        if (rem >= ((unsigned __int128)1 << (s - 1))) q += 1;
    }
    return (int64_t)q;
}

// The event stream of one node: next() returns the time of the next generation event.
struct NodeStream {
    uint32_t node, seed, blk = 0, idx = 4;
    uint32_t buf[4];
    int64_t t = 0;
    __device__ NodeStream(uint32_t v, uint32_t s) : node(v), seed(s) {}
    __device__ uint32_t next32() {
        if (idx == 4) {
            buf[0] = node;
            buf[1] = blk++;
            buf[2] = 0x676f7373u;  // "goss"
            buf[3] = 0x69702d73u;  // "ip-s"
            philox4x32_10(buf, seed, kKey1);
            idx = 0;
        }
        return buf[idx++];
    }
    __device__ int64_t next() {
        const uint32_t x0 = next32(), x1 = next32();
        double u = ((double)x0 + (double)x1 * 4294967296.0) * (1.0 / 18446744073709551616.0);
        if (u >= 1.0) u = 0x1.fffffffffffffp-1;  // generate_canonical's clamp
        t += seconds_to_ns_exact(2.0 + u * 3.0);
        return t;
    }
};

struct GenArgs {
    uint32_t n, seed;
    int64_t t_start, t_end;  // counted iff t_start <= t < t_end
    const uint32_t* off;     // emit pass: output offset of each node
    uint32_t* cnt;           // count pass
    int64_t* ns;
    uint32_t* node;
    uint32_t* id;
};

template <bool EMIT>
__global__ __launch_bounds__(256) void k_philox_gen(GenArgs a) {
    const uint32_t v = blockIdx.x * 256u + threadIdx.x;
    if (v >= a.n) return;
    NodeStream st(v, a.seed);
    uint32_t g = 0;
    uint64_t o = EMIT ? a.off[v] : 0;
    for (;;) {
        const int64_t t = st.next();
        if (t >= a.t_end) break;
        if (t < a.t_start) continue;  // no peers yet: not counted, g unchanged
        if (EMIT) {
            a.ns[o] = t;
            a.node[o] = v;
            a.id[o] = (uint32_t)((uint64_t)v * 1000000ull + (uint64_t)g * 1000ull + (uint64_t)(t % 1000));
            o++;
        }
        g++;
    }
    if (!EMIT) a.cnt[v] = g;
}

__global__ void k_gather_events(const uint32_t* __restrict__ perm, const int64_t* __restrict__ ns_sorted,
                                const uint32_t* __restrict__ node, const uint32_t* __restrict__ id, uint64_t m,
                                gossip_gen_event* __restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (k >= m) return;
    const uint32_t p = perm[k];
    out[k] = gossip_gen_event{ns_sorted[k], node[p], id[p]};
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() { hipFree(p); }
};

}  // namespace

extern "C" int gossip_schedule_create_philox(uint32_t num_nodes, uint32_t seed, int64_t t_start_ns,
                                             int64_t t_cut_ns, int64_t t_gen_end_ns, int32_t device,
                                             gossip_schedule** out) {
    if (!out) return set_error(GOSSIP_EINVAL, "NULL argument");
    *out = nullptr;
    if (num_nodes == 0) return set_error(GOSSIP_EINVAL, "num_nodes must be positive");
    if (t_start_ns < 0 || t_cut_ns < t_start_ns) return set_error(GOSSIP_EINVAL, "need 0 <= t_start <= t_cut");
    // (~0.29 events per node per simulated second: the uint32 offsets hold any schedule that
    //  fits in host memory as gossip_gen_event records)
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_error(GOSSIP_EHIP, "no HIP device: the Philox schedule is generated on the GPU");
    if (device < 0 || device >= ndev) return set_error(GOSSIP_EINVAL, "bad device ordinal");
    HIP_TRY(hipSetDevice(device));
    const int64_t t_end = (t_gen_end_ns > 0 && t_gen_end_ns < t_cut_ns) ? t_gen_end_ns : t_cut_ns;
    GenArgs a{};
    a.n = num_nodes;
    a.seed = seed;
    a.t_start = t_start_ns;
    a.t_end = t_end;
    DevBuf cnt, off, tmp, ns, node, id, ns2, perm, perm2, evd;
    const uint32_t grid = (num_nodes + 255u) / 256u;
    HIP_TRY(hipMalloc(&cnt.p, ((size_t)num_nodes + 1) * 4));
    HIP_TRY(hipMalloc(&off.p, ((size_t)num_nodes + 1) * 4));
    HIP_TRY(hipMemset(cnt.p, 0, ((size_t)num_nodes + 1) * 4));
    a.cnt = static_cast<uint32_t*>(cnt.p);
    k_philox_gen<false><<<grid, 256>>>(a);
    HIP_TRY(hipGetLastError());
    size_t tmpb = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmpb, static_cast<uint32_t*>(cnt.p),
                                             static_cast<uint32_t*>(off.p), (int)num_nodes + 1));
    HIP_TRY(hipMalloc(&tmp.p, std::max<size_t>(tmpb, 1)));
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(tmp.p, tmpb, static_cast<uint32_t*>(cnt.p),
                                             static_cast<uint32_t*>(off.p), (int)num_nodes + 1));
    uint32_t m32 = 0;
    HIP_TRY(hipMemcpy(&m32, static_cast<uint32_t*>(off.p) + num_nodes, 4, hipMemcpyDeviceToHost));
    const uint64_t m = m32;
    auto s = std::unique_ptr<gossip_schedule>(new (std::nothrow) gossip_schedule());
    if (!s) return set_error(GOSSIP_ENOMEM, "host allocation failed");
    if (m) {
        HIP_TRY(hipMalloc(&ns.p, m * 8));
        HIP_TRY(hipMalloc(&node.p, m * 4));
        HIP_TRY(hipMalloc(&id.p, m * 4));
        a.off = static_cast<const uint32_t*>(off.p);
        a.ns = static_cast<int64_t*>(ns.p);
        a.node = static_cast<uint32_t*>(node.p);
        a.id = static_cast<uint32_t*>(id.p);
        k_philox_gen<true><<<grid, 256>>>(a);
        HIP_TRY(hipGetLastError());
        // stable sort by time: events are node-major, so equal times stay in node order
        HIP_TRY(hipMalloc(&ns2.p, m * 8));
        HIP_TRY(hipMalloc(&perm.p, m * 4));
        HIP_TRY(hipMalloc(&perm2.p, m * 4));
        std::vector<uint32_t> iota(m);
        for (uint64_t k = 0; k < m; k++) iota[k] = (uint32_t)k;
        HIP_TRY(hipMemcpy(perm.p, iota.data(), m * 4, hipMemcpyHostToDevice));
        size_t sb = 0;
        auto* kin = reinterpret_cast<unsigned long long*>(ns.p);
        auto* kout = reinterpret_cast<unsigned long long*>(ns2.p);
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, kin, kout, static_cast<uint32_t*>(perm.p),
                                                   static_cast<uint32_t*>(perm2.p), (int)m));
        DevBuf sortmp;
        HIP_TRY(hipMalloc(&sortmp.p, std::max<size_t>(sb, 1)));
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(sortmp.p, sb, kin, kout, static_cast<uint32_t*>(perm.p),
                                                   static_cast<uint32_t*>(perm2.p), (int)m));
        HIP_TRY(hipMalloc(&evd.p, m * sizeof(gossip_gen_event)));
        k_gather_events<<<(uint32_t)((m + 255) / 256), 256>>>(static_cast<uint32_t*>(perm2.p),
                                                               static_cast<int64_t*>(ns2.p),
                                                               static_cast<uint32_t*>(node.p),
                                                               static_cast<uint32_t*>(id.p), m,
                                                               static_cast<gossip_gen_event*>(evd.p));
        HIP_TRY(hipGetLastError());
        try {
            s->ev.resize(m);
        } catch (const std::bad_alloc&) {
            return set_error(GOSSIP_ENOMEM, "host allocation failed");
        }
        HIP_TRY(hipMemcpy(s->ev.data(), evd.p, m * sizeof(gossip_gen_event), hipMemcpyDeviceToHost));
    }
    HIP_TRY(hipDeviceSynchronize());
    *out = s.release();
    return GOSSIP_OK;
}
