// engine.hip -- MI355X (gfx950) tick-synchronous gossip engine behind the C ABI of gossip.h.
//
// Replaces the reference's per-packet hot path (P2PNode::HandleRead -> seen-set check ->
// ReceiveShare -> GossipShareToPeers, p2pnode.cc:127-199) with one bulk step per tick
// (tick = --Latency, the PointToPoint channel Delay of p2pnetwork.cc:114):
//
//   F_t[v]   = frontier: live share columns node v emitted (received or generated) in tick t
//   inc[v]   = OR_{u in peers(v)} F_t[u]            (every emission reaches every peer, :129)
//   new[v]   = inc[v] & ~seen[v]                      (processedShares check, :189)
//   seen[v] |= new[v];  F_{t+1}[v] = new[v] | births  (ReceiveShare inserts + forwards, :155-165)
//   recv[v] += popcount(new[v]); sent[v] += |peers(v)| * popcount(new[v])
//
// sent is stored as the births' sends only (k_births): every reception forwards |peers(v)| copies
// (p2pnode.cc:163 -> :129-146), so sent = d_sent + deg x recv, formed where sent is read
// (gossip_engine_get_stats, k_sum_sent) -- the pull kernels then never load a node's |peers|.
//
// HBM layout (row-major, node rows): F0, F1, seen are n x stride uint64 words; bit b of word w
// is share column 64w+b.  A column is one share source; shares whose 32-bit ids collide
// (GenerateUniqueShareId, p2pnode.cc:201-209, collides above ~128,849 nodes) and that live in
// one connected component form a "group": adjacent bits of one word, ordered by generation
// phase, sharing one seen-set entry (the reference keys processedShares by id only).
//
// Kernels:
//   k_pull   -- CSR pull over the bit-sliced frontier (HBM-bound: one neighbour row read per
//               edge per tick, 16 B per lane, coalesced), seen/dedup, counters, liveness.
//   k_births -- source injection (GenerateAndGossipShare, p2pnode.cc:106-125), including the
//               same-tick "own generation vs arrival" rule for id groups.
//   k_reduce -- counter reductions for snapshots / totals.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <numeric>
#include <queue>
#include <string>
#include <chrono>
#include <thread>
#include <type_traits>
#include <unordered_map>
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

// gossip_engine_abort: seconds to wait for a collective being enqueued before aborting anyway
constexpr int kAbortWaitS = 10;
// A collective being enqueued on an engine's communicator (COMM_TRY, gossip_engine_abort)
struct CommIssue {
    std::atomic<int>& c;
    explicit CommIssue(std::atomic<int>& x) : c(x) { c.fetch_add(1); }
    ~CommIssue() { c.fetch_sub(1); }
};

// Per-word control for one tick (host-built, uploaded each tick).
struct WordCtl {
    uint64_t clear;   // seen bits to clear before use (word re-allocated this tick)
    uint64_t keep;    // columns that may receive this tick (phase cut at t_cut)
    uint64_t gmask;   // bits that belong to multi-source id groups
    uint64_t gstart;  // first bit of each group
    uint64_t snap;    // columns whose arrivals count toward the snapshot partial
};

enum : uint32_t { BIRTH_NOOP = 0, BIRTH_NORMAL = 1, BIRTH_GROUP = 2, BIRTH_LOST = 3 };
enum : uint32_t { BF_CONN = 1u };  // Birth::flags: before REGISTER, |peers| = connector-side keys

struct Birth {
    uint32_t node;
    uint32_t col;    // word*64 + bit
    int32_t phase;   // ns % L of the generation
    uint32_t kind;   // BIRTH_*
    uint32_t glo;    // group: first bit in word
    uint32_t glen;   // group: number of bits
    uint32_t poff;   // group: offset of member phases in the per-tick phase buffer
    uint32_t flags;  // BF_*
    uint32_t widx;   // write-sparse index of the birth's tile this tick (0xff: dense tile)
    uint32_t yid;    // young id of that tile (its seen-list entries, young_kernel.h)
};

struct PullArgs {
    const int64_t* rowptr;
    const int32_t* col;
    const uint64_t* Fcur;
    uint64_t* Fnext;
    uint64_t* seen;
    const WordCtl* ctl;     // masks, read only for words whose wflags say so
    const uint8_t* wflags;  // per word: WF_CLEAR | WF_GROUP | WF_KEEP | WF_SNAP
    uint32_t* recv;
    // (no sent: derived from recv, header comment)
    unsigned long long* live;             // liveness of this tick (OR of F_next words)
    const unsigned long long* live_prev;  // liveness of tick t-1 (nullable: all live)
    unsigned long long* snap;             // nullable
    unsigned long long* acct;             // traffic accounting (nullable)
    uint32_t n;
    uint32_t stride;
    uint32_t wbase;  // this launch covers words [wbase, wbase + wact) of every row
    uint32_t wact;
    uint32_t noskip;  // diagnostic: read every peer-row word (dense pull, known byte count)
    unsigned long long* inc;  // DENSE mode: incoming words from the MFMA GEMM (read + zeroed)
    // Tile occupancy of the frontier (CSR mode; null = legacy zero-filled F rows): bit
    // (tile & 63) of word [u * ntw + tile / 64] says F[u]'s 16-word tile row holds a bit.
    // Rows whose bit is clear are never read, so they are never zero-filled either.
    const unsigned long long* nz_cur;
    unsigned long long* nz_next;
    uint32_t ntw;
    uint32_t v0 = 0;  // first node of this engine's row range (row partition; multiple of 64)
    // 1: another kernel (k_pull_young) runs concurrently and shares the per-node outputs, so
    // counters are added and occupancy bits OR'ed atomically (nz_next zeroed beforehand)
    uint32_t shared_out = 0;
    uint32_t keep_lds = 0;  // some word of the launch has WF_KEEP: masks staged in LDS (k_pull)
    uint32_t gate_seen = 1;  // k_pull<LPW,1>: skip the own-seen loads of tiles no peer occupies
    // Pass -> tile map (option pull_tiles): a k_pull pass covers LPW / 8 tiles taken from this
    // list of launch-local tile indices (0xffff = padding) instead of LPW / 8 consecutive tiles,
    // so passes skip tiles that hold nothing for k_pull (young, retired); every group of LPW / 8
    // entries lies in one occupancy word.  Null: consecutive tiles.
    const uint16_t* ptile = nullptr;
    uint32_t nptile = 0;
    // Saturated tiles and dense-row tiles (k_pull<LPW,1> over tile lists; pull_kernel.h): per node
    // and occupancy word, bit (tile & 63) = every live column of the tile is in the node's seen
    // words (null: off); tmask[TM_WORDS * tw + TM_*] the tick's per-occupancy-word tile masks.
    unsigned long long* sat = nullptr;
    const unsigned long long* tmask = nullptr;
    // Push marks (round 6, option pull_push; pull_kernel.h): bit v of mark_cur says some peer of v
    // wrote a non-empty F_cur row of a TM_PUSH tile (the tiles whose frontier the host expects on
    // few nodes); this tick's rows of TM_PUSHW tiles mark their writer's peers in mark_next.
    const unsigned long long* mark_cur = nullptr;
    unsigned long long* mark_next = nullptr;
};

// Phase-ordered update of id groups inside one word (rare: only words holding groups).
// Groups are contiguous bit ranges in phase order; a node's first contact with the id is
// the lowest-phase arrival, and nothing arrives once any member bit is already seen.
// The id group holding bit b of gm (groups: contiguous runs of gm, each starting at a bit of gs)
__device__ __forceinline__ uint64_t group_of(uint32_t b, uint64_t gm, uint64_t gs) {
    const uint64_t below = gs & (b == 63u ? ~0ull : ((2ull << b) - 1ull));  // starts at or below b
    const uint32_t s = 63u - (uint32_t)__builtin_clzll(below);
    const uint64_t above = gs & (s == 63u ? 0ull : ~((2ull << s) - 1ull));  // starts after s
    const uint64_t upto = above ? ((above & (~above + 1ull)) - 1ull) : ~0ull;
    return gm & upto & ~((1ull << s) - 1ull);
}
// Only the groups holding an incoming bit can change `nw` (a group with none keeps none, seen or
// not), so the loop visits those -- not every group of the word
__device__ __forceinline__ uint64_t group_fix(uint64_t nw, uint64_t seen, uint64_t gm,
                                              uint64_t gs) {
    uint64_t todo = nw & gm;
    while (todo) {
        const uint64_t grp = group_of((uint32_t)__builtin_ctzll(todo), gm, gs);
        if (seen & grp) {
            nw &= ~grp;
        } else {
            const uint64_t x = nw & grp;
            nw = (nw & ~grp) | (x & (~x + 1ull));
        }
        todo &= ~grp;
    }
    return nw;
}

// Traffic accounting counters (acct): kAcctSlots counters, replicated kAcctReplicas times on
// separate 128-B lines and summed on the host.  Every wave adds its own counts at its end; with a
// single copy, thousands of waves finishing together queue their atomics on ONE L2 line and wait
// for them at the next barrier (k_dense_dedup: 4,096 waves x 3 atomics = ~100 us per C2 dispatch).
constexpr uint32_t kAcctSlots = 40, kAcctReplicas = 64;
__device__ __forceinline__ void acct_add(unsigned long long* acct, uint32_t slot, unsigned long long v) {
    atomicAdd(&acct[(blockIdx.x & (kAcctReplicas - 1u)) * kAcctSlots + slot], v);
}

// The index of the calling wave in its block, as a wave-uniform (scalar) value: the compiler's
// uniformity analysis treats threadIdx.x >> 6 as divergent, which put every per-wave node index
// and row address derived from it in VGPR pairs (64-bit VALU arithmetic, registers held across
// the kernels' node loops).
__device__ __forceinline__ uint32_t wave_in_block() {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

// x, recomputed where it is used: an empty asm that "modifies" x keeps the compiler from hoisting
// lane-derived values (slot offsets, shuffle addresses, spare words) out of the kernels' item loops,
// where dozens of them stayed live across the whole loop and set the register counts (k_pull_young
// 125 -> 64 VGPRs)
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}

// Lane `src` of v (ds_bpermute), its address computed from the caller's `lane`: HIP's __shfl
// derives the address from its own lane-id read, which the compiler hoists out of the kernels'
// loops, one live register per distinct source expression.
__device__ __forceinline__ uint32_t lane_get(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v);
}
// v of lane `src`, src wave-uniform (v_readlane: no LDS trip; reads inactive lanes too)
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)src);
}
// Sum over the wave (every lane active), wave-uniform: DPP inside each row of 16, then 4 reads.
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // lane ^ 1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // lane ^ 2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // other quad of 8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);  // other 8 of 16
    return lane_read(x, 0) + lane_read(x, 16) + lane_read(x, 32) + lane_read(x, 48);
}

#include "pull_kernel.h"
#include "dense_kernel.h"
#include "young_kernel.h"

// Bitmaps above this size run k_pull<LPW,1> with non-temporal row accesses (pull_kernel.h).
// The size is the launch's LIVE footprint, n x wact words (not the allocated capacity, which
// depends on how much headroom the device had free at allocation time).
constexpr uint64_t kPullNtBytes = 16ull << 30;

// Environment defaults of the per-engine tuning options (gossip_engine_set_option overrides
// them per engine; A/B runs and tests).
int64_t env_option(const char* name, int64_t dflt) {
    const char* e = std::getenv(name);
    return e && *e ? (int64_t)std::atoll(e) : dflt;
}

// Cap on the pull's blocks per launch (4 waves each, striding over 64-node chunks).  Measured
// (profiles/r01/grid_ab.jsonl, grid_ab2.jsonl): non-temporal (> 16 GiB) bitmaps like finer
// work units -- C4 121.4 -> 119.5 ms per launch at 16,384 blocks, its 8-rank share 37.3 -> 36.3
// ms -- while cache-resident ones kept 2,048 (C3 2.91 ms vs 3.06 ms at 16,384).  Round 3, with
// 5 waves per SIMD: C3 2.64 ms at 2,048, 2.55 at 4,096, 2.55 at 8,192, 2.69 at 1,024 blocks
// (profiles/r03/ab/r3c3_*), so cache-resident bitmaps get 4,096.
uint64_t pull_grid_cap(bool nt, int64_t ov) {
    if (ov > 0) return (uint64_t)ov;
    return nt ? 16384ull : 4096ull;
}

// Word-lanes per node of the sparse pull for windows wider than 64 words: 32 (passes of 64 words,
// two nodes per wave step: twice the independent peer chains per wave, and a window never ends in
// a half-idle 128-word pass).  Measured against 64 lanes (profiles/r01/lanes_ab.json: C4 1216
// words 127.7 -> 121.9 ms per launch, the 8-shard 320 words 44.0 -> 36.5 ms, C3 3.35 -> 3.06 ms),
// 16 lanes (C4 128.0 ms) and again in round 4 (64 lanes: C4 phase 69.0 vs 60.4 ms,
// profiles/r04/ab/r4l_*); the option that selected them was removed in round 5.
constexpr int kWideLanes = 32;

bool pull_sp(int lpw, int epn, const PullArgs& a);
template <int LPW, int EPN>
void launch_pull_t(bool nt, uint32_t grid, size_t lds, hipStream_t s, const PullArgs& a) {
    if constexpr (LPW == 32 && EPN == 1) {
        if (pull_sp(LPW, EPN, a)) {
            // push marks in their own instantiation (the other one keeps its register allocation)
            const bool push = a.mark_cur != nullptr || a.mark_next != nullptr;
            if (nt && push)
                k_pull<LPW, 1, true, true, true><<<grid, 256, lds, s>>>(a);
            else if (nt)
                k_pull<LPW, 1, true, true><<<grid, 256, lds, s>>>(a);
            else if (push)
                k_pull<LPW, 1, false, true, true><<<grid, 256, lds, s>>>(a);
            else
                k_pull<LPW, 1, false, true><<<grid, 256, lds, s>>>(a);
            return;
        }
    }
    if constexpr ((LPW == 64 || LPW == 32 || LPW == 16) && EPN == 1) {
        if (nt) {
            k_pull<LPW, 1, true><<<grid, 256, lds, s>>>(a);
            return;
        }
    }
    if constexpr (LPW * EPN <= 64) k_pull<LPW, EPN><<<grid, 256, lds, s>>>(a);
}

// the flags k_pull<.., SP = true> takes as compile-time constants (pull_kernel.h): the same
// conditions the kernel derives at run time.  Push marks (PullArgs::mark_*) run only there.
bool pull_sp(int lpw, int epn, const PullArgs& a) {
    return lpw == 32 && epn == 1 && a.tmask != nullptr && a.ptile != nullptr && a.sat != nullptr &&
           a.nptile / (uint32_t)(lpw / 8) <= kPullMaxPasses && !a.noskip && a.gate_seen;
}

template <int LPW>
void launch_pull_e(int epn, bool nt, uint32_t grid, size_t lds, hipStream_t s, const PullArgs& a) {
    switch (epn) {
        case 1: launch_pull_t<LPW, 1>(nt, grid, lds, s, a); break;
        case 2: launch_pull_t<LPW, 2>(nt, grid, lds, s, a); break;
        case 4: launch_pull_t<LPW, 4>(nt, grid, lds, s, a); break;
        case 8: launch_pull_t<LPW, 8>(nt, grid, lds, s, a); break;
        default: launch_pull_t<LPW, 8>(nt, grid, lds, s, a); break;
    }
}

// (LPW, EPN) with 8 <= LPW, LPW * EPN <= 64, both powers of two.
void launch_pull(int lpw, int epn, bool nt, uint32_t grid, size_t lds, hipStream_t s, const PullArgs& a) {
    switch (lpw) {  // lpw >= 8: one tile's 8 word-pairs sit in one lane group
        case 8: launch_pull_e<8>(epn, nt, grid, lds, s, a); break;
        case 16: launch_pull_e<16>(epn, nt, grid, lds, s, a); break;
        case 32: launch_pull_e<32>(epn, nt, grid, lds, s, a); break;
        default: launch_pull_e<64>(epn, nt, grid, lds, s, a); break;
    }
}

// GOSSIP_MODE_AUTO: the int8-MFMA contraction when the graph is dense enough that streaming its
// bit adjacency (n^2/8 bytes per tick) beats gathering 128-B frontier rows per edge
// (~16 B per (edge, word pair)): measured crossover in profiles/r02/auto_mode.jsonl -- p = 0.3
// graphs at n = 4,096 - 65,536 run 5-19x faster on MFMA.  Needs the adjacency to fit in HBM
// (n <= 2^19 here), and the handshake window's connector-only CSR has no MFMA form.
bool auto_dense(uint32_t n, uint64_t nnz, bool handshake) {
    if (handshake || n < 2048 || n > (1u << 19)) return false;
    return (double)nnz >= 0.05 * (double)n * (double)n;
}

struct BirthArgs {
    const Birth* b;
    uint32_t nb;
    const int32_t* gphase;
    uint64_t* Fnext;
    uint64_t* seen;
    uint32_t stride;
    uint32_t* gen;
    uint32_t* recv;
    uint32_t* effgen;
    uint64_t* sent;
    const uint32_t* deg;
    unsigned long long* live;
    unsigned long long* snap;  // nullable
    int64_t snap_r;            // snapshot phase threshold (valid when snap != null)
    unsigned long long* nz;    // tile occupancy of Fnext (nullable: legacy zero-filled rows)
    uint32_t ntw;
    const uint32_t* degc;      // handshake window: connector-side |peers| (read only with BF_CONN)
    uint16_t* slot;            // young tiles: F_next slots (young_kernel.h); null when off
    uint32_t cap;              // slot capacity (entries)
    const uint32_t* wt;        // write-sparse index -> tile, this tick
    uint32_t nwt;
    // a birth that gives its node's slot a second line announces it (young_kernel.h hints)
    const int64_t* rowptr;
    const int32_t* rev;
    uint8_t* hint_next;
    uint32_t stamp_next;
    uint32_t stamp1_next;      // sparse_wr: a birth that makes its slot non-empty stamps it too
    // push marks (pull_kernel.h): a birth into a push-write tile (tmask TM_PUSHW) marks its node's
    // peers, as k_pull does for the rows it writes (null: no push-write tile this tick)
    unsigned long long* mark_next;
    const unsigned long long* tmask;
    const int32_t* col;
    uint32_t sparse_wr;
    uint16_t* list;            // young tiles: seen lists (young_kernel.h)
    const uint8_t* wt_yid;     // write-sparse index -> young id, this tick
    uint32_t list_max;         // entries a list holds (kListU16 - 1; option young_list_cap)
    // fused DENSE tick (k_dense_fused): a birth also sets its bit in the transposed F_next and the
    // (column tile, K stage) bit of its stage mask (null otherwise)
    uint32_t* FTn = nullptr;
    unsigned long long* snz_n = nullptr;
    uint32_t kw = 0, nstw = 0;
};

// Seen-list entries [lo, hi] of node list ls in young id yid, word wit (bits of word w)
__device__ uint64_t list_word_bits(const uint16_t* ls, uint32_t lo, uint32_t hi, uint32_t yid, uint32_t wit) {
    uint64_t r = 0ull;
    for (uint32_t k = lo; k <= hi; k++) {
        const uint32_t e = ls[k];
        if (e != kSlotTomb && (e >> 10) == yid && ((e >> 6) & 15u) == wit) r |= 1ull << (e & 63u);
    }
    return r;
}

// A seen list that cannot take a birth's entries: its entries become the dense seen rows of the
// tiles young next tick (this tick's write-sparse ones), and the header says so (young_kernel.h)
__device__ void list_spill(const BirthArgs& a, uint64_t v, uint16_t* ls) {
    const uint32_t tot = ls[0] & 127u;
    for (uint32_t q = 0; q < a.nwt; q++) {
        uint64_t* row = a.seen + v * a.stride + (uint64_t)a.wt[q] * 16u;
        for (uint32_t k = 0; k < 16; k++) row[k] = list_word_bits(ls, 1, tot, a.wt_yid[q], k);
    }
    ls[0] = (uint16_t)kListOverflow;
}

// Young-tile slot of a birth's node: the arrival bits of the group mask gm in word w (from the
// slot entries; k_pull_young wrote them this tick), optionally tombstoning those entries.
__device__ uint64_t slot_word_bits(uint16_t* s, uint32_t hdr, uint32_t widx, uint32_t wit, uint64_t gm,
                                   bool remove) {
    uint64_t r = 0ull;
    for (uint32_t k = 1; k <= hdr; k++) {
        const uint32_t e = s[k];
        if (e == kSlotTomb || (e >> 10) != widx || ((e >> 6) & 15u) != wit) continue;
        const uint64_t b = 1ull << (e & 63u);
        if (!(b & gm)) continue;
        r |= b;
        if (remove) s[k] = (uint16_t)kSlotTomb;
    }
    return r;
}

// A slot that cannot take one more entry: expand it into dense rows of every write-sparse tile
// (zeros included -- readers of an overflowed node read those rows without occupancy bits).
__device__ void slot_spill(const BirthArgs& a, uint64_t v, uint16_t* s, uint32_t hdr) {
    for (uint32_t q = 0; q < a.nwt; q++) {
        uint64_t* row = a.Fnext + v * a.stride + (uint64_t)a.wt[q] * 16u;
        for (uint32_t k = 0; k < 16; k++) row[k] = 0ull;
    }
    for (uint32_t k = 1; k <= hdr; k++) {
        const uint32_t e = s[k];
        if (e == kSlotTomb || (e >> 10) >= a.nwt) continue;
        a.Fnext[v * a.stride + (uint64_t)a.wt[e >> 10] * 16u + ((e >> 6) & 15u)] |= 1ull << (e & 63u);
    }
    s[0] = (uint16_t)kSlotOverflow;
}

// GenerateAndGossipShare (p2pnode.cc:106-125): gen++, insert, send to all peers -- sends and
// the generation count happen even when the id is already in processedShares.  At most one
// birth per node per tick (generation intervals are >= 2 s, latency < 2 s).
__global__ __launch_bounds__(256) void k_births(BirthArgs a) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.nb) return;
    const Birth x = a.b[i];
    const uint64_t v = x.node;
    const uint32_t dv = a.deg[v];
    a.gen[v] += 1u;
    a.sent[v] += (x.flags & BF_CONN) ? a.degc[v] : dv;  // :129-146, peers at this instant
    if (x.kind == BIRTH_NOOP) return;
    if (x.kind == BIRTH_LOST) {  // sent behind the REGISTER segment (:178): lost, id processed
        a.effgen[v] += 1u;
        return;
    }
    const uint32_t w = x.col >> 6;
    const uint64_t bit = 1ull << (x.col & 63u);
    uint64_t* fp = a.Fnext + v * a.stride + w;
    uint64_t* sp = a.seen + v * a.stride + w;
    if (x.widx != 0xffu && a.slot) {
        // young tile (young_kernel.h): F_next of this node is its slot, unless overflowed; its
        // processedShares bits are in its seen list, unless that overflowed
        uint16_t* s = a.slot + v * kSlotU16;
        uint32_t hdr = s[0];
        const bool ovf = hdr == kSlotOverflow;
        uint16_t* ls = a.list + v * kListU16;
        const uint32_t lh = ls[0];
        const bool lovf = lh == kListOverflow;
        bool eff = true;
        uint64_t arr = 0ull;
        const uint64_t gm = x.kind == BIRTH_GROUP ? (x.glen >= 64 ? ~0ull : ((1ull << x.glen) - 1ull)) << x.glo : 0ull;
        if (x.kind == BIRTH_GROUP) {
            arr = ovf ? (*fp & gm) : slot_word_bits(s, hdr, x.widx, w & 15u, gm, false);
            // (the list's entries up to `kept` predate this tick; this tick's arrivals follow)
            const uint64_t prior = lovf ? (*sp & gm) & ~arr : list_word_bits(ls, 1, lh >> 7, x.yid, w & 15u) & gm;
            if (prior) {
                eff = false;
            } else if (arr) {
                const int ab = __ffsll((long long)arr) - 1;
                const int32_t aph = a.gphase[x.poff + (uint32_t)ab - x.glo];
                if (aph < x.phase) {
                    eff = false;
                } else {
                    if (ovf) *fp &= ~arr;
                    else slot_word_bits(s, hdr, x.widx, w & 15u, arr, true);
                    a.recv[v] -= 1u;  // (and its deg sends: sent is derived from recv)
                    if (a.snap && aph < a.snap_r) atomicAdd(a.snap, (unsigned long long)-1ll);
                }
            }
        }
        if (!eff) return;
        if (!ovf && hdr >= a.cap) {
            slot_spill(a, v, s, hdr);
            hdr = kSlotOverflow;
        }
        if (hdr == kSlotOverflow) {
            *fp |= bit;
        } else {
            s[1 + hdr] = (uint16_t)((x.widx << 10) | ((w & 15u) << 6) | (x.col & 63u));
            s[0] = (uint16_t)(hdr + 1u);
            if (1u + hdr == 64u) {  // the first entry of the second line: the rest of it is
                for (uint32_t k = 65; k < kSlotU16; k++) s[k] = (uint16_t)kSlotTomb;  // tombstones
                if (a.hint_next)  // and the readers of the next tick load it
                    for (int64_t j = a.rowptr[v]; j < a.rowptr[v + 1]; j++)
                        if (a.rev[j] >= 0) a.hint_next[a.rev[j]] = (uint8_t)a.stamp_next;
            } else if (hdr == 0u && a.sparse_wr && a.hint_next) {  // (young_kernel.h, empty-slot
                for (int64_t j = a.rowptr[v]; j < a.rowptr[v + 1]; j++)  //  skipping: now non-empty)
                    if (a.rev[j] >= 0) a.hint_next[a.rev[j]] = (uint8_t)a.stamp1_next;
            }
        }
        if (lovf) {
            *sp |= bit;
        } else {
            // the list takes the bit -- a group's every bit (lists hold whole groups), unless this
            // tick's arrival of the group already put them there
            const uint64_t add = x.kind == BIRTH_GROUP ? (arr ? 0ull : gm) : bit;
            uint32_t tot = lh & 127u;
            if (tot + (uint32_t)__popcll(add) > a.list_max) {
                list_spill(a, v, ls);
                *sp |= add;
            } else {
                for (uint64_t m = add; m; m &= m - 1ull)
                    ls[1 + tot++] = (uint16_t)((x.yid << 10) | ((w & 15u) << 6) | (uint32_t)__builtin_ctzll(m));
                ls[0] = (uint16_t)list_header(lh >> 7, tot);
            }
        }
        a.effgen[v] += 1u;
        atomicOr(&a.live[w], (unsigned long long)bit);
        if (a.snap && x.phase < a.snap_r) atomicAdd(a.snap, 1ull);
        return;
    }
    // Tile occupancy: a tile row the pull did not write this tick holds stale bits (it is
    // only ever read behind its occupancy bit), so the birth writes the whole row.
    const uint32_t tile = w >> 4;
    unsigned long long* nzp = a.nz ? a.nz + v * a.ntw + (tile >> 6) : nullptr;
    const unsigned long long tbit = 1ull << (tile & 63u);
    const bool fresh = nzp && (*nzp & tbit) == 0ull;
    bool eff = true;
    if (x.kind == BIRTH_GROUP) {
        const uint64_t gm = (x.glen >= 64 ? ~0ull : ((1ull << x.glen) - 1ull)) << x.glo;
        const uint64_t arr = fresh ? 0ull : (*fp & gm);
        const uint64_t prior = (*sp & gm) & ~arr;
        if (prior) {
            eff = false;  // id already in processedShares before this tick
        } else if (arr) {
            const int ab = __ffsll((long long)arr) - 1;
            const int32_t aph = a.gphase[x.poff + (uint32_t)ab - x.glo];
            if (aph < x.phase) {
                eff = false;  // the arrival came first in this tick
            } else {
                // Own generation first (ties: the generation event was scheduled earlier):
                // the arrival finds the id already processed and is dropped.
                *fp &= ~arr;
                a.recv[v] -= 1u;  // (and its deg sends: sent is derived from recv)
                if (a.snap && aph < a.snap_r) atomicAdd(a.snap, (unsigned long long)-1ll);
            }
        }
    }
    if (eff) {
        if (fresh) {
            ulonglong2* row = reinterpret_cast<ulonglong2*>(a.Fnext + v * a.stride + (w & ~15u));
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t w0 = (w & ~15u) + 2u * q;
                row[q] = make_ulonglong2(w0 == w ? bit : 0ull, w0 + 1u == w ? bit : 0ull);
            }
            *nzp |= tbit;  // one birth per node per tick: no other writer of this word
        } else {
            *fp |= bit;
        }
        if (a.mark_next && ((a.tmask[(uint64_t)TM_WORDS * (tile >> 6) + TM_PUSHW] >> (tile & 63u)) & 1ull))
            for (int64_t j = a.rowptr[v]; j < a.rowptr[v + 1]; j++) {
                const uint32_t u = (uint32_t)a.col[j];
                atomicOr(&a.mark_next[u >> 6], 1ull << (u & 63u));
            }
        *sp |= bit;
        a.effgen[v] += 1u;
        atomicOr(&a.live[w], (unsigned long long)bit);
        if (a.snap && x.phase < a.snap_r) atomicAdd(a.snap, 1ull);
        if (a.FTn) {
            atomicOr(&a.FTn[(uint64_t)x.col * a.kw + (v >> 5)], 1u << (v & 31u));
            const uint32_t st = (uint32_t)(v >> 10);  // 1,024-node K stage
            atomicOr(&a.snz_n[(uint64_t)(x.col >> 8) * a.nstw + (st >> 6)], 1ull << (st & 63u));
        }
    }
}

// Hop-batched snapshots: out[2 + 2s + 1] += popcount(F[v][w] & mask[s][w]) over the frontier
// rows whose tile occupancy bit is set (other rows hold stale bits).  mask[s] holds the columns
// whose arrival in this batched tick happened before snapshot s in real time (hop >= 1).
constexpr uint32_t kSnapGroup = 8;
__global__ __launch_bounds__(256) void k_snap_count(const uint64_t* __restrict__ F,
                                                    const unsigned long long* __restrict__ nz,
                                                    uint32_t stride, uint32_t ntw, uint32_t n,
                                                    uint32_t hw, const uint64_t* __restrict__ mask,
                                                    uint32_t s0, uint32_t ns,
                                                    unsigned long long* out) {
    unsigned long long acc[kSnapGroup] = {};
    const uint64_t total = (uint64_t)n * hw;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256u) {
        const uint32_t v = (uint32_t)(i / hw), w = (uint32_t)(i % hw), tile = w >> 4;
        if (!((nz[(uint64_t)v * ntw + (tile >> 6)] >> (tile & 63u)) & 1ull)) continue;
        const uint64_t x = F[(uint64_t)v * stride + w];
        if (!x) continue;
#pragma unroll
        for (uint32_t s = 0; s < kSnapGroup; s++)
            if (s < ns) acc[s] += (unsigned long long)__popcll(x & mask[(uint64_t)(s0 + s) * hw + w]);
    }
#pragma unroll
    for (uint32_t s = 0; s < kSnapGroup; s++) {
        unsigned long long x = acc[s];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if ((threadIdx.x & 63u) == 0 && s < ns && x) atomicAdd(&out[2 + 2 * (s0 + s) + 1], x);
    }
}

// sum over nodes of (a[v] + b[v]) (b nullable) into *out (64-bit).
__global__ __launch_bounds__(256) void k_sum_u32(const uint32_t* a, const uint32_t* b, uint32_t n,
                                                 unsigned long long* out) {
    unsigned long long s = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        s += (unsigned long long)a[i] + (b ? b[i] : 0u);
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(out, s);
}

// The DENSE phase's device stamps (s_memrealtime, 100 MHz), one thread each, in stream order:
// k_phase_start runs when the kernel before the phase has finished, k_phase_acc when the phase's
// last kernel has, and adds the span to ts[2] (ts[3] counts them).  Round 4 stamped from every
// block of the phase kernels with same-address atomics, which slowed k_transpose 6x.
// A fused tick whose kernel stamps itself (ts[4] = block 0's start, ts[5] = the last block's end:
// one no-return atomicMax per block as it ends) takes that span: the two stamp kernels' launch
// gaps (~6 us each on C2) are not the phase's.
__global__ void k_phase_start(unsigned long long* ts) {
    ts[0] = __builtin_amdgcn_s_memrealtime();
    ts[4] = ~0ull;
    ts[5] = 0ull;
}
__global__ void k_phase_acc(unsigned long long* ts) {
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    if (ts[5] > ts[4])
        ts[2] += ts[5] - ts[4];
    else if (now > ts[0])
        ts[2] += now - ts[0];
    ts[3] += 1ull;
}

// Σ sent = Σ (births' sends + deg x recv), the derived sent counter (header comment)
__global__ __launch_bounds__(256) void k_sum_sent(const uint64_t* sb, const uint32_t* recv, const uint32_t* deg,
                                                  uint32_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        s += sb[i] + (unsigned long long)recv[i] * deg[i];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(out, s);
}

struct Instance {
    uint32_t nsrc = 1;       // sources (share generations) in this instance
    uint32_t first_ev = 0;   // index of rank-0 member in ev[] (groups: member list)
    uint32_t word = 0;
    uint8_t lo = 0;
    uint8_t state = 0;       // 0 unallocated, 1 live, 2 retired
};

// Per-tick young-tile control (young_kernel.h), uploaded through the staging ring.
struct YoungPack {
    YoungTile yt[kYoungMax];  // k_pull_young's tiles, sorted by tile
    uint32_t wt[64];          // write-sparse index -> tile (births, spills)
    uint8_t lv[kYoungMax];    // positions in yt of the leaving tiles, by tile
    uint8_t ymap[64];         // young id -> position in yt (0xff: none): seen-list entries
    uint8_t wt_yid[64];       // write-sparse index -> young id (births' list spills)
};

constexpr int kRing = 4;   // host staging slots
constexpr int kLag = 2;    // ticks of lag before liveness is read back
// late_age auto: the exit test on every tile.  A tile whose frontier rows are sparse never
// exits (its unseen bits are not covered before the last peer), and the test costs a few
// shuffles per peer batch: C4 1.179e13 -> 1.259e13 edge events/s (peer rows 274 -> 216 GB per
// launch, ages 7/8 alone give the same), C3 3.11 -> 3.07 ms per tick (profiles/r02/late_ab.txt)
constexpr int64_t kAutoLateAge = 1;
// young_skip auto: stamp non-empty slots when under this fraction of them is expected non-empty
// (a stamp costs a writer a byte store per peer; a skipped peer saves its reader a 128-B line)
constexpr double kSkipSlotFrac = 0.3;
// pull_push auto: a tile's F_next rows mark their peers when the marked nodes are expected to be
// under this fraction of all (an unmarked node skips the tile: no own-seen read, no occupancy words)
constexpr double kPushFrac = 0.5;
constexpr double kYoungMinEntries = 16.0;  // young auto: expected slot entries per node (see alloc_device)
constexpr uint32_t kTileWords = 16;  // allocation unit: 16 words = 1024 shares = 128 B per row
// hint stamps of tick t (young_kernel.h), never 0 (the value hint bytes start with): a second
// line, 129..255; (empty-slot skipping) a non-empty slot of one line, 1..127.  A byte keeps its
// value until its writer stamps it again, so a stale byte can match only 254 ticks later (127 is
// odd: the same frontier buffer), and a stale match only costs a line read.
inline uint32_t hint_stamp1(int64_t t) { return 1u + (uint32_t)(((t % 127) + 127) % 127); }
inline uint32_t hint_stamp(int64_t t) { return 0x80u | hint_stamp1(t); }

}  // namespace

struct gossip_engine {
    gossip_config cfg{};
    int device = 0;
    int num_cus = 256;  // compute units of the device (launch sizing)
    hipStream_t stream = nullptr;
    bool have_graph = false, have_sched = false;
    // ---- graph
    uint32_t n = 0;
    uint64_t nnz = 0;
    std::vector<int64_t> h_rowptr;
    std::vector<int32_t> h_col;
    std::vector<uint32_t> h_peers, h_sockets;
    std::vector<uint32_t> comp;  // connected component label (computed on demand)
    int64_t* d_rowptr = nullptr;
    int32_t* d_col = nullptr;
    uint32_t* d_deg = nullptr;
    // ---- NS-3 handshake window (GOSSIP_F_HANDSHAKE)
    bool handshake = false;
    std::vector<uint32_t> h_degc;   // |peers(v)| before REGISTER arrives = keys (v, *)
    int64_t* d_rowptr_c = nullptr;  // connector edges a -> b of the keys (a, b), rows b
    int32_t* d_col_c = nullptr;
    uint32_t* d_degc = nullptr;
    // ---- hop batching (GOSSIP_F_HOP_BATCH): generation g of every node is born in batched
    // tick tick0 + 1 + g (phase kept); per-column cut / snapshot masks use the real times
    bool batch = false, done = false;
    int64_t last_birth_tick = -1;
    std::vector<int64_t> ev_orig_ns;      // real generation time of ev[k]
    // ---- NS-3 link timing (gossip_engine_set_link_timing; hop-batched runs only): share k
    // reaches hop h at ev_orig_ns[k] + h * (L + ev_delta[k])
    bool link_timing = false;
    int64_t link_npb = 0, link_defer = 0;
    // ---- row partition (gossip_engine_set_row_partition): this engine pulls, dedups and
    // counts rows [v0, v1) only; the other rows of the frontier arrive by an exchange after
    // every tick (RCCL over xGMI, or gossip_engine_group_run on one device)
    uint32_t row_rank = 0, row_count = 1, v0 = 0, v1 = 0;
    std::vector<uint32_t> row_lo;  // rank r owns [row_lo[r], row_lo[r + 1])
    ncclComm_t comm = nullptr;
    uint32_t link_hdr = 0;
    std::vector<int64_t> ev_delta;
    uint64_t* d_smask[4] = {};            // per ring slot: snapshot masks [snap][word]
    uint64_t* h_smask[4] = {};
    // ---- schedule (this shard)
    std::vector<gossip_gen_event> ev;   // sorted by ns
    std::vector<uint32_t> ev_inst;      // instance of each event
    std::vector<uint8_t> ev_rank;       // bit rank inside its instance
    std::vector<Instance> inst;
    std::vector<uint32_t> grp_members;  // groups: event indices in rank order
    std::vector<uint32_t> inst_moff;    // groups: offset in grp_members
    std::vector<uint64_t> tick_lo;      // ev range per tick: [tick_lo[t-t0], tick_lo[t-t0+1])
    uint32_t max_births = 0;
    uint32_t max_group_phases = 0;
    // ---- window / words
    uint32_t stride = 0;     // words per node row (capacity, even)
    uint32_t hw = 0;         // high-water words in use (even)
    std::vector<WordCtl> ctl;
    std::vector<uint8_t> tile_alloc;
    std::vector<int64_t> tile_last_inject;
    std::vector<std::vector<uint32_t>> word_insts;
    std::vector<int32_t> col_phase;     // per column: generation phase (ns % L)
    std::vector<uint32_t> col_src;      // per column: source event index
    std::priority_queue<uint32_t, std::vector<uint32_t>, std::greater<uint32_t>> free_tiles;
    int64_t open_tile = -1;
    uint32_t open_word_in_tile = 0;
    uint32_t open_bit = 64;
    std::vector<uint32_t> reset_now;    // words allocated this tick
    // ---- time
    int64_t L = 0, t0 = 0, tick0 = 0, tick_end = 0, cur = 0;
    int64_t cut_tick = -1, cut_r = 0;
    // ---- snapshots
    struct Snap {
        int64_t t_ns, tick, r;
        uint64_t gen_total;
        uint64_t own_gen_total;  // generations of this engine's rows (row partition)
    };
    std::vector<Snap> snaps;
    // ---- device state
    uint64_t* d_F[2] = {nullptr, nullptr};
    uint64_t* d_seen = nullptr;      // row v's seen words at d_seen + v * stride (v in [seen_lo, seen_lo + seen_n))
    uint64_t* d_seen_mem = nullptr;  // the allocation: a row-partitioned rank holds only its own rows
    uint32_t seen_lo = 0, seen_n = 0;
    // CSR mode: tile occupancy of F[0]/F[1] (n x ntw words, bit per 16-word tile row)
    unsigned long long* d_nz[2] = {nullptr, nullptr};
    uint32_t ntw = 0;
    // DENSE mode: adjacency bits (n_pad x n_pad) and the frontier transposed to share-column
    // bit rows (stride*64 x n_pad bits), both uint32 words along the node index
    bool dense = false;
    uint32_t n_pad = 0;
    uint32_t* d_Ab = nullptr;
    // the transposed frontier of F[0] / F[1]: k_transpose fills FT[fcur] (three-kernel path), or
    // k_dense_fused + k_births fill FT[nxt] for the next tick (fused path, dense_kernel.h)
    uint32_t* d_FT[2] = {nullptr, nullptr};
    // fused path: per column tile (256 columns) and 1,024-node K stage, bit = FT holds a bit there;
    // three buffers by tick: tick t reads [t % 3], writes [(t + 1) % 3] (with k_births), zeroes [(t + 2) % 3]
    unsigned long long* d_snz[3] = {nullptr, nullptr, nullptr};
    uint32_t snz_nstw = 0;              // mask words per column tile
    bool ft_valid = false;              // d_FT[fcur] / d_snz[fcur] were written by the fused path
    // Fused row partition (round 6): every DENSE tick of a row rank runs k_dense_fused over its own
    // rows and the ranks all-gather FT_next slices (exchange_ft) instead of F_next rows -- with the
    // RCCL and lockstep (group_run) backends, when the schedule holds no id group (a group word
    // needs the three-kernel path, whose k_transpose reads every rank's F rows)
    bool fused_rows = false;
    bool group_mode = false;            // stepped by gossip_engine_group_run
    uint32_t* d_ftmsg = nullptr;        // this rank's FT slice message (k_ft_pack)
    uint32_t* d_ftrecv = nullptr;       // RCCL: every rank's message, all-gathered
    uint64_t ftmsg_cap = 0, ftrecv_cap = 0;  // (u64 words: ensure_dev)
    uint64_t ft_words(uint32_t wact) const;  // one rank's message (u32 words) at window wact
    uint32_t ft_smax() const;                // u32 words of the largest rank's rows
    int ft_pack(int64_t t);                  // this rank's message of tick t (engine stream)
    int ft_unpack(int64_t t, uint32_t r, const uint32_t* msg);  // rank r's message into this rank
    int exchange_ft(int64_t t);
    int64_t opt_dense_fused = 1;        // 1: k_dense_fused when the tick allows it (tick_step_a)
    int64_t dense_rounds = -1;          // k_dense_fused's most data-parallel rounds (A/B env GOSSIP_DENSE_ROUNDS; -1: all)
    int64_t dense_gm = 4;               // k_dense_fused's row blocks per tile group (A/B env GOSSIP_DENSE_GM)
    uint64_t fused_launches = 0;
    uint32_t* d_tix = nullptr;          // fused path: per-tile tickets of split tiles (n_pad / 256 x stride / 4)
    unsigned long long* d_inc = nullptr;  // n x stride incoming words (GEMM -> pull)
    uint32_t *d_recv = nullptr, *d_gen = nullptr, *d_effgen = nullptr;
    uint64_t* d_sent = nullptr;
    unsigned long long* d_phase_ts = nullptr;  // DENSE phase span: [0] start, [2] sum of spans, [3] count, [4]/[5] fused kernel's own start / end
    unsigned long long* d_live[3] = {nullptr, nullptr, nullptr};  // liveness ring (tick % 3)
    unsigned long long* d_scalars = nullptr;  // [0]=scratch, [1..]=snapshot base/partial
    unsigned long long* d_acct = nullptr;     // k_pull traffic accounting (since reset)
    WordCtl* d_ctl[kRing] = {};
    uint8_t* d_wflags[kRing] = {};
    uint8_t* h_wflags[kRing] = {};
    Birth* d_births[kRing] = {};
    int32_t* d_gphase[kRing] = {};
    int fcur = 0;
    uint64_t device_bytes = 0;
    // ---- host staging
    WordCtl* h_ctl[kRing] = {};
    Birth* h_births[kRing] = {};
    int32_t* h_gphase[kRing] = {};
    hipEvent_t slot_done[kRing] = {};
    unsigned long long* h_live[kRing] = {};
    hipEvent_t live_done[kRing] = {};
    bool live_pending[kRing] = {};
    int64_t live_tick[kRing] = {};
    // ---- tuning options (gossip_engine_set_option; environment defaults)
    int64_t opt_pull_nt = -1;         // -1 = by live footprint (kPullNtBytes), 0/1 forced
    int64_t opt_pull_grid = 0;        // 0 = pull_grid_cap's default
    int64_t opt_dense_min_tiles = 512;  // block tiles the MFMA K split aims for
    int64_t opt_young = -1;           // young tiles (k_pull_young): -1 auto, 0 off, 1 on
    int64_t opt_young_age = 5;        // write-sparse while the oldest shares are <= this many hops
    int64_t opt_young_cap = 127;      // slot entries per node before it overflows to dense rows
    int64_t opt_young_overlap = 1;    // k_pull_young beside k_pull on a second stream, launched first (1), or after it (0)
    int64_t opt_young_grid = 0;       // k_pull_young blocks, 0 = twice the pull grid (C4: 32,768 vs 16,384 blocks, -0.26 ms per phase over 3 same-box pairs, profiles/r04/ab/)
    int64_t opt_pull_gate = 1;        // k_pull: occupancy-gated own-seen loads
    int64_t opt_pull_tiles = 1;       // k_pull: passes over the listed (allocated, non-young) tiles only
    int64_t opt_pull_tile_order = 1;  // ... listed in age order within an occupancy word
    // per staging slot: the pass -> tile lists of the tick's k_pull launches (PullArgs::ptile)
    uint16_t* h_ptile[kRing] = {};
    uint16_t* d_ptile[kRing] = {};
    uint64_t ptile_cap = 0;
    std::vector<uint32_t> pt_off, pt_cnt;  // per launch window of this tick
    bool pt_used = false;                  // the last tick's k_pull ran over tile lists
    // Saturated tiles and dense-row tiles (pull_kernel.h; options pull_sat, dense_rows)
    int64_t opt_pull_sat = 1;              // 1: k_pull keeps and trusts per-node saturation bits
    int64_t opt_dense_rows = -1;           // -1 auto (BFS layer model), 0 off, 1 every listed tile
    unsigned long long* d_sat = nullptr;   // n x ntw words
    unsigned long long* h_tmask[kRing] = {};
    unsigned long long* d_tmask[kRing] = {};
    uint32_t tmask_cap = 0;                // words per slot
    bool sat_used = false;                 // this tick's k_pull keeps saturation bits
    std::vector<int64_t> tile_listed;      // last tick a tile was in k_pull's lists
    // last tick k_pull wrote the tile's saturation bits (listed in a launch that kept them): the
    // bits are trusted only the tick after, so turning pull_sat off and on again never trusts
    // bits written before a tick that listed the tile without them
    std::vector<int64_t> tile_satw;
    std::vector<int64_t> tile_dw;          // last tick every node's F_next row of the tile was written
    // push marks (pull_kernel.h, option pull_push): -1 auto (the BFS layer model expects the rows of
    // a tile's F_next on few enough nodes that their peers are under kPushFrac of all), 0 off, 1 every
    // listed tile that is not dense-row (tests)
    int64_t opt_pull_push = -1;
    std::vector<int64_t> tile_pushw;       // last tick k_pull marked the peers of the tile's row writers
    // per tile (this life): (tick, generations) of the births that landed in it -- its frontier by
    // the layer model is the sum of their floods (an old tile can take a late generation of an id
    // instance it holds: one young flood among stragglers)
    std::vector<std::vector<std::pair<int64_t, uint32_t>>> tile_births;
    void note_birth(uint32_t tl, int64_t t) {
        auto& h = tile_births[tl];
        if (!h.empty() && h.back().first == t)
            h.back().second++;
        else
            h.emplace_back(t, 1u);
    }
    unsigned long long* d_mark[2] = {nullptr, nullptr};  // per tick parity: bit v = v is marked
    uint64_t push_tiles = 0, pushw_tiles = 0;  // (tile, tick) pairs read / written as push tiles since reset
    int64_t mark_tick = INT64_MIN;         // the tick whose k_pull wrote d_mark[tick & 1]
    uint64_t mark_launches = 0;            // k_pull launches that read a mark bitmap since reset
    bool push_write(uint32_t tl, int64_t t) const;
    // expected F_next entries per node of tile tl at tick t (BFS layer model over its births)
    double frontier_entries(uint32_t tl, int64_t t) const;
    std::vector<int64_t> tile_inj_prev;    // the injection tick before tile_last_inject
    std::vector<uint32_t> tile_cols;       // columns allocated in the tile (this life)
    std::vector<double> hop_front;         // expected frontier fraction per hop (BFS layer model)
    uint32_t last_lpw = 0, last_dense_tiles = 0;
    uint64_t sat_launches = 0;
    bool dense_row_hop(uint32_t tl, int64_t hop) const;
    void mark_inject(uint32_t tl, int64_t t) {
        if (tile_last_inject[tl] != t) {
            tile_inj_prev[tl] = tile_last_inject[tl];
            tile_last_inject[tl] = t;
        }
    }
    int64_t opt_young_nt = 1;         // k_pull_young reads peers' slot lines non-temporally
    // empty-slot skipping (young_kernel.h): -1 auto (the BFS layer model expects fewer than
    // kSkipSlotFrac of the slots written this tick to be non-empty), 0 off, 1 every tick (tests)
    int64_t opt_young_skip = -1;
    bool skip_wr_last = false;        // last tick's slot writers stamped non-empty slots
    uint64_t skip_ticks = 0;          // ticks whose k_pull_young read only stamped slots
    int64_t opt_young_idle = 1;       // 1: k_pull_young's idle-node chunk pass (young_kernel.h), 0: off
    uint64_t idle_ticks = 0;          // k_pull_young launches with the idle-node pass
    int64_t opt_young_list_cap = kListU16 - 1;  // seen-list entries (tests: small lists overflow)
    int64_t opt_late_age = -1;        // k_pull early exit for tiles >= this many ticks old (0: off, -1: auto)
    int64_t late_age_now() const {    // auto: every tile of a gathering (CSR) pull
        return opt_late_age >= 0 ? opt_late_age : dense ? 0 : kAutoLateAge;
    }
    hipStream_t ystream = nullptr;    // the second stream (created on first use)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timers_phase;  // pull phase (both kernels)
    double phase_ms_done = 0.0;
    int64_t opt_mem_limit = 0;        // bytes of device memory the engine may hold (0: the device's)
    uint32_t last_nt = 0, last_grid = 0;  // variant of the last pull launch (counters)
    // ---- young tiles (young_kernel.h)
    bool young = false;
    uint16_t* d_slot[2] = {nullptr, nullptr};  // per frontier buffer: n x kSlotU16
    int32_t* d_rev = nullptr;                   // CSR entry of the reverse edge (-1: none)
    uint8_t* d_hint[2] = {nullptr, nullptr};    // per frontier buffer: second-line hints per entry
    std::vector<int64_t> tile_first;           // tick of a tile's first birth
    std::vector<uint8_t> tile_widx;            // write-sparse index of the last tick (0xff: none)
    std::vector<uint32_t> wt_last;             // write-sparse index -> tile of the last tick
    std::vector<uint8_t> tile_yid;             // young id of a young tile (kYidNone: not young)
    uint64_t yid_used = 0;                     // young ids in use (0 .. 62)
    uint16_t* d_ylist = nullptr;               // n x kListU16 seen lists (young_kernel.h)
    unsigned long long* d_ywork = nullptr;     // per 64-node chunk: nodes with work (k_young_idle)
    YoungPack* h_young[kRing] = {};
    YoungPack* d_young[kRing] = {};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timers_young;
    double young_ms_done = 0.0;
    uint64_t young_launches = 0;
    uint32_t last_young_grid = 0;
    // ---- timing / counters
    std::vector<std::pair<hipEvent_t, hipEvent_t>> timers;
    std::vector<hipEvent_t> event_pool;
    uint64_t pull_launches = 0, pull_bytes = 0, ticks = 0;
    double pull_ms_done = 0.0;
    // ---- trace
    bool trace = false;
    struct Tr {
        uint32_t node, id;
        int64_t tick;
        uint32_t hop;
        uint8_t via;
    };
    std::vector<Tr> tr;

    ~gossip_engine();
    int alloc_device();
    int prepare_instances();
    int compute_components();
    int tick_step(int64_t t);
    int tick_step_a(int64_t t);  // up to the tick's kernels (pull, births, snapshot counts)
    int tick_step_b(int64_t t);  // exchange (RCCL) + liveness read-back + bookkeeping
    int exchange_rccl(int64_t t);
    // compressed row exchange (row partition): message buffers and traffic counters
    int pack_rows(int64_t t, uint32_t c, hipStream_t s);
    int unpack_rows(int64_t t, uint32_t r, uint32_t c, const uint64_t* msg, uint64_t words, hipStream_t s);
    int ensure_dev(uint64_t*& p, uint64_t& cap, uint64_t words, uint64_t preserve = 0);
    uint64_t* d_msg = nullptr;       // this rank's packed message
    uint64_t msg_cap = 0, msg_words = 0;
    uint32_t* d_cnt = nullptr;
    uint64_t cnt_cap = 0;
    void* d_scan_tmp = nullptr;
    size_t scan_tmp_bytes = 0;
    uint64_t* d_recv_msgs = nullptr;  // the other ranks' messages (RCCL / host-staged import)
    uint64_t recv_cap = 0;
    uint64_t* d_sizes = nullptr;
    // RCCL exchange with device-side sizes (exchange_rccl): per (rank, chunk) a row capacity that
    // every rank derives from the same all-gathered row counts, so each broadcast's length is known
    // without reading the message first; rows beyond it go in a second round after the tick's one
    // host wait.
    std::vector<uint64_t> xcap;          // [r * kMaxChunks + c] rows
    uint64_t* d_tot = nullptr;           // all-gathered row counts of the tick [c * row_count + r]
    uint64_t* h_tot = nullptr;           // pinned copy
    uint64_t* d_ovf = nullptr;           // overflow rows received in the second round
    uint64_t ovf_cap = 0;
    bool xchunks_checked = false;
    uint64_t x_overflow_rounds = 0;      // (rank, chunk) messages that needed a second round
    int pack_dev(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, hipStream_t s);
    int unpack_dev(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, const uint64_t* msg, const uint64_t* rows,
                   uint64_t r0, uint64_t r1, bool prefix, hipStream_t s);
    uint64_t sizes_cap = 0;
    std::atomic<bool> aborted{false};  // gossip_engine_abort: comm torn down by another thread
    std::atomic<int> comm_issuing{0};  // collectives being issued on comm right now (COMM_TRY)
    uint64_t exchange_bytes_out = 0, exchange_bytes_in = 0;
    bool tick_open = false;          // host-staged stepping: tick_begin done, tick_end pending
    // Pipelined exchange (option xchunks, row partition only): the own rows go through the pull
    // and the births in `nchunks` row chunks on the engine stream, chunk c ending with
    // ev_chunk[c]; chunk c's message is packed, sent and the other ranks' chunk c unpacked on
    // xstream while the engine stream computes chunk c + 1.  Every rank uses the same chunk
    // count (checked by the RCCL backend).  kWholeRows = one message of all own rows.
    static constexpr uint32_t kMaxChunks = 16, kWholeRows = 0xffffffffu;
    int64_t opt_xchunks = 4;
    uint32_t nchunks = 1;            // chunks of the current tick
    hipStream_t xstream = nullptr;
    hipEvent_t ev_chunk[kMaxChunks] = {};
    hipEvent_t ev_xdone = nullptr;
    int64_t packed_tick = -1;        // host-staged export: message of (tick, chunk) already packed
    uint32_t packed_chunk = 0;
    void chunk_rows(uint32_t r, uint32_t c, uint64_t* lo, uint64_t* hi) const;
    int pack_range(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, hipStream_t s);
    int unpack_range(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, const uint64_t* msg, uint64_t words,
                     hipStream_t s);
    // Row-partition rehearsal (option rehearse_rows = R, one unpartitioned CSR engine): the pull
    // runs as R row-range launches, and every range's F_next rows go through the real pack and
    // unpack kernels (into the same rows: idempotent), each step timed per range -- one rank's
    // compute and exchange work of an R-rank partition, on one GPU, with the data of the whole.
    int64_t opt_rehearse_rows = 0;
    std::vector<uint64_t> rr_lo;  // R + 1 range bounds (512-row blocks, set_row_partition's rule)
    struct RehearseEv { uint32_t range, kind; hipEvent_t a, b; };  // kind 0 pull, 1 pack, 2 unpack
    std::vector<RehearseEv> rr_events;
    std::vector<double> rr_ms[3];
    std::vector<uint64_t> rr_bytes, rr_bytes_max;
    uint64_t rr_ticks = 0;
    int rehearse_exchange(int64_t t);
    void rehearse_harvest();
    int ensure_xstream();
    int retire_from(int64_t known_tick, const unsigned long long* live);
    int retire_early(int64_t t);
    uint32_t soft_cap() const;
    uint64_t early_retires = 0;  // ticks whose allocation waited for the last tick's liveness
    int alloc_bits(uint32_t k, uint32_t* word, uint8_t* lo, int64_t t);
    int grow(uint32_t new_stride);
    uint32_t grows = 0;
    int decode_trace(int64_t t);
    hipEvent_t get_event();
};

gossip_engine::~gossip_engine() {
    if (xstream) hipStreamSynchronize(xstream);
    if (stream) hipStreamSynchronize(stream);
    for (auto& p : timers) {
        hipEventDestroy(p.first);
        hipEventDestroy(p.second);
    }
    for (auto e : event_pool) hipEventDestroy(e);
    // Teardown: errors are ignored (nothing to report them to from a destructor).
    hipFree(d_rowptr); hipFree(d_col); hipFree(d_deg);
    hipFree(d_rowptr_c); hipFree(d_col_c); hipFree(d_degc);
    for (int k = 0; k < 4; k++) { hipFree(d_smask[k]); hipHostFree(h_smask[k]); }
    hipFree(d_F[0]); hipFree(d_F[1]); hipFree(d_seen_mem); hipFree(d_nz[0]); hipFree(d_nz[1]); hipFree(d_sat); hipFree(d_mark[0]); hipFree(d_mark[1]); hipFree(d_Ab); hipFree(d_FT[0]); hipFree(d_FT[1]); hipFree(d_snz[0]); hipFree(d_snz[1]); hipFree(d_snz[2]); hipFree(d_tix); hipFree(d_inc); hipFree(d_ftmsg); hipFree(d_ftrecv);
    hipFree(d_recv); hipFree(d_gen); hipFree(d_effgen); hipFree(d_sent); hipFree(d_phase_ts);
    hipFree(d_live[0]); hipFree(d_live[1]); hipFree(d_live[2]); hipFree(d_scalars); hipFree(d_acct);
    hipFree(d_msg); hipFree(d_cnt); hipFree(d_scan_tmp); hipFree(d_recv_msgs); hipFree(d_sizes);
    hipFree(d_tot); hipFree(d_ovf); hipHostFree(h_tot);
    for (int k = 0; k < kRing; k++) { hipFree(d_ptile[k]); hipHostFree(h_ptile[k]); }
    for (int k = 0; k < kRing; k++) { hipFree(d_tmask[k]); hipHostFree(h_tmask[k]); }
    hipFree(d_slot[0]); hipFree(d_slot[1]);
    hipFree(d_rev); hipFree(d_hint[0]); hipFree(d_hint[1]); hipFree(d_ylist); hipFree(d_ywork);
    for (int k = 0; k < kRing; k++) { hipFree(d_young[k]); hipHostFree(h_young[k]); }
    for (auto& p : timers_young) {
        hipEventDestroy(p.first);
        hipEventDestroy(p.second);
    }
    if (comm && !aborted.load()) ncclCommDestroy(comm);  // (an aborted communicator is already freed)
    for (int k = 0; k < kRing; k++) {
        hipFree(d_ctl[k]); hipFree(d_births[k]); hipFree(d_gphase[k]); hipFree(d_wflags[k]);
        hipHostFree(h_wflags[k]);
        hipHostFree(h_ctl[k]); hipHostFree(h_births[k]); hipHostFree(h_gphase[k]);
        hipHostFree(h_live[k]);
        if (slot_done[k]) hipEventDestroy(slot_done[k]);
        if (live_done[k]) hipEventDestroy(live_done[k]);
    }
    for (auto& p : timers_phase) {
        hipEventDestroy(p.first);
        hipEventDestroy(p.second);
    }
    if (ev_fork) hipEventDestroy(ev_fork);
    if (ev_join) hipEventDestroy(ev_join);
    if (ystream) hipStreamDestroy(ystream);
    for (auto ev : ev_chunk)
        if (ev) hipEventDestroy(ev);
    if (ev_xdone) hipEventDestroy(ev_xdone);
    if (xstream) hipStreamDestroy(xstream);
    if (stream) hipStreamDestroy(stream);
}

hipEvent_t gossip_engine::get_event() {
    if (event_pool.empty()) {
        // (created in batches, outside the launch sequence of a tick as far as possible: an event
        // created between two launches of a timed phase delays the second one)
        for (int k = 0; k < 64; k++) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) break;
            event_pool.push_back(e);
        }
    }
    if (!event_pool.empty()) {
        hipEvent_t e = event_pool.back();
        event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
}

int gossip_engine::compute_components() {
    if (comp.empty()) comp = gossip::components(n, h_rowptr.data(), h_col.data());
    return GOSSIP_OK;
}

// Group generations into instances: (shareId, connected component).  Within a component a
// later generation of an id either joins the live flood (a group) or finds the id already
// processed everywhere (no-op); in different components the floods never meet.
int gossip_engine::prepare_instances() {
    const uint64_t m = ev.size();
    const bool any_collision = gossip::any_id_collision(m, ev.data());
    if (any_collision) compute_components();
    // Key each event by (id, component); singles use their own index.
    // (the phase and time ride in the key: the sort touches no event)
    struct Key {
        uint32_t id, comp, ev;
        int64_t ph, ns;
    };
    std::vector<Key> keys(m);
    for (uint64_t k = 0; k < m; k++) {
        const gossip_gen_event& e = ev[k];
        keys[k] = Key{e.share_id, any_collision ? comp[e.node] : 0u, (uint32_t)k, e.ns % L, e.ns};
    }
    std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) {
        if (a.id != b.id) return a.id < b.id;
        if (a.comp != b.comp) return a.comp < b.comp;
        if (a.ph != b.ph) return a.ph < b.ph;  // phase order
        return a.ns != b.ns ? a.ns < b.ns : a.ev < b.ev;
    });
    // Shard ownership: deterministic hash of the instance key.
    const uint32_t S = cfg.shard_count > 1 ? cfg.shard_count : 1;
    std::vector<uint8_t> keep(m, 1);
    std::vector<uint32_t> inst_of(m, 0);
    std::vector<uint8_t> rank_of(m, 0);
    inst.clear();
    grp_members.clear();
    inst_moff.clear();
    uint64_t k = 0, id_end = 0;
    while (k < m) {
        uint64_t e = k + 1;
        while (e < m && keys[e].id == keys[k].id && keys[e].comp == keys[k].comp) e++;
        if (id_end <= k) {  // extent of this id over all components
            id_end = e;
            while (id_end < m && keys[id_end].id == keys[k].id) id_end++;
        }
        const bool lone = (id_end - k) == 1 && (e - k) == 1 && (k == 0 || keys[k - 1].id != keys[k].id);
        const uint32_t ns = (uint32_t)(e - k);
        if (ns > 64)
            return set_error(GOSSIP_EINVAL, "more than 64 generations share one id in one component");
        // Same rules as gossip_shard_events / _by_tick (host.cpp): lone ids by (id, node), others
        // by (id, component); hashed, or (GOSSIP_F_SHARD_BY_TICK) by the tick of the instance's
        // first generation
        bool mine = S == 1;
        if (!mine && (cfg.flags & GOSSIP_F_SHARD_BY_TICK)) {
            int64_t first = keys[k].ns;
            for (uint64_t q = k + 1; q < e; q++) first = std::min(first, keys[q].ns);
            mine = (uint64_t)(first / L) % S == cfg.shard_rank;
        } else if (!mine) {
            const uint64_t hkey = lone ? gossip::instance_hash(keys[k].id, ev[keys[k].ev].node, true)
                                       : gossip::instance_hash(keys[k].id, keys[k].comp, false);
            mine = (hkey % S) == cfg.shard_rank;
        }
        if (!mine) {
            for (uint64_t q = k; q < e; q++) keep[keys[q].ev] = 0;
        } else {
            Instance I;
            I.nsrc = ns;
            I.first_ev = keys[k].ev;
            const uint32_t id = (uint32_t)inst.size();
            inst_moff.push_back((uint32_t)grp_members.size());
            if (ns > 1)
                for (uint64_t q = k; q < e; q++) grp_members.push_back(keys[q].ev);
            for (uint64_t q = k; q < e; q++) {
                inst_of[keys[q].ev] = id;
                rank_of[keys[q].ev] = (uint8_t)(q - k);
            }
            inst.push_back(I);
        }
        k = e;
    }
    // Compact to the owned events (ev stays sorted by ns); remap member indices.
    std::vector<uint32_t> newidx(m, UINT32_MAX);
    std::vector<gossip_gen_event> ev2;
    ev2.reserve(m);
    ev_inst.clear();
    ev_rank.clear();
    std::vector<int64_t> orig2;
    for (uint64_t q = 0; q < m; q++) {
        if (!keep[q]) continue;
        newidx[q] = (uint32_t)ev2.size();
        ev2.push_back(ev[q]);
        if (!ev_orig_ns.empty()) orig2.push_back(ev_orig_ns[q]);
        ev_inst.push_back(inst_of[q]);
        ev_rank.push_back(rank_of[q]);
    }
    for (auto& x : grp_members) x = newidx[x];
    for (auto& I : inst) I.first_ev = newidx[I.first_ev];
    ev.swap(ev2);
    if (!ev_orig_ns.empty()) ev_orig_ns.swap(orig2);
    // Tick buckets.
    const int64_t nt = tick_end - tick0 + 1;
    tick_lo.assign((size_t)nt + 1, 0);
    for (const auto& x : ev) {
        const int64_t t = x.ns / L;
        if (t < tick0 || t >= tick_end)
            return set_error(GOSSIP_EINVAL, "generation event outside [t_start, t_cut)");
        tick_lo[(size_t)(t - tick0) + 1]++;
    }
    max_births = 0;
    for (int64_t t = 0; t < nt; t++) {
        max_births = std::max<uint32_t>(max_births, (uint32_t)tick_lo[t + 1]);
        tick_lo[t + 1] += tick_lo[t];
    }
    max_group_phases = 0;
    for (int64_t t = 0; t < nt; t++) {
        uint32_t s = 0;
        for (uint64_t q = tick_lo[t]; q < tick_lo[t + 1]; q++) {
            const Instance& I = inst[ev_inst[q]];
            if (I.nsrc > 1) s += I.nsrc;
        }
        max_group_phases = std::max(max_group_phases, s);
    }
    return GOSSIP_OK;
}

int gossip_engine::alloc_device() {
    // Capacity: peak births over a window of the estimated flood lifetime (BFS depth from a
    // sample node + margin), unless the caller fixed max_words.
    uint32_t words = cfg.max_words;
    if (words == 0) {
        // Flood lifetime estimate: the largest BFS depth from a few sample roots (host BFS
        // over the CSR), plus the liveness read-back lag and slack.  Exceeding the estimate
        // is reported as GOSSIP_ECAPACITY, never silently truncated.
        int ecc = 0;
        std::vector<int32_t> dist(n, -1);
        std::vector<uint32_t> fr, nx;
        const uint32_t roots[4] = {0u, n / 3u, (2u * n) / 3u, n - 1u};
        for (uint32_t root : roots) {
            std::fill(dist.begin(), dist.end(), -1);
            fr.assign(1, root);
            dist[root] = 0;
            int depth = 0;
            while (!fr.empty()) {
                nx.clear();
                for (uint32_t u : fr)
                    for (int64_t j = h_rowptr[u]; j < h_rowptr[u + 1]; j++) {
                        const uint32_t w = (uint32_t)h_col[j];
                        if (dist[w] < 0) {
                            dist[w] = dist[u] + 1;
                            nx.push_back(w);
                        }
                    }
                if (!nx.empty()) depth++;
                fr.swap(nx);
            }
            ecc = std::max(ecc, depth);
        }
        // (the window widens itself if this is short: gossip_engine::grow)
        const int64_t life = ecc + kLag + 1;
        const int64_t nt = tick_end - tick0;
        uint64_t peak = 0, run = 0;
        std::vector<uint64_t> cnt((size_t)nt, 0);
        for (int64_t t = 0; t < nt; t++) {
            uint64_t c = 0;
            for (uint64_t q = tick_lo[t]; q < tick_lo[t + 1]; q++) {
                const Instance& I = inst[ev_inst[q]];
                c += (ev_rank[q] == 0) ? I.nsrc : 0;
            }
            cnt[t] = c;
            run += c;
            if (t >= life) run -= cnt[t - life];
            peak = std::max(peak, run);
        }
        uint64_t w = (peak + 63) / 64 + 2 * kTileWords;  // + partially filled tiles
        w = (w + 1) & ~1ull;
        words = (uint32_t)std::max<uint64_t>(w, 2);
    }
    stride = (words + kTileWords - 1) / kTileWords * kTileWords;  // rows start on 128-B lines
    // Young tiles: the CSR tick pull on graphs whose frontier rows outgrow the caches (C3/C4).
    {
        const bool ok = !dense && !batch && !handshake && row_count == 1 && opt_rehearse_rows <= 1 &&
                        !(cfg.flags & GOSSIP_F_NOSKIP) &&
                        n < (1u << 31);  // (peer ids carry a hint in bit 31)
        if (opt_young == 1 && !ok)
            return set_error(GOSSIP_EINVAL, "young tiles need the CSR tick engine (not DENSE, HOP_BATCH, "
                                            "HANDSHAKE, NOSKIP or a row partition)");
        // auto: the frontier rows outgrow the caches (n >= 2^20) and the young tiles hold enough
        // bits to pay for their per-node slot reads: expected slot entries per node, ~ births per
        // tick x deg^(young_age - 1) / n, >= kYoungMinEntries (C4 at 2 / 4 shards: ~50 / ~25
        // entries, young tiles win; at 8 shards ~12: they lose 8 %, profiles/r02/)
        const double avg_deg = n ? (double)nnz / n : 0.0;
        const double est_entries = (double)max_births * std::pow(avg_deg, (double)(opt_young_age - 1)) / std::max<uint32_t>(n, 1);
        young = ok && (opt_young == 1 || (opt_young == -1 && n >= (1u << 20) && est_entries >= kYoungMinEntries));
    }
    // slots, plus the second-line hints (young_kernel.h): reverse-edge index + 2 hint bytes per entry
    const uint64_t slot_bytes = young ? 2ull * n * kSlotU16 * 2u + (uint64_t)n * kListU16 * 2u + nnz * 6u : 0ull;
    size_t freeb = 0, totalb = 0;
    HIP_TRY(hipMemGetInfo(&freeb, &totalb));
    if (opt_mem_limit > 0) {  // a memory budget below the device's (tests, co-located engines)
        const uint64_t graph = (uint64_t)n * 4 + nnz * 4 + ((uint64_t)n + 1) * 8;
        const uint64_t lim = (uint64_t)opt_mem_limit > graph ? (uint64_t)opt_mem_limit - graph : 0ull;
        freeb = (size_t)std::min<uint64_t>(freeb, lim);
    }
    if (cfg.max_words == 0 && row_count == 1 && opt_rehearse_rows <= 1) {
        // (row-partitioned ranks skip this: their strides must agree for the row exchange; a row
        // rehearsal leaves the memory to its exchange messages)
        // Headroom over the estimate: up to +25% (at least 2 tiles) of row capacity, as far as
        // device memory allows.  Unused capacity costs memory only -- the kernels touch the live
        // words [0, wact) of a row -- while a short estimate on a graph whose bitmaps fill the
        // card cannot be widened later (grow needs a fourth bitmap).  A C4 shard cut to a
        // 20-tick slice measured 1,200 words estimated and more needed.
        const uint64_t want = stride + std::max<uint64_t>(stride / 4, 2 * kTileWords);
        const uint64_t other = (uint64_t)n * 24 + nnz * 4 + ((uint64_t)n + 1) * 8 + slot_bytes +
                               24ull * n * ((want + 1023u) / 1024u) + (4ull << 30);  // + RCCL / context (24: nz x 2 + sat)
        const uint64_t per_word = 3ull * n * 8 + (dense ? 16ull * n_pad : 0ull);  // (DENSE: FT x 2)
        uint64_t fit = freeb > other ? ((uint64_t)freeb - other) / per_word : 0ull;
        fit = fit / kTileWords * kTileWords;
        stride = (uint32_t)std::max<uint64_t>(stride, std::min<uint64_t>(want / kTileWords * kTileWords, fit));
    }
    const uint64_t bm = (uint64_t)n * stride * 8;
    // seen rows: a row-partitioned rank dedups only its own rows (F_cur / F_next stay whole: the
    // pull reads every peer's row, the exchange writes the other ranks' rows)
    rr_lo.clear();
    if (opt_rehearse_rows > 1) {  // rehearsal ranges: set_row_partition's blocks (ceil(n / R) -> 512 rows)
        if (dense) return set_error(GOSSIP_EINVAL, "rehearse_rows: CSR engines only");
        const uint64_t R = (uint64_t)opt_rehearse_rows;
        const uint64_t rpr = ((uint64_t)(n + R - 1) / R + 511) / 512 * 512;
        for (uint64_t r = 0; r <= R; r++) rr_lo.push_back(std::min<uint64_t>(n, r * rpr));
    }
    seen_lo = row_count > 1 ? v0 : 0u;
    seen_n = row_count > 1 ? v1 - v0 : n;
    const uint64_t bm_seen = (uint64_t)seen_n * stride * 8;
    const uint64_t need = 2 * bm + bm_seen + (uint64_t)n * 24 + (nnz * 4) + ((uint64_t)n + 1) * 8 + slot_bytes +
                          24ull * n * ((stride + 1023u) / 1024u) +
                          (dense ? (uint64_t)stride * 8 * n_pad : 0ull);
    if (need > (uint64_t)freeb)
        return set_error(GOSSIP_ENOMEM, "device memory: need " + std::to_string(need) +
                                            " bytes for a " + std::to_string(stride) +
                                            "-word window, " + std::to_string(freeb) + " free");
    HIP_TRY(hipMalloc(&d_F[0], bm));
    HIP_TRY(hipMalloc(&d_F[1], bm));
    HIP_TRY(hipMalloc(&d_seen_mem, std::max<uint64_t>(bm_seen, 8)));
    d_seen = d_seen_mem - (uint64_t)seen_lo * stride;
    HIP_TRY(hipMemsetAsync(d_F[0], 0, bm, stream));
    HIP_TRY(hipMemsetAsync(d_F[1], 0, bm, stream));
    HIP_TRY(hipMemsetAsync(d_seen_mem, 0, bm_seen, stream));
    {
        ntw = (stride + 1023u) / 1024u;
        const size_t nzb = (size_t)n * ntw * 8;
        for (int k = 0; k < 2; k++) {
            HIP_TRY(hipMalloc(&d_nz[k], nzb));
            HIP_TRY(hipMemsetAsync(d_nz[k], 0, nzb, stream));
        }
        if (!dense) {  // saturation bits (k_pull over tile lists)
            HIP_TRY(hipMalloc(&d_sat, nzb));
            HIP_TRY(hipMemsetAsync(d_sat, 0, nzb, stream));
        }
        if (!dense && row_count == 1 && !handshake)  // push marks: a bit per node and tick parity
            for (int k = 0; k < 2; k++) {
                HIP_TRY(hipMalloc(&d_mark[k], ((size_t)n + 64) / 64 * 8));
                HIP_TRY(hipMemsetAsync(d_mark[k], 0, ((size_t)n + 64) / 64 * 8, stream));
            }
    }
    {  // BFS layer model for the dense-row tiles: frontier fraction per hop of one flood
        hop_front.clear();
        const double avg_deg = n ? (double)nnz / n : 0.0;
        double reached = n ? 1.0 / n : 0.0, front = reached;
        for (int h = 0; h < 64 && front > 0.0; h++) {
            hop_front.push_back(front);
            const double nx = (1.0 - reached) * (1.0 - std::exp(-avg_deg * front));
            reached += nx;
            front = nx;
        }
    }
    HIP_TRY(hipMalloc(&d_recv, (size_t)n * 4));
    HIP_TRY(hipMalloc(&d_gen, (size_t)n * 4));
    HIP_TRY(hipMalloc(&d_effgen, (size_t)n * 4));
    HIP_TRY(hipMalloc(&d_sent, (size_t)n * 8));
    {
        const unsigned long long init[6] = {~0ull, 0ull, 0ull, 0ull, ~0ull, 0ull};
        HIP_TRY(hipMalloc(&d_phase_ts, sizeof(init)));
        HIP_TRY(hipMemcpy(d_phase_ts, init, sizeof(init), hipMemcpyHostToDevice));
    }
    HIP_TRY(hipMemsetAsync(d_recv, 0, (size_t)n * 4, stream));
    HIP_TRY(hipMemsetAsync(d_gen, 0, (size_t)n * 4, stream));
    HIP_TRY(hipMemsetAsync(d_effgen, 0, (size_t)n * 4, stream));
    HIP_TRY(hipMemsetAsync(d_sent, 0, (size_t)n * 8, stream));
    for (int k = 0; k < 3; k++) {
        HIP_TRY(hipMalloc(&d_live[k], (size_t)stride * 8));
        HIP_TRY(hipMemsetAsync(d_live[k], 0, (size_t)stride * 8, stream));
    }
    const size_t nsc = 2 + 2 * snaps.size();
    HIP_TRY(hipMalloc(&d_scalars, nsc * 8));
    HIP_TRY(hipMemsetAsync(d_scalars, 0, nsc * 8, stream));
    HIP_TRY(hipMalloc(&d_acct, kAcctSlots * kAcctReplicas * 8));
    HIP_TRY(hipMemsetAsync(d_acct, 0, kAcctSlots * kAcctReplicas * 8, stream));
    if (young) {
        for (int k = 0; k < 2; k++) {
            // empty slots: header 0, every entry a tombstone (readers scatter whole lines)
            HIP_TRY(hipMalloc(&d_slot[k], (size_t)n * kSlotU16 * 2u));
            HIP_TRY(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(d_slot[k]), (unsigned short)kSlotTomb,
                                      (size_t)n * kSlotU16, stream));
            HIP_TRY(hipMemset2DAsync(d_slot[k], kSlotU16 * 2u, 0, 2, n, stream));
            // (+16: the idle-node pass reads whole 4-B words of it)
            if (k == 0) HIP_TRY(hipMalloc(&d_ywork, ((size_t)n + 127) / 64 * 8));
            HIP_TRY(hipMalloc(&d_hint[k], (size_t)nnz + 16));
            HIP_TRY(hipMemsetAsync(d_hint[k], 0, (size_t)nnz + 16, stream));  // stamps are >= 1
        }
        {  // reverse edges: rev[j] = the entry of v in the list of u = col[j] (j in v's list)
            std::vector<int32_t> rev(nnz, -1), perm(nnz);
            const int th = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
            gossip::parallel_for(n, th, [&](uint64_t lo, uint64_t hi) {  // each row's entries by id
                for (uint64_t u = lo; u < hi; u++) {
                    const int64_t b = h_rowptr[u], e = h_rowptr[u + 1];
                    for (int64_t j = b; j < e; j++) perm[j] = (int32_t)j;
                    std::sort(perm.begin() + b, perm.begin() + e,
                              [&](int32_t x, int32_t y) { return h_col[x] < h_col[y]; });
                }
            });
            gossip::parallel_for(n, th, [&](uint64_t lo, uint64_t hi) {
                for (uint64_t v = lo; v < hi; v++)
                    for (int64_t j = h_rowptr[v]; j < h_rowptr[v + 1]; j++) {
                        const uint32_t u = (uint32_t)h_col[j];
                        auto b = perm.begin() + h_rowptr[u], e = perm.begin() + h_rowptr[u + 1];
                        auto it = std::lower_bound(b, e, (int32_t)v,
                                                   [&](int32_t x, int32_t val) { return h_col[x] < val; });
                        if (it != e && (uint32_t)h_col[*it] == v) rev[j] = *it;
                    }
            });
            HIP_TRY(hipMalloc(&d_rev, std::max<size_t>(nnz, 1) * 4));
            if (nnz) HIP_TRY(hipMemcpy(d_rev, rev.data(), nnz * 4, hipMemcpyHostToDevice));
        }
        for (int k = 0; k < kRing; k++) {
            HIP_TRY(hipMalloc(&d_young[k], sizeof(YoungPack)));
            HIP_TRY(hipHostMalloc(&h_young[k], sizeof(YoungPack), hipHostMallocDefault));
        }
        // empty seen lists: header 0, every entry a tombstone
        HIP_TRY(hipMalloc(&d_ylist, (size_t)n * kListU16 * 2u));
        HIP_TRY(hipMemsetD16Async(reinterpret_cast<hipDeviceptr_t>(d_ylist), (unsigned short)kSlotTomb,
                                  (size_t)n * kListU16, stream));
        HIP_TRY(hipMemset2DAsync(d_ylist, kListU16 * 2u, 0, 2, n, stream));
    }
    const uint32_t bcap = std::max<uint32_t>(max_births, 1);
    const uint32_t pcap = std::max<uint32_t>(max_group_phases, 1);
    for (int k = 0; k < kRing; k++) {
        HIP_TRY(hipMalloc(&d_ctl[k], (size_t)stride * sizeof(WordCtl)));
        HIP_TRY(hipMalloc(&d_wflags[k], (size_t)stride + 16));
        HIP_TRY(hipHostMalloc(&h_wflags[k], (size_t)stride + 16, hipHostMallocDefault));
        HIP_TRY(hipMalloc(&d_births[k], (size_t)bcap * sizeof(Birth)));
        HIP_TRY(hipMalloc(&d_gphase[k], (size_t)pcap * 4));
        HIP_TRY(hipHostMalloc(&h_ctl[k], (size_t)stride * sizeof(WordCtl), hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&h_births[k], (size_t)bcap * sizeof(Birth), hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&h_gphase[k], (size_t)pcap * 4, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&h_live[k], (size_t)stride * 8, hipHostMallocDefault));
        HIP_TRY(hipEventCreateWithFlags(&slot_done[k], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&live_done[k], hipEventDisableTiming));
    }
    device_bytes = 2 * bm + bm_seen + (d_sat ? 24ull : 16ull) * n * ntw + (uint64_t)n * 20 + nnz * 4 + ((uint64_t)n + 1) * 8 + 2ull * stride * 8 + slot_bytes +
                   kRing * ((uint64_t)stride * sizeof(WordCtl) + (uint64_t)bcap * sizeof(Birth) + pcap * 4);
    if (dense) {
        const uint64_t ft = (uint64_t)stride * 8 * n_pad;
        snz_nstw = (n_pad / kStageK + 63u) / 64u;
        const uint64_t snzb = (uint64_t)(stride / 4u) * snz_nstw * 8u;
        for (int k = 0; k < 3; k++) {
            if (k < 2) {
                HIP_TRY(hipMalloc(&d_FT[k], ft));
                HIP_TRY(hipMemsetAsync(d_FT[k], 0, ft, stream));
            }
            HIP_TRY(hipMalloc(&d_snz[k], snzb));
            HIP_TRY(hipMemsetAsync(d_snz[k], 0, snzb, stream));
        }
        ft_valid = false;
        HIP_TRY(hipMalloc(&d_inc, bm));
        HIP_TRY(hipMemsetAsync(d_inc, 0, bm, stream));
        const uint64_t tixb = (uint64_t)(n_pad / kDenseTile) * (stride / 4u) * 4u;
        HIP_TRY(hipMalloc(&d_tix, tixb));
        HIP_TRY(hipMemsetAsync(d_tix, 0, tixb, stream));
        device_bytes += 2 * ft + 3 * snzb + bm + tixb + (uint64_t)n_pad * n_pad / 8;
    }
    if (batch && !snaps.empty())
        for (int k = 0; k < kRing; k++) {
            HIP_TRY(hipMalloc(&d_smask[k], (size_t)stride * snaps.size() * 8));
            HIP_TRY(hipHostMalloc(&h_smask[k], (size_t)stride * snaps.size() * 8, hipHostMallocDefault));
        }
    WordCtl z{0ull, ~0ull, 0ull, 0ull, 0ull};
    ctl.assign(stride, z);
    tile_alloc.assign(stride / kTileWords, 0);
    tile_last_inject.assign(stride / kTileWords, INT64_MIN);
    tile_first.assign(stride / kTileWords, INT64_MIN);
    tile_widx.assign(stride / kTileWords, 0xffu);
    tile_yid.assign(stride / kTileWords, (uint8_t)kYidNone);
    tile_listed.assign(stride / kTileWords, INT64_MIN);
    tile_satw.assign(stride / kTileWords, INT64_MIN);
    tile_dw.assign(stride / kTileWords, INT64_MIN);
    tile_pushw.assign(stride / kTileWords, INT64_MIN);
    tile_births.assign(stride / kTileWords, {});
    tile_inj_prev.assign(stride / kTileWords, INT64_MIN);
    tile_cols.assign(stride / kTileWords, 0u);
    word_insts.assign(stride, {});
    col_phase.assign((size_t)stride * 64, 0);
    col_src.assign((size_t)stride * 64, UINT32_MAX);
    HIP_TRY(hipStreamSynchronize(stream));
    return GOSSIP_OK;
}

// Widen every node row to new_stride words (rare: the capacity estimate was short).  Rows are
// copied with 2-D copies one bitmap at a time so the peak is 3 old + 1 new bitmaps.
int gossip_engine::grow(uint32_t new_stride) {
    HIP_TRY(hipStreamSynchronize(stream));
    const uint64_t nb = (uint64_t)n * new_stride * 8;
    size_t freeb = 0, totalb = 0;
    HIP_TRY(hipMemGetInfo(&freeb, &totalb));
    int ok = nb + (64ull << 20) <= (uint64_t)freeb ? 1 : 0;
    if (opt_mem_limit > 0 && device_bytes + 3 * (nb - (uint64_t)n * stride * 8) > (uint64_t)opt_mem_limit) ok = 0;
    if (comm) {
        // Row-partitioned ranks widen in lockstep (their strides must agree for the exchange):
        // all of them grow or all fail, never one rank alone while the others wait in the next
        // exchange.
        int* d_ok = reinterpret_cast<int*>(d_scalars);  // scratch word [0]
        HIP_TRY(hipMemcpyAsync(d_ok, &ok, sizeof(int), hipMemcpyHostToDevice, stream));
        {
            CommIssue issuing_(comm_issuing);
            if (aborted.load()) return set_error(GOSSIP_ESTATE, "RCCL: the row partition was aborted");
            if (ncclAllReduce(d_ok, d_ok, 1, ncclInt32, ncclMin, comm, stream) != ncclSuccess)
                return set_error(GOSSIP_EHIP, "RCCL: capacity agreement failed");
        }
        HIP_TRY(hipMemcpyAsync(&ok, d_ok, sizeof(int), hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipStreamSynchronize(stream));
    }
    if (!ok)
        return set_error(GOSSIP_ECAPACITY, "live-share window exceeded " + std::to_string(stride) +
                                               " words per node and there is no device memory to widen it" +
                                               (comm ? " (on some rank of the row partition)" : ""));
    uint64_t** bufs[3] = {&d_F[0], &d_F[1], &d_seen_mem};
    for (uint64_t** b : bufs) {
        const uint64_t rows = *b == d_seen_mem ? seen_n : n;
        uint64_t* nbuf = nullptr;
        HIP_TRY(hipMalloc(&nbuf, std::max<uint64_t>(rows * new_stride * 8, 8)));
        HIP_TRY(hipMemsetAsync(nbuf, 0, rows * new_stride * 8, stream));
        if (rows)
            HIP_TRY(hipMemcpy2DAsync(nbuf, (size_t)new_stride * 8, *b, (size_t)stride * 8, (size_t)stride * 8, rows,
                                     hipMemcpyDeviceToDevice, stream));
        HIP_TRY(hipStreamSynchronize(stream));
        HIP_TRY(hipFree(*b));
        *b = nbuf;
    }
    d_seen = d_seen_mem - (uint64_t)seen_lo * new_stride;
    auto regrow_dev = [&](auto*& p, size_t elem, size_t oldn, size_t newn) -> int {
        void* q = nullptr;
        HIP_TRY(hipMalloc(&q, newn * elem));
        HIP_TRY(hipMemset(q, 0, newn * elem));
        HIP_TRY(hipMemcpy(q, (const void*)p, oldn * elem, hipMemcpyDeviceToDevice));
        HIP_TRY(hipFree((void*)p));
        p = reinterpret_cast<std::remove_reference_t<decltype(p)>>(q);
        return GOSSIP_OK;
    };
    auto regrow_host = [&](auto*& p, size_t elem, size_t oldn, size_t newn) -> int {
        void* q = nullptr;
        HIP_TRY(hipHostMalloc(&q, newn * elem, hipHostMallocDefault));
        std::memset(q, 0, newn * elem);
        std::memcpy(q, (const void*)p, oldn * elem);
        HIP_TRY(hipHostFree((void*)p));
        p = reinterpret_cast<std::remove_reference_t<decltype(p)>>(q);
        return GOSSIP_OK;
    };
    const uint32_t new_ntw = (new_stride + 1023u) / 1024u;
    if (new_ntw != ntw) {  // tile numbering is unchanged: widen the nz rows
        for (int k = 0; k < 2; k++) {
            unsigned long long* q = nullptr;
            const size_t nzb = (size_t)n * new_ntw * 8;
            HIP_TRY(hipMalloc(&q, nzb));
            HIP_TRY(hipMemsetAsync(q, 0, nzb, stream));
            HIP_TRY(hipMemcpy2DAsync(q, (size_t)new_ntw * 8, d_nz[k], (size_t)ntw * 8, (size_t)ntw * 8, n,
                                     hipMemcpyDeviceToDevice, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            HIP_TRY(hipFree(d_nz[k]));
            d_nz[k] = q;
        }
        device_bytes += 16ull * n * (new_ntw - ntw);
        for (unsigned long long** sp : {&d_sat}) {  // (a cache: zeros = nothing saturated)
            if (!*sp) continue;
            HIP_TRY(hipFree(*sp));
            HIP_TRY(hipMalloc(sp, (size_t)n * new_ntw * 8));
            HIP_TRY(hipMemset(*sp, 0, (size_t)n * new_ntw * 8));
            device_bytes += 8ull * n * (new_ntw - ntw);
        }
        ntw = new_ntw;
    }
    int rc = 0;
    for (int k = 0; k < 3 && !rc; k++) rc = regrow_dev(d_live[k], 8, stride, new_stride);
    for (int k = 0; k < kRing && !rc; k++) {
        rc = regrow_dev(d_ctl[k], sizeof(WordCtl), stride, new_stride);
        if (!rc) rc = regrow_dev(d_wflags[k], 1, stride + 16, new_stride + 16);
        if (!rc) rc = regrow_host(h_ctl[k], sizeof(WordCtl), stride, new_stride);
        if (!rc) rc = regrow_host(h_wflags[k], 1, stride + 16, new_stride + 16);
        if (!rc) rc = regrow_host(h_live[k], 8, stride, new_stride);
    }
    if (rc) return rc;
    if (dense) {  // transposed frontier: the new columns are appended (column c at c x kw words, its
                  // stage masks at c / 256 x nstw), so the old ones are copied and stay valid -- a
                  // fused row partition could not rebuild them (k_transpose reads every rank's F rows)
        const uint64_t ft = (uint64_t)new_stride * 8 * n_pad, ft_old = (uint64_t)stride * 8 * n_pad;
        const uint64_t snzb = (uint64_t)(new_stride / 4u) * snz_nstw * 8u, snzb_old = (uint64_t)(stride / 4u) * snz_nstw * 8u;
        for (int k = 0; k < 3; k++) {
            if (k < 2) {
                uint32_t* q = nullptr;
                HIP_TRY(hipMalloc(&q, ft));
                HIP_TRY(hipMemset(q, 0, ft));
                HIP_TRY(hipMemcpy(q, d_FT[k], ft_old, hipMemcpyDeviceToDevice));
                HIP_TRY(hipFree(d_FT[k]));
                d_FT[k] = q;
            }
            unsigned long long* z = nullptr;
            HIP_TRY(hipMalloc(&z, snzb));
            HIP_TRY(hipMemset(z, 0, snzb));
            HIP_TRY(hipMemcpy(z, d_snz[k], snzb_old, hipMemcpyDeviceToDevice));
            HIP_TRY(hipFree(d_snz[k]));
            d_snz[k] = z;
        }
        HIP_TRY(hipFree(d_inc));
        d_inc = nullptr;
        HIP_TRY(hipMalloc(&d_inc, nb));
        HIP_TRY(hipMemset(d_inc, 0, nb));
        HIP_TRY(hipFree(d_tix));
        d_tix = nullptr;
        const uint64_t tixb = (uint64_t)(n_pad / kDenseTile) * (new_stride / 4u) * 4u;
        HIP_TRY(hipMalloc(&d_tix, tixb));
        HIP_TRY(hipMemset(d_tix, 0, tixb));
        device_bytes += (uint64_t)(new_stride - stride) * (16ull * n_pad + 8ull * n + 6ull * snz_nstw);
    }
    if (batch && !snaps.empty())
        for (int k = 0; k < kRing; k++) {  // rebuilt every tick: no copy
            HIP_TRY(hipFree(d_smask[k]));
            HIP_TRY(hipHostFree(h_smask[k]));
            HIP_TRY(hipMalloc(&d_smask[k], (size_t)new_stride * snaps.size() * 8));
            HIP_TRY(hipHostMalloc(&h_smask[k], (size_t)new_stride * snaps.size() * 8, hipHostMallocDefault));
        }
    WordCtl z{0ull, ~0ull, 0ull, 0ull, 0ull};
    ctl.resize(new_stride, z);
    tile_alloc.resize(new_stride / kTileWords, 0);
    tile_last_inject.resize(new_stride / kTileWords, INT64_MIN);
    tile_first.resize(new_stride / kTileWords, INT64_MIN);
    tile_listed.resize(new_stride / kTileWords, INT64_MIN);
    tile_satw.resize(new_stride / kTileWords, INT64_MIN);
    tile_dw.resize(new_stride / kTileWords, INT64_MIN);
    tile_pushw.resize(new_stride / kTileWords, INT64_MIN);
    tile_births.resize(new_stride / kTileWords);
    tile_inj_prev.resize(new_stride / kTileWords, INT64_MIN);
    tile_cols.resize(new_stride / kTileWords, 0u);
    tile_widx.resize(new_stride / kTileWords, 0xffu);
    tile_yid.resize(new_stride / kTileWords, (uint8_t)kYidNone);
    word_insts.resize(new_stride);
    col_phase.resize((size_t)new_stride * 64, 0);
    col_src.resize((size_t)new_stride * 64, UINT32_MAX);
    device_bytes += (2ull * n + seen_n) * (uint64_t)(new_stride - stride) * 8;
    stride = new_stride;
    grows++;
    return GOSSIP_OK;
}

// Columns are handed out in TILES of kTileWords words (1024 shares = one 128-B line per node
// row), so every line of a frontier/seen row holds shares of the same age and the pull's
// skip decisions are line-coherent.  Births fill the open tile word by word; an id group
// never straddles a word.
int gossip_engine::alloc_bits(uint32_t k, uint32_t* word, uint8_t* lo, int64_t t) {
    if ((cfg.flags & GOSSIP_F_TILE_PER_TICK) && open_tile >= 0 && tile_last_inject[(uint32_t)open_tile] < t)
        open_tile = -1;
    if (open_tile >= 0 && open_bit + k > 64 && open_word_in_tile + 1 < kTileWords) {
        open_word_in_tile++;
        open_bit = 0;
    }
    if (open_tile < 0 || open_bit + k > 64) {
        uint32_t tl;
        // Near the window's capacity, retire from the last tick's liveness before widening the
        // high-water mark: the regular retirement reads liveness kLag = 2 ticks late (the host
        // prepares tick t while the GPU runs t - 1), so every drained tile is held two ticks past
        // its flood; waiting here for tick t - 1 (a stall of the host's tick preparation, only on
        // ticks that would otherwise widen the window into its last margin) frees the tiles whose
        // floods ended a tick earlier.
        if (free_tiles.empty() && hw + kTileWords > soft_cap()) {
            const int rc = retire_early(t);
            if (rc) return rc;
        }
        if (!free_tiles.empty()) {
            tl = free_tiles.top();
            free_tiles.pop();
        } else {
            if (hw + kTileWords > stride) {
                const uint32_t ns = (uint32_t)((stride + stride / 4 + kTileWords) / kTileWords * kTileWords);
                const int rc = grow(ns);
                if (rc) return rc;
            }
            tl = hw / kTileWords;
            hw += kTileWords;
        }
        tile_alloc[tl] = 1;
        tile_first[tl] = t;
        tile_cols[tl] = 0;  // (a new life: nothing of the previous one is trusted)
        tile_listed[tl] = INT64_MIN;
        tile_satw[tl] = INT64_MIN;
        tile_dw[tl] = INT64_MIN;
        tile_pushw[tl] = INT64_MIN;
        tile_births[tl].clear();
        for (uint32_t q = 0; q < kTileWords; q++) reset_now.push_back(tl * kTileWords + q);
        open_tile = tl;
        open_word_in_tile = 0;
        open_bit = 0;
    }
    *word = (uint32_t)open_tile * kTileWords + open_word_in_tile;
    *lo = (uint8_t)open_bit;
    open_bit += k;
    mark_inject((uint32_t)open_tile, t);
    tile_cols[(uint32_t)open_tile] += k;
    return GOSSIP_OK;
}

// Dense-row tile (pull_kernel.h): is the tile's frontier at `hop` expected to hold a bit in every
// node's row?  BFS layer model of the graph (alloc_device): a row of c columns at a hop whose
// frontier covers a fraction f of the nodes holds ~c f bits; at >= kDenseRowBits an empty row is
// improbable (e^-32), and a misjudged tile costs bytes, never results (its rows are all written).
constexpr double kDenseRowBits = 32.0;
bool gossip_engine::dense_row_hop(uint32_t tl, int64_t hop) const {
    if (opt_dense_rows == 1) return hop >= 1;
    if (hop < 0 || hop >= (int64_t)hop_front.size()) return false;
    return (double)tile_cols[tl] * hop_front[(size_t)hop] >= kDenseRowBits;
}

// Push marks (pull_kernel.h): does the F_next of tile tl at tick t sit on few enough nodes that
// their peers -- the nodes that must pull the tile next tick -- are under kPushFrac of all?  BFS
// layer model: a share born at tick b is at hop t - b in F_next and its frontier holds hop_front[t -
// b] of the nodes (beyond the model's last hop: none -- stragglers); the tile's births together give
// the expected frontier entries per node, each marks avg_deg nodes, and a node is marked with
// probability 1 - e^-(marks per node).  A misjudged tile costs marking work, never results (a marked
// node pulls the tile as before).
double gossip_engine::frontier_entries(uint32_t tl, int64_t t) const {
    double e = 0.0;
    for (const auto& b : tile_births[tl]) {
        const int64_t h = t - b.first;
        if (h >= 0 && h < (int64_t)hop_front.size()) e += (double)b.second * hop_front[(size_t)h];
    }
    return e;
}
bool gossip_engine::push_write(uint32_t tl, int64_t t) const {
    if (opt_pull_push == 1) return true;
    const double avg_deg = n ? (double)nnz / n : 0.0;
    return 1.0 - std::exp(-frontier_entries(tl, t) * avg_deg) < kPushFrac;
}

// High-water mark above which alloc_bits first retires from the freshest liveness (retire_early):
// the capacity less max(2 tiles, 1/16 of it).
uint32_t gossip_engine::soft_cap() const {
    const uint32_t margin = std::max<uint32_t>(2u * kTileWords, stride / 16u / kTileWords * kTileWords);
    return stride > margin ? stride - margin : 0u;
}

int gossip_engine::retire_early(int64_t t) {
    if (row_count > 1 || batch) return GOSSIP_OK;  // (ranks retire in lockstep; batched ticks are not timed)
    const int64_t kt = t - 1;
    const int ls = (int)(((kt % kRing) + kRing) % kRing);
    if (kt < tick0 || !live_pending[ls] || live_tick[ls] != kt) return GOSSIP_OK;
    HIP_TRY(hipEventSynchronize(live_done[ls]));
    live_pending[ls] = false;  // (consumed: the regular step of tick t + 1 has nothing left to read)
    early_retires++;
    return retire_from(kt, h_live[ls]);
}

int gossip_engine::retire_from(int64_t known_tick, const unsigned long long* live) {
    const uint32_t ntiles = hw / kTileWords;
    for (uint32_t tl = 0; tl < ntiles; tl++) {
        if (!tile_alloc[tl] || tile_last_inject[tl] > known_tick) continue;
        bool any = false;
        for (uint32_t q = 0; q < kTileWords; q++) any |= live[tl * kTileWords + q] != 0ull;
        if (any) continue;
        for (uint32_t q = 0; q < kTileWords; q++) {
            const uint32_t w = tl * kTileWords + q;
            for (uint32_t id : word_insts[w]) inst[id].state = 2;
            word_insts[w].clear();
            ctl[w].gmask = 0ull;
            ctl[w].gstart = 0ull;
            for (int b = 0; b < 64; b++) col_src[(size_t)w * 64 + b] = UINT32_MAX;
        }
        tile_alloc[tl] = 0;
        free_tiles.push(tl);
        if ((int64_t)tl == open_tile) open_tile = -1;
    }
    return GOSSIP_OK;
}

int gossip_engine::tick_step(int64_t t) {
    int rc = tick_step_a(t);
    return rc ? rc : tick_step_b(t);
}

int gossip_engine::tick_step_a(int64_t t) {
    const int slot = (int)(t % kRing);
    // 1. liveness of tick t-kLag -> retire words whose floods have drained.
    {
        const int64_t kt = t - kLag;
        const int ls = (int)(((kt % kRing) + kRing) % kRing);
        if (kt >= tick0 && live_pending[ls] && live_tick[ls] == kt) {
            HIP_TRY(hipEventSynchronize(live_done[ls]));
            live_pending[ls] = false;
            int rc = retire_from(kt, h_live[ls]);
            if (rc) return rc;
        }
    }
    // 2. staging slot reuse
    HIP_TRY(hipEventSynchronize(slot_done[slot]));
    // 3. births of tick t
    reset_now.clear();
    uint32_t nb = 0, np = 0;
    // (hop-batched runs keep stepping after the last birth tick until the floods retire)
    const size_t tb = (size_t)(t - tick0);
    const uint64_t lo = tb + 1 < tick_lo.size() ? tick_lo[tb] : 0, hi = tb + 1 < tick_lo.size() ? tick_lo[tb + 1] : 0;
    Birth* B = h_births[slot];
    int32_t* GP = h_gphase[slot];
    for (uint64_t q = lo; q < hi; q++) {
        const gossip_gen_event& e = ev[q];
        Instance& I = inst[ev_inst[q]];
        Birth b{};
        b.node = e.node;
        b.phase = (int32_t)(e.ns % L);
        // handshake window (tick0 = t_start / L): REGISTER lands at tick0 + 3 before any
        // other event of that instant, so births up to tick0 + 2 see connector-side peers only
        if (handshake && t < tick0 + 3) b.flags = BF_CONN;
        if (handshake && t < tick0 + 2) {
            // sent before the connector sockets are ESTABLISHED: lost (unique id, checked)
            b.kind = BIRTH_LOST;
            I.state = 2;
            if (trace) tr.push_back(Tr{e.node, e.share_id, t, 0u, (uint8_t)0});
        } else if (I.state == 2) {
            b.kind = BIRTH_NOOP;
        } else {
            if (I.state == 0) {
                uint32_t w;
                uint8_t l;
                int rc = alloc_bits(I.nsrc, &w, &l, t);
                if (rc) return rc;
                I.word = w;
                I.lo = l;
                I.state = 1;
                word_insts[w].push_back(ev_inst[q]);
                if (I.nsrc > 1) {
                    const uint64_t gm = (I.nsrc >= 64 ? ~0ull : ((1ull << I.nsrc) - 1ull)) << l;
                    ctl[w].gmask |= gm;
                    ctl[w].gstart |= 1ull << l;
                    const uint32_t off = inst_moff[ev_inst[q]];
                    for (uint32_t r = 0; r < I.nsrc; r++) {
                        const uint32_t m = grp_members[off + r];
                        col_phase[(size_t)w * 64 + l + r] = (int32_t)(ev[m].ns % L);
                        col_src[(size_t)w * 64 + l + r] = m;
                    }
                } else {
                    col_phase[(size_t)w * 64 + l] = b.phase;
                    col_src[(size_t)w * 64 + l] = (uint32_t)q;
                }
            }
            mark_inject(I.word / kTileWords, t);
            note_birth(I.word / kTileWords, t);
            b.col = I.word * 64u + I.lo + ev_rank[q];
            if (I.nsrc > 1) {
                b.kind = BIRTH_GROUP;
                b.glo = I.lo;
                b.glen = I.nsrc;
                b.poff = np;
                for (uint32_t r = 0; r < I.nsrc; r++)
                    GP[np++] = col_phase[(size_t)I.word * 64 + I.lo + r];
            } else {
                b.kind = BIRTH_NORMAL;
            }
        }
        if (e.node >= v0 && e.node < v1) B[nb++] = b;  // row partition: own nodes only
    }
    // 3b. young tiles of this tick (young_kernel.h): every tile F_cur holds in slots (it was
    //     write-sparse last tick) plus fresh tiles opened by this tick's births; the youngest of
    //     them stay (or become) write-sparse while their oldest shares are <= young_age hops old.
    uint32_t ny = 0, nwt = 0, ny_read = 0, ny_leave = 0;
    bool skip_wr = false;  // this tick's slot writers stamp non-empty slots (young_skip)
    YoungPack* YP = young ? h_young[slot] : nullptr;
    std::vector<uint8_t> new_widx;
    if (young) {
        const uint32_t ntiles = hw / kTileWords;
        struct Cand {
            uint32_t tile;
            bool rd;
            int64_t first;
        };
        std::vector<Cand> cand;
        uint32_t nrd = 0;
        for (uint32_t tl = 0; tl < ntiles; tl++) {
            if (!tile_alloc[tl]) continue;
            const bool rd = tile_widx[tl] != 0xffu;
            const bool fresh = tile_first[tl] == t && t + 1 - tile_first[tl] <= opt_young_age;
            if (rd || fresh) cand.push_back(Cand{tl, rd, tile_first[tl]});
            nrd += rd;
        }
        std::sort(cand.begin(), cand.end(), [](const Cand& a, const Cand& b) {
            return a.first != b.first ? a.first > b.first : a.tile < b.tile;  // youngest first
        });
        new_widx.assign(tile_widx.size(), 0xffu);
        // read tiles sit at their F_cur entry index (young_kernel.h): nr = last tick's write count
        ny_read = (uint32_t)wt_last.size();
        for (uint32_t r = 0; r < ny_read; r++) YP->yt[r] = YoungTile{wt_last[r], 0u, (uint8_t)r, 0xffu, 0};
        uint32_t nfresh = 0;
        YoungTile fresh[kYoungMax];
        uint32_t fresh_room = kYoungMax > nrd ? kYoungMax - nrd : 0u;  // nrd <= kYoungWriteMax < kYoungMax
        for (const Cand& c : cand) {
            const bool wr_age = t + 1 - c.first <= opt_young_age && nwt < kYoungWriteMax;
            if (!c.rd) {
                if (!wr_age || fresh_room == 0) continue;  // stays a dense tile (it is dead this tick)
                fresh_room--;
            }
            YoungTile y{c.tile, (uint8_t)((c.rd ? YT_READ : 0u) | (wr_age ? YT_WRITE : 0u)),
                        c.rd ? tile_widx[c.tile] : (uint8_t)0xffu, (uint8_t)0xffu, 0};
            if (wr_age) {
                y.w_idx = (uint8_t)nwt;
                YP->wt[nwt++] = c.tile;
                new_widx[c.tile] = y.w_idx;
            }
            if (c.rd)
                YP->yt[y.r_idx] = y;  // (a read tile whose tile is gone keeps flags 0: no output)
            else
                fresh[nfresh++] = y;
        }
        std::sort(fresh, fresh + nfresh, [](const YoungTile& a, const YoungTile& b) { return a.tile < b.tile; });
        for (uint32_t k = 0; k < nfresh; k++) YP->yt[ny_read + k] = fresh[k];
        ny = ny_read + nfresh;
        for (uint32_t r = 0; r < ny_read; r++)
            if (YP->yt[r].flags == YT_READ) YP->lv[ny_leave++] = (uint8_t)r;
        std::sort(YP->lv, YP->lv + ny_leave, [&](uint8_t a, uint8_t b) { return YP->yt[a].tile < YP->yt[b].tile; });
        // young ids (the seen lists' tile index, young_kernel.h): a fresh young tile takes the lowest
        // free id; a tile leaving the set (or gone) gives its id back after this tick -- this
        // tick's k_pull_young drops its entries from every list, so no list still names it
        std::memset(YP->ymap, 0xff, sizeof(YP->ymap));
        std::memset(YP->wt_yid, 0xff, sizeof(YP->wt_yid));
        uint64_t yid_free_after = 0;
        for (uint32_t q = 0; q < ny; q++) {
            YoungTile& y = YP->yt[q];
            uint8_t id = tile_yid[y.tile];
            if (id == kYidNone) {  // a fresh tile
                const uint64_t avail = ~yid_used & ((1ull << 63) - 1ull);
                if (!avail) return set_error(GOSSIP_EHIP, "young ids exhausted");  // (<= 48 young tiles)
                id = (uint8_t)__builtin_ctzll(avail);
                yid_used |= 1ull << id;
                tile_yid[y.tile] = id;
            }
            y.yid = id;
            YP->ymap[id] = (uint8_t)q;
            if (y.flags & YT_WRITE) YP->wt_yid[y.w_idx] = id;
            else yid_free_after |= 1ull << id;  // leaving, or its tile is gone
        }
        for (uint32_t q = 0; q < ny; q++)
            if ((yid_free_after >> YP->yt[q].yid) & 1ull) tile_yid[YP->yt[q].tile] = kYidNone;
        yid_used &= ~yid_free_after;
        for (uint32_t q = 0; q < nb; q++) {
            const uint32_t tl = B[q].col >> 10;
            B[q].widx = tl < new_widx.size() ? new_widx[tl] : 0xffu;
            B[q].yid = B[q].widx != 0xffu ? tile_yid[tl] : kYidNone;
        }
        // empty-slot skipping: expected slot entries per node of F_next = sum over the write-sparse
        // tiles of columns x frontier fraction at F_next's hop (t - first: births are hop 0), and a
        // node's slot is non-empty with probability 1 - e^-entries
        skip_wr = false;
        if (opt_young_skip == 1) {
            skip_wr = nwt > 0;
        } else if (opt_young_skip == -1 && nwt) {
            double e = 0.0;
            for (uint32_t q = 0; q < nwt; q++) e += frontier_entries(YP->wt[q], t);
            skip_wr = 1.0 - std::exp(-e) < kSkipSlotFrac;
        }
    } else {
        for (uint32_t q = 0; q < nb; q++) B[q].widx = 0xffu;
    }
    // 3c. row chunks of the pipelined exchange: births grouped by chunk (a node has at most one
    //     birth per tick, so their order inside a launch is free)
    fused_rows = row_count > 1 && dense && opt_dense_fused && (comm || group_mode) && max_group_phases == 0 &&
                 !(cfg.flags & GOSSIP_F_NOSKIP);
    nchunks = (row_count > 1 && !fused_rows) ? (uint32_t)std::min<int64_t>(kMaxChunks, std::max<int64_t>(1, opt_xchunks)) : 1u;
    uint32_t cb_off[kMaxChunks + 1] = {};
    cb_off[1] = nb;
    if (nchunks > 1) {
        uint64_t clo[kMaxChunks + 1];
        for (uint32_t c = 0; c < nchunks; c++) chunk_rows(row_rank, c, &clo[c], &clo[c + 1]);
        auto chunk_of = [&](uint32_t v) {
            uint32_t c = 0;
            while (c + 1 < nchunks && v >= clo[c + 1]) c++;
            return c;
        };
        uint32_t cnt[kMaxChunks] = {};
        for (uint32_t q = 0; q < nb; q++) cnt[chunk_of(B[q].node)]++;
        for (uint32_t c = 0; c < nchunks; c++) cb_off[c + 1] = cb_off[c] + cnt[c];
        std::vector<Birth> tmp(B, B + nb);
        uint32_t at[kMaxChunks];
        std::copy(cb_off, cb_off + nchunks, at);
        for (uint32_t q = 0; q < nb; q++) B[at[chunk_of(tmp[q].node)]++] = tmp[q];
    }
    // 4. per-word control for this tick
    for (uint32_t w : reset_now) ctl[w].clear = ~0ull;
    const bool is_cut = (t == cut_tick && cut_r > 0);
    int snap_idx = -1;
    for (size_t s = 0; s < snaps.size() && !batch; s++)
        if (snaps[s].tick == t && snaps[s].r > 0) snap_idx = (int)s;
    WordCtl* C = h_ctl[slot];
    uint8_t* WF = h_wflags[slot];
    const size_t nsnap = batch ? snaps.size() : 0;
    bool smask_any = false;
    if (nsnap && hw) std::memset(h_smask[slot], 0, (size_t)nsnap * hw * 8);
    bool keep_any = false;  // some word has a keep mask (k_pull stages them in LDS)
    bool group_any = false; // some word holds an id group (k_dense_fused leaves those ticks to the 3-kernel path)
    for (uint32_t w = 0; w < hw; w++) {
        WordCtl c = ctl[w];
        if (batch) {
            // column c (generation at real time tb, batched birth tick bt) is at hop t - bt: its
            // arrival counts iff tb + hop*L' < t_cut (PrintStatistics), and toward snapshot s
            // iff tb + hop*L' < T_s, with L' = L (+ the share's serialisation, link timing)
            uint64_t km = 0ull;
            for (int bb = 0; bb < 64; bb++) {
                const uint32_t q = col_src[(size_t)w * 64 + bb];
                if (q == UINT32_MAX) {
                    km |= 1ull << bb;
                    continue;
                }
                const int64_t hop = t - ev[q].ns / L;
                const int64_t ta = ev_orig_ns[q] + hop * (L + (link_timing ? ev_delta[q] : 0));
                if (ta < cfg.t_cut_ns) km |= 1ull << bb;
                for (size_t s = 0; s < nsnap; s++)
                    if (hop >= 1 && ta < snaps[s].t_ns) {
                        h_smask[slot][s * hw + w] |= 1ull << bb;
                        smask_any = true;
                    }
            }
            c.keep = km;
        } else if (is_cut || snap_idx >= 0) {
            uint64_t km = 0ull, sm = 0ull;
            for (int bb = 0; bb < 64; bb++) {
                const int32_t ph = col_phase[(size_t)w * 64 + bb];
                if (is_cut && ph < cut_r) km |= 1ull << bb;
                if (snap_idx >= 0 && ph < snaps[snap_idx].r) sm |= 1ull << bb;
            }
            if (is_cut) c.keep = km;
            if (snap_idx >= 0) c.snap = sm;
        }
        C[w] = c;
        WF[w] = (uint8_t)((c.clear ? WF_CLEAR : 0u) | (c.gmask ? WF_GROUP : 0u) |
                          (c.keep != ~0ull ? WF_KEEP : 0u) | (c.snap ? WF_SNAP : 0u));
        keep_any |= c.keep != ~0ull;
        group_any |= c.gmask != 0ull;
    }
    if (const int64_t late = late_age_now())  // bottom-up early exit in k_pull (tiles >= late ticks old)
        for (uint32_t w = 0; w < hw; w++) {
            const uint32_t tl = w / kTileWords;
            if (tile_alloc[tl] && t + 1 - tile_first[tl] >= late) WF[w] |= (uint8_t)WF_LATE;
        }
    for (uint32_t i = 0; i < ny; i++)  // k_pull leaves these words to k_pull_young
        if (YP->yt[i].flags)
            for (uint32_t q = 0; q < kTileWords; q++) WF[YP->yt[i].tile * kTileWords + q] |= (uint8_t)WF_YOUNG;
    for (uint32_t w : reset_now) ctl[w].clear = 0ull;
    for (uint32_t q = 0; q < nb; q++)  // (k_dense_fused writes the 16-word tiles births land in)
        if (B[q].kind == BIRTH_NORMAL || B[q].kind == BIRTH_GROUP) WF[B[q].col >> 6] |= (uint8_t)WF_BIRTH;
    // 4b. k_pull's pass -> tile lists (option pull_tiles), one per launch window: the allocated,
    //     non-young tiles, grouped by occupancy word and padded to whole passes of LPW / 8 tiles
    //     (LPW as run_pull picks it below).  Young tiles are k_pull_young's, retired tiles hold
    //     nothing; a pass then never spends its lanes on them.
    pt_off.clear();
    pt_cnt.clear();
    const bool use_ptile = opt_pull_tiles && !dense && !(cfg.flags & GOSSIP_F_NOSKIP) && hw;
    pt_used = use_ptile;
    const bool sat_on = use_ptile && opt_pull_sat != 0 && row_count == 1 && !(cfg.flags & GOSSIP_F_NOSKIP) && d_sat;
    const bool dr_used = use_ptile && opt_dense_rows != 0 && row_count == 1 && !(cfg.flags & GOSSIP_F_NOSKIP);
    if (use_ptile) {
        const uint64_t need = (uint64_t)hw / kTileWords + 16ull * ((hw + kPullLdsWords - 1) / kPullLdsWords) + 16;
        if (need > ptile_cap) {
            HIP_TRY(hipStreamSynchronize(stream));
            for (int k = 0; k < kRing; k++) {
                hipFree(d_ptile[k]);
                hipHostFree(h_ptile[k]);
                HIP_TRY(hipMalloc(&d_ptile[k], need * 2));
                HIP_TRY(hipHostMalloc(&h_ptile[k], need * 2, hipHostMallocDefault));
            }
            ptile_cap = need;
        }
        uint16_t* P = h_ptile[slot];
        uint32_t at = 0;
        for (uint32_t wb = 0; wb < hw; wb += kPullLdsWords) {
            const uint32_t wl = std::min(kPullLdsWords, hw - wb);
            int lpw = 8;
            while (lpw < 64 && 2 * lpw < (int)wl) lpw *= 2;
            if (lpw == 64) lpw = kWideLanes;  // (run_pull: wide windows)
            const uint32_t tpp = (uint32_t)lpw / 8u;
            pt_off.push_back(at);
            const uint32_t t0 = wb / kTileWords, t1 = (wb + wl) / kTileWords;
            // per occupancy word, the tiles in age order (option pull_tile_order): a pass's tiles
            // then reach their early exit (late_age) after similar numbers of peer batches, so
            // fewer lanes idle while the wave finishes the pass's slowest tile
            std::vector<uint32_t> grp;
            auto flush = [&]() {
                if (opt_pull_tile_order)
                    std::stable_sort(grp.begin(), grp.end(), [&](uint32_t x, uint32_t y) { return tile_first[x] < tile_first[y]; });
                for (uint32_t tl : grp) P[at++] = (uint16_t)(tl - t0);
                for (size_t k = grp.size(); k % tpp; k++) P[at++] = 0xffffu;
                grp.clear();
            };
            uint32_t group_tw = 0xffffffffu;
            for (uint32_t tl = t0; tl < t1; tl++) {
                if (!tile_alloc[tl] || (WF[tl * kTileWords] & WF_YOUNG) PULL_DIAG_SKIP(tl)) continue;
                const uint32_t tw = tl >> 6;
                if (tw != group_tw) {  // a pass never straddles two occupancy words
                    flush();
                    group_tw = tw;
                }
                grp.push_back(tl);
            }
            flush();
            pt_cnt.push_back(at - pt_off.back());
        }
        if (at) HIP_TRY(hipMemcpyAsync(d_ptile[slot], P, (size_t)at * 2, hipMemcpyHostToDevice, stream));
    }
    // 4c. saturation bits and dense-row tiles of k_pull (pull_kernel.h), per listed tile:
    //   dense row (TM_DENSE): every node's F_cur row of the tile was written last tick (WF_DW by
    //     k_pull, YT_DW by k_pull_young for a tile leaving the young set) -- read without
    //     occupancy words;
    //   WF_DW: the tile's F_cur at the next tick is expected dense (dense_row_hop), so k_pull
    //     writes every node's row this tick;
    //   sat trusted (TM_SATOK): k_pull wrote the tile's sat bits last tick (listed then, same life)
    //     and no birth landed in it since then (a birth adds a live column the bits did not see);
    //   TM_NZ: listed and not dense-row: the tiles that still need their peers' occupancy words.
    // Row partitions keep neither (another rank's rows arrive only where occupied).
    sat_used = sat_on;
    last_dense_tiles = 0;
    // push marks ride on the saturation words (an unmarked node's push tiles read as saturated)
    const bool push_on = sat_on && opt_pull_push != 0 && d_mark[0];
    bool pushw_any = false;
    if (sat_used || dr_used) {
        if (TM_WORDS * ntw > tmask_cap) {
            HIP_TRY(hipStreamSynchronize(stream));
            const uint32_t cap = TM_WORDS * std::max<uint32_t>(ntw, 8u);
            for (int k = 0; k < kRing; k++) {
                hipFree(d_tmask[k]);
                hipHostFree(h_tmask[k]);
                HIP_TRY(hipMalloc(&d_tmask[k], (size_t)cap * 8));
                HIP_TRY(hipHostMalloc(&h_tmask[k], (size_t)cap * 8, hipHostMallocDefault));
            }
            tmask_cap = cap;
        }
        unsigned long long* TM = h_tmask[slot];
        std::memset(TM, 0, (size_t)TM_WORDS * ntw * 8);
        const uint32_t ntiles = hw / kTileWords;
        // Push-write tiles only when the NEXT tick is expected light: every tile k_pull will list
        // then (the listed ones now, the tiles leaving the young set now) has its F_next on few
        // enough nodes (push_write) and none turns dense-row.  The k_pull instantiation that reads
        // and writes marks holds more registers (pull_kernel.h PUSH): on a tick with dense tiles
        // (every C4 tick at 2 shards) it costs more than it skips (58.4 -> 60.1 ms per phase).
        bool light_next = push_on;
        if (push_on && opt_pull_push != 1) {
            for (uint32_t tl = 0; tl < ntiles && light_next; tl++)
                if (tile_alloc[tl] && !(WF[tl * kTileWords] & WF_YOUNG))
                    light_next = push_write(tl, t) && !(dr_used && dense_row_hop(tl, t - tile_first[tl]));
            for (uint32_t i = 0; young && i < ny_leave && light_next; i++)
                light_next = push_write(YP->yt[YP->lv[i]].tile, t);
        }
        for (uint32_t tl = 0; tl < ntiles; tl++) {
            if (!tile_alloc[tl] || (WF[tl * kTileWords] & WF_YOUNG) PULL_DIAG_SKIP(tl)) continue;  // not listed
            const unsigned long long bit = 1ull << (tl & 63u);
            unsigned long long* m = TM + (size_t)TM_WORDS * (tl >> 6);
            const bool fresh = tile_first[tl] == t;
            const bool dr = dr_used && !fresh && tile_dw[tl] == t - 1;
            if (dr) last_dense_tiles++;
            m[dr ? TM_DENSE : TM_NZ] |= bit;
            // sat bits written by k_pull last tick, no birth since
            const bool clean = !fresh && tile_last_inject[tl] != t - 1 && tile_inj_prev[tl] != t - 1;
            if (sat_used && clean && tile_satw[tl] == t - 1) m[TM_SATOK] |= bit;
            bool dw = false;
            if (dr_used && dense_row_hop(tl, t - tile_first[tl])) {  // F_cur's hop next tick
                for (uint32_t q = 0; q < kTileWords; q++) WF[tl * kTileWords + q] |= (uint8_t)WF_DW;
                tile_dw[tl] = t;
                dw = true;
            }
            // push marks: the tile's F_cur rows were written by last tick's k_pull alone (listed then
            // with TM_PUSHW, no birth since) -> skipped at unmarked nodes; this tick's rows mark
            // peers when next tick's frontier is expected on few nodes
            // (births of t - 1 into the tile marked their nodes' peers too: k_births)
            if (push_on && !dr && !fresh && tile_pushw[tl] == t - 1) {
                m[TM_PUSH] |= bit;
                push_tiles++;
            }
            if (light_next && !dw && push_write(tl, t)) {  // (tile_pushw: set by the launch that marks)
                m[TM_PUSHW] |= bit;
                pushw_any = true;
            }
            tile_listed[tl] = t;
        }
        if (dr_used && young)  // tiles leaving the young set: k_pull_young writes their dense rows
            for (uint32_t i = 0; i < ny_leave; i++) {
                YoungTile& y = YP->yt[YP->lv[i]];
                if (dense_row_hop(y.tile, t - tile_first[y.tile])) {
                    y.flags |= (uint8_t)YT_DW;
                    tile_dw[y.tile] = t;
                }
            }
        HIP_TRY(hipMemcpyAsync(d_tmask[slot], TM, (size_t)TM_WORDS * ntw * 8, hipMemcpyHostToDevice, stream));
    }
    // 5. upload + launches
    const uint32_t wact = hw;
    if (wact) HIP_TRY(hipMemcpyAsync(d_ctl[slot], C, (size_t)wact * sizeof(WordCtl), hipMemcpyHostToDevice, stream));
    if (wact) HIP_TRY(hipMemcpyAsync(d_wflags[slot], WF, (size_t)wact, hipMemcpyHostToDevice, stream));
    if (nb) HIP_TRY(hipMemcpyAsync(d_births[slot], B, (size_t)nb * sizeof(Birth), hipMemcpyHostToDevice, stream));
    if (np) HIP_TRY(hipMemcpyAsync(d_gphase[slot], GP, (size_t)np * 4, hipMemcpyHostToDevice, stream));
    if (smask_any) HIP_TRY(hipMemcpyAsync(d_smask[slot], h_smask[slot], nsnap * hw * 8, hipMemcpyHostToDevice, stream));
    if (ny) HIP_TRY(hipMemcpyAsync(d_young[slot], YP, sizeof(YoungPack), hipMemcpyHostToDevice, stream));
    HIP_TRY(hipEventRecord(slot_done[slot], stream));
    const int lv = (int)(t % 3);
    if (wact) HIP_TRY(hipMemsetAsync(d_live[lv], 0, (size_t)wact * 8, stream));
    unsigned long long* snap_ptr = snap_idx >= 0 ? d_scalars + 2 + 2 * snap_idx + 1 : nullptr;
    const int nxt = fcur ^ 1;
    // DENSE ticks run k_dense_fused (dense_kernel.h) unless the tick has id groups, row chunks
    // (row partition: other ranks' rows reach F_next without FT), or the diagnostic no-skip pull
    const bool fused_tick = dense && wact && opt_dense_fused && nchunks == 1 && (row_count == 1 || fused_rows) &&
                            !(cfg.flags & GOSSIP_F_NOSKIP) && !group_any && ntw <= kFActWords &&
                            (uint64_t)(wact / 4u) * (n_pad / kStageK) < (1ull << 20);  // (its packed unit scan)
    if (fused_rows && wact && !fused_tick)  // (the other ranks' F rows are not exchanged)
        return set_error(GOSSIP_ECAPACITY, "fused row partition: the window outgrew the fused kernel (<= 4,096 words)");
    // births [off, off + cnt) of the staged array (all of them, or one row chunk's)
    auto launch_births = [&](uint32_t off, uint32_t cnt) -> int {
        if (!cnt) return GOSSIP_OK;
        BirthArgs b;
        b.b = d_births[slot] + off; b.nb = cnt; b.gphase = d_gphase[slot];
        b.Fnext = d_F[nxt]; b.seen = d_seen; b.stride = stride;
        b.gen = d_gen; b.recv = d_recv; b.effgen = d_effgen; b.sent = d_sent; b.deg = d_deg;
        b.live = d_live[lv]; b.snap = snap_ptr; b.snap_r = snap_idx >= 0 ? snaps[snap_idx].r : 0;
        b.nz = d_nz[nxt];
        b.ntw = ntw;
        b.degc = d_degc;
        b.slot = (young && nwt) ? d_slot[nxt] : nullptr;
        b.cap = (uint32_t)std::min<int64_t>(kSlotU16 - 1, std::max<int64_t>(1, opt_young_cap));
        b.wt = young ? d_young[slot]->wt : nullptr;
        b.nwt = nwt;
        b.rowptr = d_rowptr; b.rev = d_rev;
        b.hint_next = young ? d_hint[nxt] : nullptr;
        b.stamp_next = hint_stamp(t);
        b.stamp1_next = hint_stamp1(t);
        b.sparse_wr = skip_wr ? 1u : 0u;
        b.mark_next = pushw_any ? d_mark[t & 1] : nullptr;
        b.tmask = pushw_any ? d_tmask[slot] : nullptr;
        b.col = d_col;
        b.list = d_ylist;
        b.list_max = (uint32_t)opt_young_list_cap;
        b.wt_yid = young ? d_young[slot]->wt_yid : nullptr;
        if (fused_tick) {
            b.FTn = d_FT[nxt];
            b.snz_n = d_snz[(t + 1) % 3];
            b.kw = n_pad / 32u;
            b.nstw = snz_nstw;
        }
        k_births<<<(cnt + 255) / 256, 256, 0, stream>>>(b);
        HIP_TRY(hipGetLastError());
        return GOSSIP_OK;
    };
    // end of row chunk c on the engine stream: its exchange may start (exchange_rccl, export)
    auto end_chunk = [&](uint32_t c) -> int {
        if (!ev_chunk[c]) HIP_TRY(hipEventCreateWithFlags(&ev_chunk[c], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev_chunk[c], stream));
        return GOSSIP_OK;
    };
    if (wact) {
        PullArgs a;
        a.rowptr = d_rowptr; a.col = d_col;
        if (handshake && t == tick0 + 3) {  // shares sent in [t_start+2L, t_start+3L): a -> b only
            a.rowptr = d_rowptr_c;
            a.col = d_col_c;
        }
        a.Fcur = d_F[fcur]; a.Fnext = d_F[nxt]; a.seen = d_seen; a.ctl = d_ctl[slot];
        a.wflags = d_wflags[slot];
        a.recv = d_recv; a.live = d_live[lv]; a.snap = snap_ptr;
        a.live_prev = (t - 1 >= tick0) ? d_live[(t - 1) % 3] : nullptr;
        a.acct = d_acct;
        a.nz_cur = d_nz[fcur];
        a.nz_next = d_nz[nxt];
        a.ntw = ntw;
        a.n = v1; a.stride = stride; a.wbase = 0; a.wact = wact;
        a.v0 = v0;  // row partition: this engine's rows [v0, v1)
        a.noskip = (cfg.flags & GOSSIP_F_NOSKIP) ? 1u : 0u;
        a.keep_lds = keep_any ? 1u : 0u;
        a.gate_seen = opt_pull_gate ? 1u : 0u;
        // non-temporal rows iff the frontier the launch gathers from (n rows x wact live words)
        // exceeds kPullNtBytes
        const bool nt_rows = opt_pull_nt >= 0 ? opt_pull_nt == 1 : (uint64_t)n * wact * 8u > kPullNtBytes;
        // blocks for rows [lo, hi): 64 nodes per wave step sequence, 4 waves per block
        auto grid_for = [&](uint64_t lo, uint64_t hi) {
            const uint64_t chunks = (hi - lo + 63) / 64;
            return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((chunks + 3) / 4, pull_grid_cap(nt_rows, opt_pull_grid)));
        };
        const uint32_t grid = grid_for(v0, v1);
        last_nt = nt_rows ? 1u : 0u;
        last_grid = grid;
        const double avg_deg = n ? (double)nnz / n : 0.0;
        // One launch per kPullLdsWords words of the window (its per-word state lives in LDS).
        // Lane layout: word-lanes cover the launch's words in one pass when possible (at least
        // the 8 word-pairs of one tile); spare lanes of the wave split the peer list
        // (edge-lanes) when peers are many -- and never in DENSE mode, which gathers nothing.
        auto run_pull = [&](const PullArgs& base, bool split_edges) {
            const uint32_t grid = grid_for(base.v0, base.n);
            for (uint32_t wb = 0, li = 0; wb < wact; wb += kPullLdsWords, li++) {
                PullArgs c = base;
                c.wbase = wb;
                c.wact = std::min(kPullLdsWords, wact - wb);
                if (use_ptile && split_edges && li < pt_off.size()) {
                    c.ptile = d_ptile[slot] + pt_off[li];
                    c.nptile = pt_cnt[li];
                }
                int lpw = 8;
                while (lpw < 64 && 2 * lpw < (int)c.wact) lpw *= 2;
                // windows wider than 64 words keep one peer walk per node (the pipelined path)
                const bool wide_window = lpw == 64 && split_edges;
                if (wide_window) lpw = kWideLanes;
                int epn = 1;
                while (split_edges && !wide_window && lpw * epn * 2 <= 64 && epn * 8 < avg_deg) epn *= 2;
                // saturation bits / dense-row tiles: the gathering kernel (EPN 1) over tile lists
                size_t extra_lds = 0;
                if (c.ptile && epn == 1 && (sat_used || dr_used)) {
                    c.tmask = d_tmask[slot];
                    c.sat = sat_used ? d_sat : nullptr;
                    if (push_on && pull_sp(lpw, epn, c)) {  // marks of last tick's push-write rows / this tick's
                        c.mark_cur = mark_tick == t - 1 ? d_mark[(t - 1) & 1] : nullptr;
                        mark_launches += c.mark_cur != nullptr;
                        c.mark_next = pushw_any ? d_mark[t & 1] : nullptr;
                        // a tile is read as a push tile next tick only if a launch that marks
                        // covered it (tile_pushw): the mark bitmap then holds every writer's peers
                        if (c.mark_next)
                            for (uint32_t tl = wb / kTileWords; tl < (wb + c.wact) / kTileWords; tl++)
                                if ((h_tmask[slot][(size_t)TM_WORDS * (tl >> 6) + TM_PUSHW] >> (tl & 63u)) & 1ull) {
                                    tile_pushw[tl] = t;
                                    pushw_tiles++;
                                }
                    }
                    extra_lds = kPullSatLds + ((c.mark_cur || c.mark_next) ? kPullPushLds : 0);
                    sat_launches += sat_used;
                    if (sat_used)  // this launch writes the sat bits of its listed tiles
                        for (uint32_t tl = wb / kTileWords; tl < (wb + c.wact) / kTileWords; tl++)
                            if (tile_listed[tl] == t) tile_satw[tl] = t;
                }
                last_lpw = (uint32_t)lpw;
                const size_t lds = pull_lds_bytes(c.wact, c.keep_lds != 0, c.nptile) + extra_lds;
                launch_pull(lpw, epn, nt_rows, grid, lds, stream, c);
            }
        };
        hipEvent_t e0 = nullptr, e1 = nullptr, p0 = nullptr, p1 = nullptr;
        a.inc = nullptr;
        // DENSE phase = transpose + MFMA + dedup, timed as ONE unit (below)
        const bool dense_timing = dense && (cfg.flags & GOSSIP_F_TIMING);
        // The DENSE phase is timed on the device by two one-thread stamp kernels around it
        // (k_phase_start, k_phase_acc): an event pair around the phase also counted the host's
        // launch latency (273 us against a 136 us span on C2, profiles/r04).
        unsigned long long* pts = dense_timing ? d_phase_ts : nullptr;
        // a fused tick after a three-kernel one: the stage masks it writes were not zeroed, and
        // k_transpose builds the ones it reads
        if (fused_tick && !ft_valid)
            for (int64_t k = 0; k < 2; k++)
                HIP_TRY(hipMemsetAsync(d_snz[(t + k) % 3], 0, (size_t)(stride / 4u) * snz_nstw * 8u, stream));
        if (pts) k_phase_start<<<1, 1, 0, stream>>>(pts);
        if (dense && !(fused_tick && ft_valid)) {
            // transpose the frontier to share-column bit rows (the fused path's FT[fcur] was
            // written by the last tick's k_dense_fused + k_births)
            dim3 eg(n_pad / 256u, wact);
            k_transpose<<<eg, 256, 0, stream>>>(d_F[fcur], stride, n, n_pad / 32u, wact, a.live_prev,
                                                d_nz[fcur], ntw, d_FT[fcur], fused_tick ? d_snz[t % 3] : nullptr,
                                                snz_nstw);
            HIP_TRY(hipGetLastError());
        }
        // young tiles beside k_pull: the two kernels touch disjoint words; they share the per-node
        // counters and occupancy words, which k_pull then updates atomically (shared_out) into
        // occupancy words zeroed here
        const bool overlap = !dense && ny && opt_young_overlap != 0;
        if (overlap) {
            if (!ystream) {
                // (launch order, stream priorities and smaller young grids measured no better:
                // profiles/r02, r03/ab/r3v_*; those variants were removed in round 5)
                HIP_TRY(hipStreamCreateWithFlags(&ystream, hipStreamNonBlocking));
                HIP_TRY(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
                HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
            }
            HIP_TRY(hipMemsetAsync(d_nz[nxt] + (uint64_t)v0 * ntw, 0, (size_t)(v1 - v0) * ntw * 8u, stream));
            a.shared_out = 1u;
        } else if (use_ptile) {
            // k_pull writes whole occupancy words only for the words its listed tiles fall in
            HIP_TRY(hipMemsetAsync(d_nz[nxt] + (uint64_t)v0 * ntw, 0, (size_t)(v1 - v0) * ntw * 8u, stream));
        }
        if (pushw_any)  // this tick's push marks start empty (last read by the pull of t - 1)
            HIP_TRY(hipMemsetAsync(d_mark[t & 1], 0, ((size_t)n + 64) / 64 * 8, stream));
        if (cfg.flags & GOSSIP_F_TIMING) {
            e0 = get_event();
            e1 = get_event();
            HIP_TRY(hipEventRecord(e0, stream));
            if (!dense) {  // (every tick: a tick without young tiles is a phase of k_pull alone)
                p0 = get_event();
                HIP_TRY(hipEventRecord(p0, stream));
            }
        }
        auto launch_young = [&](hipStream_t ys) -> int {
            YoungArgs y;
            y.rowptr = a.rowptr; y.col = a.col;
            y.Fcur = d_F[fcur]; y.Fnext = d_F[nxt]; y.seen = d_seen;
            y.slot_cur = d_slot[fcur]; y.slot_next = d_slot[nxt];
            y.ctl = d_ctl[slot]; y.wflags = d_wflags[slot];
            y.recv = d_recv; y.live = d_live[lv];
            y.snap = snap_ptr; y.acct = d_acct; y.nz_next = d_nz[nxt]; y.ntw = ntw;
            y.yt = d_young[slot]->yt; y.ny = ny; y.nr = ny_read; y.nt = ny_leave;
            y.lv = d_young[slot]->lv;
            y.n = v1; y.v0 = v0; y.stride = stride;
            y.cap = (uint32_t)std::min<int64_t>(kSlotU16 - 1, std::max<int64_t>(1, opt_young_cap));
            y.hint_cur = d_hint[fcur]; y.hint_next = d_hint[nxt]; y.rev = d_rev;
            y.stamp_cur = hint_stamp(t - 1); y.stamp_next = hint_stamp(t);
            y.stamp1_cur = hint_stamp1(t - 1); y.stamp1_next = hint_stamp1(t);
            y.sparse_rd = (skip_wr_last && ny_read) ? 1u : 0u;  // (last tick's writers stamped)
            y.sparse_wr = skip_wr ? 1u : 0u;
            // idle nodes skip the node walk (young_kernel.h) when only stamped slots are read and
            // every read tile stays young (no list entry is dropped or materialised)
            bool stay = true;
            for (uint32_t r = 0; r < ny_read; r++) stay &= (YP->yt[r].flags & YT_WRITE) != 0;
            y.fast = (opt_young_idle != 0 && (y.sparse_rd || !ny_read) && stay) ? 1u : 0u;
            y.work = d_ywork;
            idle_ticks += y.fast;
            skip_ticks += y.sparse_rd;
            y.slot_nt = opt_young_nt ? 1u : 0u;
            y.list = d_ylist;
            // (k_pull_young leaves kListReserve entries of the capacity to k_births' appends)
            y.list_cap = opt_young_list_cap > 2 * (int64_t)kListReserve ? (uint32_t)opt_young_list_cap - kListReserve
                                                                        : (uint32_t)opt_young_list_cap / 2u;
            y.ymap = d_young[slot]->ymap;
            const uint32_t yg = (uint32_t)std::max<uint64_t>(
                1, std::min<uint64_t>(((uint64_t)(v1 - v0) + 3) / 4,
                                      opt_young_grid > 0 ? (uint64_t)opt_young_grid : 2u * pull_grid_cap(nt_rows, opt_pull_grid)));
            hipEvent_t y0 = nullptr, y1 = nullptr;
            if (cfg.flags & GOSSIP_F_TIMING) {
                y0 = get_event();
                y1 = get_event();
                HIP_TRY(hipEventRecord(y0, ys));
            }
            last_young_grid = yg;
            if (y.fast) {  // the idle nodes first (young_kernel.h, k_young_idle)
                const uint64_t nch = ((uint64_t)(v1 - v0) + 63) / 64;
                k_young_idle<<<(uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((nch + 3) / 4, 16384)), 256, 0, ys>>>(y);
            }
            if (y.sparse_rd || y.fast || !ny_read)
                k_pull_young<true><<<yg, 256, young_lds_bytes(ny, ny_read), ys>>>(y);
            else
                k_pull_young<false><<<yg, 256, young_lds_bytes(ny, ny_read), ys>>>(y);
            HIP_TRY(hipGetLastError());
            if (cfg.flags & GOSSIP_F_TIMING) {
                HIP_TRY(hipEventRecord(y1, ys));
                timers_young.emplace_back(y0, y1);
            }
            young_launches++;
            return GOSSIP_OK;
        };
        // DENSE mode: dedup of the incoming words of rows [base.v0, base.n), one node per wave
        // step, the grid sized to the rows (k_dense_dedup, dense_kernel.h)
        auto run_dedup = [&](const PullArgs& base) {
            const uint64_t rows = base.n > base.v0 ? base.n - base.v0 : 0;
            const uint32_t g = (uint32_t)std::max<uint64_t>(
                1, std::min<uint64_t>((rows + kDedupWaves - 1) / kDedupWaves, 2u * (uint32_t)num_cus));
            for (uint32_t wb = 0; wb < wact; wb += kPullLdsWords) {
                PullArgs c = base;
                c.wbase = wb;
                c.wact = std::min(kPullLdsWords, wact - wb);
                k_dense_dedup<<<g, 64 * kDedupWaves, pull_lds_bytes(c.wact, c.keep_lds != 0), stream>>>(c);
            }
        };
        // the MFMA contraction of rows [lo, hi) (DENSE mode) into the incoming words
        auto run_dense = [&](uint64_t lo, uint64_t hi) -> int {
            BitsArgs gm;
            gm.Ab = d_Ab; gm.FT = d_FT[fcur]; gm.inc = d_inc; gm.live_prev = a.live_prev; gm.acct = d_acct;
            gm.n = (uint32_t)hi; gm.n_pad = n_pad; gm.kw = n_pad / 32u; gm.stride = stride;
            gm.mb0 = (uint32_t)lo / kDenseTile;  // row partition: this engine's row blocks only
            gm.mb = (std::min((uint32_t)hi + kDenseTile - 1u, n_pad) - (uint32_t)lo) / kDenseTile;
            gm.nt = wact / 4u;
            const uint32_t nst = n_pad / kStageK;
            uint32_t ks = 1;  // split K until the chip has ~2 tiles per CU (>= 2 stages per split)
            const uint64_t min_tiles = (uint64_t)std::max<int64_t>(1, opt_dense_min_tiles);
            while ((uint64_t)gm.mb * gm.nt * ks < min_tiles && ks * 4 <= nst) ks *= 2;
            gm.ksplit = ks;
            gm.total = gm.mb * gm.nt * ks;
            k_dense_bits<<<(gm.total + 7u) / 8u * 8u, 512, 0, stream>>>(gm);
            HIP_TRY(hipGetLastError());
            return GOSSIP_OK;
        };
        if (nchunks > 1) {
            // Pipelined exchange: pull (+ the MFMA contraction) and births per row chunk, each
            // chunk closed by its event so that its exchange overlaps the next chunk.  Timed as
            // without chunks: the MFMA contraction (DENSE) or the pull (CSR), summed over chunks.
            const bool timing = (cfg.flags & GOSSIP_F_TIMING) != 0;
            for (uint32_t c = 0; c < nchunks; c++) {
                uint64_t lo, hi;
                chunk_rows(row_rank, c, &lo, &hi);
                if (hi > lo) {  // (chunk 0 never is empty: a rank owns >= 512 rows)
                    hipEvent_t c0 = timing ? (c ? get_event() : e0) : nullptr;
                    hipEvent_t c1 = timing ? (c ? get_event() : e1) : nullptr;
                    if (timing) HIP_TRY(hipEventRecord(c0, stream));
                    PullArgs ac = a;
                    ac.v0 = (uint32_t)lo;
                    ac.n = (uint32_t)hi;
                    if (dense) {
                        const int rc = run_dense(lo, hi);
                        if (rc) return rc;
                        if (timing) HIP_TRY(hipEventRecord(c1, stream));
                        ac.inc = d_inc;
                        run_dedup(ac);
                    } else {
                        run_pull(ac, true);
                        if (timing) HIP_TRY(hipEventRecord(c1, stream));
                    }
                    if (timing) timers.emplace_back(c0, c1);
                }
                int rc = launch_births(cb_off[c], cb_off[c + 1] - cb_off[c]);
                if (rc) return rc;
                if ((rc = end_chunk(c))) return rc;
            }
            if (pts) k_phase_acc<<<1, 1, 0, stream>>>(pts);  // (row chunks: the chunks' births are inside the span)
            if (p0) event_pool.push_back(p0);  // (timed per chunk above)
        } else if (fused_tick) {
            // the whole DENSE pull in one persistent kernel (contraction, dedup, FT of F_next)
            FusedArgs f;
            // a row rank: its rows [v0, v1) (row blocks of 256 from v0 / 256; v0 is 512-aligned)
            const uint64_t r0 = row_count > 1 ? v0 : 0u;
            const uint32_t rows = row_count > 1 ? v1 - v0 : n;
            f.Ab = d_Ab + r0 * (n_pad / 32u); f.FTc = d_FT[fcur]; f.FTn = d_FT[nxt] + r0 / 32u;
            f.mb0 = (uint32_t)(r0 / kDenseTile);
            f.snz_c = d_snz[t % 3];  // (by the last tick's fused kernel + births, or k_transpose above)
            f.snz_n = d_snz[(t + 1) % 3];
            f.snz_z = d_snz[(t + 2) % 3];
            f.snz_zwords = (stride / 4u) * snz_nstw;
            f.seen = d_seen + r0 * stride; f.Fnext = d_F[nxt] + r0 * stride; f.ctl = d_ctl[slot]; f.wflags = d_wflags[slot];
            f.recv = d_recv + r0; f.live = d_live[lv]; f.live_prev = a.live_prev; f.snap = snap_ptr; f.acct = d_acct;
            f.nz_next = d_nz[nxt] + r0 * ntw; f.ntw = ntw;
            f.n = rows; f.n_pad = n_pad; f.kw = n_pad / 32u; f.stride = stride;
            f.nst = n_pad / kStageK; f.nstw = snz_nstw;
            f.mb = row_count > 1 ? (rows + kDenseTile - 1u) / kDenseTile : n_pad / kDenseTile;
            f.nt = wact / 4u; f.total = f.mb * f.nt;
            if (f.nt > kFMaxCt)  // (fused_tick's ntw gate implies it: the kernel's LDS tables hold kFMaxCt)
                return set_error(GOSSIP_EHIP, "k_dense_fused: window wider than its column-tile tables");
            f.wact = wact;
            f.inc = d_inc + r0 * stride;
            f.tix = d_tix;
            f.rmax = dense_rounds < 0 ? 0xffffffffu : (uint32_t)dense_rounds;
            f.pts = (pts && ft_valid) ? pts : nullptr;  // (a tick with k_transpose keeps the stamp-kernel span)
            f.gm = (uint32_t)std::min<int64_t>(dense_gm, 64);
            uint32_t fg = (uint32_t)std::min<uint64_t>(f.total, (uint64_t)num_cus);
            if (fg >= 8u) fg &= ~7u;
            k_dense_fused<<<fg, 512, 0, stream>>>(f);
            HIP_TRY(hipGetLastError());
            fused_launches++;
            if (cfg.flags & GOSSIP_F_TIMING) {
                HIP_TRY(hipEventRecord(e1, stream));
                timers.emplace_back(e0, e1);
            }
            if (pts) k_phase_acc<<<1, 1, 0, stream>>>(pts);
        } else if (dense) {
            // The timed kernel in DENSE mode is the MFMA contraction (pull_ms); its incoming
            // words are then consumed by k_dense_dedup.  The whole phase -- transpose, MFMA,
            // dedup -- is timed as pull_phase_ms.
            const int rc = run_dense(v0, v1);
            if (rc) return rc;
            if (cfg.flags & GOSSIP_F_TIMING) {
                HIP_TRY(hipEventRecord(e1, stream));
                timers.emplace_back(e0, e1);
            }
            a.inc = d_inc;
            run_dedup(a);
            if (pts) k_phase_acc<<<1, 1, 0, stream>>>(pts);
        } else if (opt_rehearse_rows > 1 && !ny) {
            // row-partition rehearsal: one pull launch per rank's row range, each timed
            for (uint32_t r = 0; r + 1 < (uint32_t)rr_lo.size(); r++) {
                PullArgs ar = a;
                ar.v0 = (uint32_t)rr_lo[r];
                ar.n = (uint32_t)rr_lo[r + 1];
                if (ar.n <= ar.v0) continue;
                hipEvent_t ra = nullptr, rb = nullptr;
                if (cfg.flags & GOSSIP_F_TIMING) {
                    ra = get_event();
                    rb = get_event();
                    HIP_TRY(hipEventRecord(ra, stream));
                }
                run_pull(ar, true);
                if (cfg.flags & GOSSIP_F_TIMING) {
                    HIP_TRY(hipEventRecord(rb, stream));
                    rr_events.push_back({r, 0u, ra, rb});
                }
            }
            if (cfg.flags & GOSSIP_F_TIMING) {
                HIP_TRY(hipEventRecord(e1, stream));
                timers.emplace_back(e0, e1);
                if (p0) event_pool.push_back(p0);  // (no phase timer on this path)
            }
        } else {
            if (overlap) {
                HIP_TRY(hipEventRecord(ev_fork, stream));
                HIP_TRY(hipStreamWaitEvent(ystream, ev_fork, 0));
                const int rc = launch_young(ystream);
                if (rc) return rc;
            }
            run_pull(a, true);
            if (cfg.flags & GOSSIP_F_TIMING) {
                HIP_TRY(hipEventRecord(e1, stream));
                timers.emplace_back(e0, e1);
            }
            if (overlap) {
                HIP_TRY(hipEventRecord(ev_join, ystream));
                HIP_TRY(hipStreamWaitEvent(stream, ev_join, 0));
            } else if (ny) {  // the young tiles (young_kernel.h), after k_pull wrote the nz words
                const int rc = launch_young(stream);
                if (rc) return rc;
            }
            if (p0 && (cfg.flags & GOSSIP_F_TIMING)) {  // the whole pull phase
                p1 = get_event();
                HIP_TRY(hipEventRecord(p1, stream));
                timers_phase.emplace_back(p0, p1);
            }
        }
        HIP_TRY(hipGetLastError());
        pull_launches++;
        pull_bytes += 8ull * (n + 1) + 4ull * nnz + 8ull * wact * nnz + 24ull * wact * n + 16ull * n;
    }
    if (nchunks == 1 || !wact) {  // (chunked ticks with live words launched them per chunk)
        for (uint32_t c = 0; c < nchunks; c++) {
            int rc = launch_births(nchunks == 1 ? 0u : cb_off[c], nchunks == 1 ? nb : cb_off[c + 1] - cb_off[c]);
            if (rc) return rc;
            if ((rc = end_chunk(c))) return rc;
        }
    }
    if (young) {  // F_next's slots hold this tick's write-sparse tiles: next tick reads them
        tile_widx.swap(new_widx);
        wt_last.assign(YP->wt, YP->wt + nwt);
        skip_wr_last = skip_wr && ny && wact;  // (stamped only if this tick launched the young kernel)
    }
    if (smask_any) {  // hop-batched snapshots: arrivals of this tick that precede each snapshot
        const uint64_t cells = (uint64_t)(v1 - v0) * hw;
        const uint32_t g = (uint32_t)std::min<uint64_t>((cells + 255) / 256, 4096);
        for (uint32_t s0 = 0; s0 < nsnap; s0 += kSnapGroup) {
            k_snap_count<<<g, 256, 0, stream>>>(d_F[nxt] + (uint64_t)v0 * stride, d_nz[nxt] + (uint64_t)v0 * ntw,
                                                stride, ntw, v1 - v0, hw, d_smask[slot], s0,
                                                (uint32_t)std::min<size_t>(kSnapGroup, nsnap - s0), d_scalars);
            HIP_TRY(hipGetLastError());
        }
    }
    ft_valid = fused_tick;  // FT[nxt] / d_snz[(t + 1) % 3] describe the next tick's F_cur
    if (pushw_any && wact) mark_tick = t;  // (d_mark[t & 1] holds this tick's marks)
    return GOSSIP_OK;
}

// ---- compressed row exchange (row partition) --------------------------------------------
// A rank's message for tick t and row chunk c: its rows [lo, hi) of F_next (the chunk, or all
// its rows), restricted to OCCUPIED 16-word tile rows (the nz bits; unoccupied rows hold stale
// words no reader loads), plus -- in its last chunk only -- its partial liveness.  Layout in
// uint64 words:
//   [0]                      number of rows R
//   [1, 1 + m)               nz words of rows lo..hi-1 (m = (hi - lo) * ntw)
//   [.., + ceil((k+1)/2))    uint32 row offsets: rows of node lo+i start at offset[i] (k = hi-lo)
//   [.., + 16 R)             the rows, node by node, tile by tile
//   [.., + wact)             liveness words of this rank's rows (last chunk / whole rows)
// The receiver knows k and whether liveness is present from (rank, chunk), so R follows from
// the message size: no header read-back.

// Rows of rank r's chunk c: 512-row blocks (the dense tile and the row-partition granule), the
// last chunks possibly empty; kWholeRows = all of rank r's rows.
void gossip_engine::chunk_rows(uint32_t r, uint32_t c, uint64_t* lo, uint64_t* hi) const {
    const uint64_t a = row_lo[r], b = row_lo[r + 1];
    if (c == kWholeRows || nchunks <= 1) {
        *lo = a;
        *hi = b;
        return;
    }
    const uint64_t per = ((b - a + nchunks - 1) / nchunks + 511) / 512 * 512;
    *lo = std::min<uint64_t>(b, a + (uint64_t)c * per);
    *hi = std::min<uint64_t>(b, *lo + per);
}

int gossip_engine::ensure_xstream() {
    if (xstream) return GOSSIP_OK;
    HIP_TRY(hipStreamCreateWithFlags(&xstream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&ev_xdone, hipEventDisableTiming));
    return GOSSIP_OK;
}

struct PackLayout {
    uint64_t nz, off, rows, live, total;
};
PackLayout pack_layout(uint64_t k, uint32_t ntw, uint64_t nrows, uint32_t wact) {
    PackLayout L;
    L.nz = 1;
    L.off = L.nz + k * ntw;
    L.rows = L.off + (k + 2) / 2;
    L.live = L.rows + 16 * nrows;
    L.total = L.live + wact;
    return L;
}

// per node: number of occupied tile rows; nz words copied into the message
__global__ __launch_bounds__(256) void k_pack_count(const unsigned long long* __restrict__ nz, uint64_t k, uint32_t ntw,
                                                    uint64_t* __restrict__ msg_nz, uint32_t* __restrict__ cnt) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i > k) return;
    if (i == k) {
        cnt[i] = 0u;  // the scan's last element = total
        return;
    }
    uint32_t c = 0;
    for (uint32_t w = 0; w < ntw; w++) {
        const unsigned long long x = nz[i * ntw + w];
        msg_nz[i * ntw + w] = x;
        c += (uint32_t)__popcll(x);
    }
    cnt[i] = c;
}

// one wave per node: its occupied tile rows, 4 rows per instruction (16 lanes x 8 B each).
// Only message rows [r0, r1) move (r1 capped by *total when total is given: the row count read on
// the device from a message header); `rows` points at message row r0.
template <bool PACK>
__global__ __launch_bounds__(256) void k_move_rows(uint64_t* __restrict__ F, uint32_t stride, uint64_t lo, uint64_t k,
                                                   const uint64_t* __restrict__ nz, uint32_t ntw,
                                                   const uint32_t* __restrict__ off, uint64_t* __restrict__ rows,
                                                   uint64_t r0 = 0, uint64_t r1 = ~0ull,
                                                   const uint64_t* __restrict__ total = nullptr) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + wave_in_block();
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    if (total) r1 = min(r1, *total);
    for (uint64_t i = wave; i < k; i += nwaves) {
        uint64_t o = off[i];
        if (o >= r1) break;  // (offsets grow with i)
        for (uint32_t w = 0; w < ntw; w++) {
            unsigned long long m = (unsigned long long)nz[i * ntw + w];
            while (m) {
                // the g-th of the next 4 set bits goes to lanes 16g .. 16g+15
                const uint32_t g = lane >> 4;
                unsigned long long mm = m;
                for (uint32_t r = 0; r < g && mm; r++) mm &= mm - 1ull;
                const uint32_t cntb = (uint32_t)min(4, __popcll(m));
                if (g < cntb && o + g >= r0 && o + g < r1) {
                    const uint32_t tile = w * 64u + (uint32_t)__builtin_ctzll(mm);
                    uint64_t* frow = F + (lo + i) * stride + (uint64_t)tile * 16u + (lane & 15u);
                    uint64_t* mrow = rows + (o + g - r0) * 16u + (lane & 15u);
                    if (PACK) *mrow = *frow;
                    else *frow = *mrow;
                }
                for (uint32_t r = 0; r < cntb; r++) m &= m - 1ull;
                o += cntb;
            }
        }
    }
}

__global__ void k_or_words(const uint64_t* __restrict__ src, uint32_t n, unsigned long long* __restrict__ dst) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w < n && src[w]) dst[w] |= src[w];
}

// message header = its row count, the exclusive scan's last element (the RCCL exchange reads it
// on the device: no host wait per chunk)
__global__ void k_msg_header(const uint32_t* __restrict__ off_end, uint64_t* __restrict__ hdr) { *hdr = *off_end; }

// RCCL message layout: a fixed prefix (header, occupancy words, row offsets, liveness) whose size
// every rank knows, then the rows; a broadcast carries the prefix and up to `cap` rows
struct DevLayout {
    uint64_t nz, off, live, rows;  // rows = prefix words
};
DevLayout dev_layout(uint64_t k, uint32_t ntw, uint32_t wlive) {
    DevLayout L;
    L.nz = 1;
    L.off = L.nz + k * ntw;
    L.live = L.off + (k + 2) / 2;
    L.rows = L.live + wlive;
    return L;
}

#define NCCL_TRY(x)                                                                         \
    do {                                                                                    \
        ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess) return set_error(GOSSIP_EHIP, std::string("RCCL: ") + ncclGetErrorString(r_)); \
    } while (0)
// A collective on the engine's communicator (member functions): never after gossip_engine_abort
// freed it (another thread's abort of a failing partition), whose later calls would use freed
// memory -- the engine then reports GOSSIP_ESTATE.  The issue is bracketed by comm_issuing, and
// gossip_engine_abort raises `aborted` first and then waits for comm_issuing == 0 before it frees
// the communicator (both sequentially consistent): a call that saw `aborted` clear finishes
// enqueueing before the abort, a later one sees it set -- unless the enqueue blocks on a failed
// peer for kAbortWaitS, when the abort goes ahead to unblock it.  A grouped exchange takes one
// bracket for its whole ncclGroupStart .. ncclGroupEnd (exchange_rccl).
// CommIssue is defined at the top of the file.
#define COMM_TRY(x)                                                                         \
    do {                                                                                    \
        CommIssue issuing_(comm_issuing);                                                   \
        if (aborted.load()) return set_error(GOSSIP_ESTATE, "RCCL: the row partition was aborted"); \
        NCCL_TRY(x);                                                                        \
    } while (0)

// The exchange's message / receive buffers (row partition) grow with the frontier; they count in
// device_bytes (the engine's footprint, gossip_counters) and fail cleanly with GOSSIP_ENOMEM --
// the callers' cue to split the shares into more shards -- when the device or the mem_limit
// option has no room left, instead of a HIP error mid-run.
// preserve > 0: the first `preserve` words of the old buffer are copied into the new one (the old
// buffer is then freed only after the copy, so the room check counts both).
int gossip_engine::ensure_dev(uint64_t*& p, uint64_t& cap, uint64_t words, uint64_t preserve) {
    if (words <= cap) return GOSSIP_OK;
    HIP_TRY(hipStreamSynchronize(stream));  // (rare: growth) both streams may still read p
    if (xstream) HIP_TRY(hipStreamSynchronize(xstream));
    const uint64_t ncap = std::max<uint64_t>(words, cap + cap / 2);
    size_t freeb = 0, totalb = 0;
    HIP_TRY(hipMemGetInfo(&freeb, &totalb));
    const uint64_t room = (uint64_t)freeb + (preserve ? 0 : cap * 8);  // (without a copy the old buffer is freed first)
    if (ncap * 8 > room || (opt_mem_limit > 0 && device_bytes + (ncap - cap) * 8 > (uint64_t)opt_mem_limit))
        return set_error(GOSSIP_ENOMEM, "row exchange: no device memory for a " + std::to_string(ncap * 8) +
                                            "-byte message buffer (" + std::to_string(device_bytes) + " bytes held)");
    uint64_t* q = nullptr;
    if (preserve) {
        HIP_TRY(hipMalloc(&q, ncap * 8));
        HIP_TRY(hipMemcpy(q, p, std::min(preserve, cap) * 8, hipMemcpyDeviceToDevice));
    }
    hipFree(p);
    p = nullptr;
    device_bytes -= cap * 8;
    cap = 0;
    if (!preserve) HIP_TRY(hipMalloc(&q, ncap * 8));
    p = q;
    cap = ncap;
    device_bytes += cap * 8;
    return GOSSIP_OK;
}

// Pack this rank's rows of chunk c of F_next (after the chunk's pull and births) into d_msg on
// stream s; msg_words = size.  (One host wait: the row count sizes the message.)
int gossip_engine::pack_rows(int64_t t, uint32_t c, hipStream_t s) {
    uint64_t lo, hi;
    chunk_rows(row_rank, c, &lo, &hi);
    const uint32_t wlive = (c == kWholeRows || c + 1 >= nchunks) ? hw : 0u;  // liveness: last chunk
    return pack_range(t, lo, hi, wlive, s);
}

// Pack rows [lo, hi) of F_next (+ `wlive` liveness words) into d_msg on stream s.
int gossip_engine::pack_range(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, hipStream_t s) {
    const int nxt = fcur ^ 1, lv = (int)(t % 3);
    const uint64_t k = hi - lo;
    int rc = ensure_dev(d_msg, msg_cap, pack_layout(k, ntw, 0, wlive).rows);
    if (rc) return rc;
    if (k + 1 > cnt_cap) {
        HIP_TRY(hipStreamSynchronize(s));
        hipFree(d_cnt);
        cnt_cap = k + 1;
        HIP_TRY(hipMalloc(&d_cnt, cnt_cap * 4));
    }
    const PackLayout L0 = pack_layout(k, ntw, 0, wlive);
    uint32_t* off = reinterpret_cast<uint32_t*>(d_msg + L0.off);
    k_pack_count<<<(uint32_t)((k + 1 + 255) / 256), 256, 0, s>>>(d_nz[nxt] + lo * ntw, k, ntw, d_msg + L0.nz, d_cnt);
    HIP_TRY(hipGetLastError());
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d_cnt, off, (int)(k + 1), s));
    if (tmp > scan_tmp_bytes) {
        HIP_TRY(hipStreamSynchronize(s));
        hipFree(d_scan_tmp);
        scan_tmp_bytes = tmp;
        HIP_TRY(hipMalloc(&d_scan_tmp, tmp));
    }
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(d_scan_tmp, tmp, d_cnt, off, (int)(k + 1), s));
    uint32_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, off + k, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const PackLayout L = pack_layout(k, ntw, total, wlive);
    // (the layout's header parts do not depend on the row count: grow keeping them; through
    // ensure_dev, so the growth counts in device_bytes and respects mem_limit)
    if (L.total > msg_cap) {
        if ((rc = ensure_dev(d_msg, msg_cap, L.total, L.rows))) return rc;
        off = reinterpret_cast<uint32_t*>(d_msg + L.off);
    }
    const unsigned long long hdr = total;
    HIP_TRY(hipMemcpyAsync(d_msg, &hdr, 8, hipMemcpyHostToDevice, s));
    if (total) {
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((k + 3) / 4, 4096));
        k_move_rows<true><<<g, 256, 0, s>>>(d_F[nxt], stride, lo, k, d_msg + L.nz, ntw, off, d_msg + L.rows);
        HIP_TRY(hipGetLastError());
    }
    if (wlive) HIP_TRY(hipMemcpyAsync(d_msg + L.live, d_live[lv], (size_t)wlive * 8, hipMemcpyDeviceToDevice, s));
    msg_words = L.total;
    exchange_bytes_out += L.total * 8;
    return GOSSIP_OK;
}

// Unpack rank r's message of chunk c (device buffer, `words` long) into this engine's F_next,
// nz_next and (last chunk) liveness, on stream s.  No host wait.
int gossip_engine::unpack_rows(int64_t t, uint32_t r, uint32_t c, const uint64_t* msg, uint64_t words, hipStream_t s) {
    uint64_t lo, hi;
    chunk_rows(r, c, &lo, &hi);
    const uint32_t wlive = (c == kWholeRows || c + 1 >= nchunks) ? hw : 0u;
    const PackLayout L0 = pack_layout(hi - lo, ntw, 0, wlive);
    if (words < L0.total || (words - L0.total) % 16u)
        return set_error(GOSSIP_EINVAL, "row exchange: message of rank " + std::to_string(r) +
                                            " has the wrong size (ranks diverged?)");
    return unpack_range(t, lo, hi, wlive, msg, words, s);
}

// Unpack a message of rows [lo, hi) (+ `wlive` liveness words) into F_next / nz_next / liveness.
int gossip_engine::unpack_range(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, const uint64_t* msg,
                                uint64_t words, hipStream_t s) {
    const int nxt = fcur ^ 1, lv = (int)(t % 3);
    const uint64_t k = hi - lo;
    const PackLayout L0 = pack_layout(k, ntw, 0, wlive);
    const uint64_t total = (words - L0.total) / 16u;
    const PackLayout L = pack_layout(k, ntw, total, wlive);
    if (k) HIP_TRY(hipMemcpyAsync(d_nz[nxt] + lo * ntw, msg + L.nz, (size_t)k * ntw * 8, hipMemcpyDeviceToDevice, s));
    if (total) {
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((k + 3) / 4, 4096));
        k_move_rows<false><<<g, 256, 0, s>>>(d_F[nxt], stride, lo, k, msg + L.nz, ntw,
                                             reinterpret_cast<const uint32_t*>(msg + L.off),
                                             const_cast<uint64_t*>(msg + L.rows));
        HIP_TRY(hipGetLastError());
    }
    if (wlive) {
        k_or_words<<<(wlive + 255) / 256, 256, 0, s>>>(msg + L.live, wlive, d_live[lv]);
        HIP_TRY(hipGetLastError());
    }
    exchange_bytes_in += words * 8;
    return GOSSIP_OK;
}

// Rehearsal of the row exchange (option rehearse_rows): every range's F_next rows are packed
// into its message and unpacked again into the same rows (the data are unchanged), so a range's
// pack time, its message size and its unpack time -- what every OTHER rank spends on it -- are
// measured with the real kernels.
int gossip_engine::rehearse_exchange(int64_t t) {
    const bool timing = (cfg.flags & GOSSIP_F_TIMING) != 0;
    const uint32_t R = (uint32_t)rr_lo.size() - 1;
    if (rr_bytes.size() != R) rr_bytes.assign(R, 0);
    if (rr_bytes_max.size() != R) rr_bytes_max.assign(R, 0);
    for (uint32_t r = 0; r < R; r++) {
        const uint64_t lo = rr_lo[r], hi = rr_lo[r + 1];
        if (hi <= lo) continue;
        hipEvent_t a = timing ? get_event() : nullptr, b = timing ? get_event() : nullptr;
        if (timing) HIP_TRY(hipEventRecord(a, stream));
        int rc = pack_range(t, lo, hi, hw, stream);
        if (rc) return rc;
        if (timing) {
            HIP_TRY(hipEventRecord(b, stream));
            rr_events.push_back({r, 1u, a, b});
        }
        rr_bytes[r] += msg_words * 8;
        rr_bytes_max[r] = std::max<uint64_t>(rr_bytes_max[r], msg_words * 8);
        hipEvent_t c = timing ? get_event() : nullptr, d = timing ? get_event() : nullptr;
        if (timing) HIP_TRY(hipEventRecord(c, stream));
        if ((rc = unpack_range(t, lo, hi, hw, d_msg, msg_words, stream))) return rc;
        if (timing) {
            HIP_TRY(hipEventRecord(d, stream));
            rr_events.push_back({r, 2u, c, d});
        }
    }
    rr_ticks++;
    return GOSSIP_OK;
}

void gossip_engine::rehearse_harvest() {
    const uint32_t R = rr_lo.empty() ? 0u : (uint32_t)rr_lo.size() - 1;
    for (auto& v : rr_ms)
        if (v.size() != R) v.assign(R, 0.0);
    for (const RehearseEv& x : rr_events) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, x.a, x.b) == hipSuccess && x.range < R) rr_ms[x.kind][x.range] += ms;
        event_pool.push_back(x.a);
        event_pool.push_back(x.b);
    }
    rr_events.clear();
}

// Pack rows [lo, hi) of F_next into d_msg in the device-sized layout (dev_layout; the header = the
// row count, written on the device): no host wait.  d_msg holds the worst case, every tile row.
int gossip_engine::pack_dev(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, hipStream_t s) {
    const int nxt = fcur ^ 1, lv = (int)(t % 3);
    const uint64_t k = hi - lo;
    const DevLayout L = dev_layout(k, ntw, wlive);
    int rc = ensure_dev(d_msg, msg_cap, L.rows + 16ull * k * (hw / kTileWords));
    if (rc) return rc;
    if (k + 1 > cnt_cap) {
        HIP_TRY(hipStreamSynchronize(s));
        hipFree(d_cnt);
        cnt_cap = k + 1;
        HIP_TRY(hipMalloc(&d_cnt, cnt_cap * 4));
    }
    uint32_t* off = reinterpret_cast<uint32_t*>(d_msg + L.off);
    k_pack_count<<<(uint32_t)((k + 1 + 255) / 256), 256, 0, s>>>(d_nz[nxt] + lo * ntw, k, ntw, d_msg + L.nz, d_cnt);
    HIP_TRY(hipGetLastError());
    size_t tmp = 0;
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d_cnt, off, (int)(k + 1), s));
    if (tmp > scan_tmp_bytes) {  // (first use of a chunk size only)
        HIP_TRY(hipStreamSynchronize(s));
        hipFree(d_scan_tmp);
        scan_tmp_bytes = tmp;
        HIP_TRY(hipMalloc(&d_scan_tmp, tmp));
    }
    HIP_TRY(hipcub::DeviceScan::ExclusiveSum(d_scan_tmp, tmp, d_cnt, off, (int)(k + 1), s));
    k_msg_header<<<1, 1, 0, s>>>(off + k, d_msg);
    const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((k + 3) / 4, 4096));
    k_move_rows<true><<<g, 256, 0, s>>>(d_F[nxt], stride, lo, k, d_msg + L.nz, ntw, off, d_msg + L.rows);
    HIP_TRY(hipGetLastError());
    if (wlive) HIP_TRY(hipMemcpyAsync(d_msg + L.live, d_live[lv], (size_t)wlive * 8, hipMemcpyDeviceToDevice, s));
    return GOSSIP_OK;
}

// Unpack message rows [r0, r1) of another rank's rows [lo, hi): `msg` is its prefix (header,
// occupancy, offsets, liveness), `rows` points at message row r0.  prefix: first round -- also
// the occupancy and liveness words, and r1 capped by the header's row count on the device.
int gossip_engine::unpack_dev(int64_t t, uint64_t lo, uint64_t hi, uint32_t wlive, const uint64_t* msg,
                              const uint64_t* rows, uint64_t r0, uint64_t r1, bool prefix, hipStream_t s) {
    const int nxt = fcur ^ 1, lv = (int)(t % 3);
    const uint64_t k = hi - lo;
    const DevLayout L = dev_layout(k, ntw, wlive);
    if (prefix && k)
        HIP_TRY(hipMemcpyAsync(d_nz[nxt] + lo * ntw, msg + L.nz, (size_t)k * ntw * 8, hipMemcpyDeviceToDevice, s));
    if (r1 > r0 && k) {
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((k + 3) / 4, 4096));
        k_move_rows<false><<<g, 256, 0, s>>>(d_F[nxt], stride, lo, k, msg + L.nz, ntw,
                                             reinterpret_cast<const uint32_t*>(msg + L.off),
                                             const_cast<uint64_t*>(rows), r0, r1, prefix ? msg : nullptr);
        HIP_TRY(hipGetLastError());
    }
    if (prefix && wlive) {
        k_or_words<<<(wlive + 255) / 256, 256, 0, s>>>(msg + L.live, wlive, d_live[lv]);
        HIP_TRY(hipGetLastError());
    }
    return GOSSIP_OK;
}

// Row partition over RCCL, pipelined, with device-side sizes.  Per row chunk c, once the engine
// stream has pulled it (ev_chunk[c]), the exchange stream packs the rank's rows (row count in the
// message header, on the device), all-gathers the ranks' row counts into d_tot (device), and
// broadcasts every rank's message prefix + its first xcap[r][c] rows -- a length every rank
// derives from earlier ticks' counts, so no host wait -- then unpacks the others' chunk c (rows
// capped by their header) while the engine stream pulls chunk c + 1.  After the last chunk: ONE
// host wait reads the tick's counts; rows beyond a capacity (the first ticks, a growing frontier)
// go in a second round (re-pack, broadcast the tail, unpack), and the capacities grow to 1.25x.
// The engine stream joins the exchange stream before the tick's liveness read-back (tick_step_b).
int gossip_engine::exchange_rccl(int64_t t) {
    if (aborted.load()) return set_error(GOSSIP_ESTATE, "RCCL: the row partition was aborted");
    int rc = ensure_xstream();
    if (rc) return rc;
    const uint32_t R = row_count;
    if (xcap.size() != (size_t)R * kMaxChunks) xcap.assign((size_t)R * kMaxChunks, 0ull);
    if (!d_tot) {
        HIP_TRY(hipMalloc(&d_tot, (size_t)R * kMaxChunks * 8));
        HIP_TRY(hipHostMalloc(&h_tot, (size_t)R * kMaxChunks * 8, hipHostMallocDefault));
    }
    if (!xchunks_checked) {  // once: every rank must issue the same collectives per tick
        if ((rc = ensure_dev(d_sizes, sizes_cap, 2 * R))) return rc;
        const unsigned long long mine = nchunks;
        HIP_TRY(hipMemcpyAsync(d_sizes + row_rank, &mine, 8, hipMemcpyHostToDevice, xstream));
        COMM_TRY(ncclAllGather(d_sizes + row_rank, d_sizes, 1, ncclUint64, comm, xstream));
        std::vector<unsigned long long> all(R);
        HIP_TRY(hipMemcpyAsync(all.data(), d_sizes, R * 8, hipMemcpyDeviceToHost, xstream));
        HIP_TRY(hipStreamSynchronize(xstream));
        for (uint32_t r = 0; r < R; r++)
            if (all[r] != nchunks) return set_error(GOSSIP_EINVAL, "row exchange: ranks use different xchunks options");
        xchunks_checked = true;
    }
    auto geom = [&](uint32_t r, uint32_t c, uint64_t* lo, uint64_t* hi, uint32_t* wl) {
        chunk_rows(r, c, lo, hi);
        *wl = (c + 1 >= nchunks) ? hw : 0u;  // liveness rides in the last chunk
    };
    // receive buffers for the whole tick: [c][r] prefix + capacity rows
    std::vector<uint64_t> at((size_t)nchunks * R, 0ull);
    uint64_t tot_words = 0;
    for (uint32_t c = 0; c < nchunks; c++)
        for (uint32_t r = 0; r < R; r++) {
            if (r == row_rank) continue;
            uint64_t lo, hi;
            uint32_t wl;
            geom(r, c, &lo, &hi, &wl);
            at[(size_t)c * R + r] = tot_words;
            tot_words += dev_layout(hi - lo, ntw, wl).rows + 16ull * xcap[(size_t)r * kMaxChunks + c];
        }
    if ((rc = ensure_dev(d_recv_msgs, recv_cap, std::max<uint64_t>(tot_words, 1)))) return rc;
    for (uint32_t c = 0; c < nchunks; c++) {
        uint64_t lo, hi;
        uint32_t wl;
        geom(row_rank, c, &lo, &hi, &wl);
        HIP_TRY(hipStreamWaitEvent(xstream, ev_chunk[c], 0));
        if ((rc = pack_dev(t, lo, hi, wl, xstream))) return rc;
        COMM_TRY(ncclAllGather(d_msg, d_tot + (size_t)c * R, 1, ncclUint64, comm, xstream));
        {
            // ONE issue bracket around the whole group: `aborted` is tested once,
            // before ncclGroupStart, and the group is always closed -- an early return between
            // ncclGroupStart and ncclGroupEnd would leave this thread's RCCL group open, holding
            // broadcasts on a communicator the abort then frees
            CommIssue issuing_(comm_issuing);
            if (aborted.load()) return set_error(GOSSIP_ESTATE, "RCCL: the row partition was aborted");
            ncclResult_t gr = ncclGroupStart();
            for (uint32_t r = 0; r < R && gr == ncclSuccess; r++) {
                uint64_t rlo, rhi;
                uint32_t rwl;
                geom(r, c, &rlo, &rhi, &rwl);
                const uint64_t words = dev_layout(rhi - rlo, ntw, rwl).rows + 16ull * xcap[(size_t)r * kMaxChunks + c];
                uint64_t* buf = r == row_rank ? d_msg : d_recv_msgs + at[(size_t)c * R + r];
                gr = ncclBroadcast(buf, buf, words, ncclUint64, (int)r, comm, xstream);
                if (r == row_rank) exchange_bytes_out += words * 8;
                else exchange_bytes_in += words * 8;
            }
            const ncclResult_t ge = ncclGroupEnd();
            if (gr != ncclSuccess || ge != ncclSuccess)
                return set_error(GOSSIP_EHIP, std::string("RCCL: ") + ncclGetErrorString(gr != ncclSuccess ? gr : ge));
        }
        for (uint32_t r = 0; r < R; r++) {
            if (r == row_rank) continue;
            uint64_t rlo, rhi;
            uint32_t rwl;
            geom(r, c, &rlo, &rhi, &rwl);
            const uint64_t* msg = d_recv_msgs + at[(size_t)c * R + r];
            if ((rc = unpack_dev(t, rlo, rhi, rwl, msg, msg + dev_layout(rhi - rlo, ntw, rwl).rows, 0,
                                 xcap[(size_t)r * kMaxChunks + c], true, xstream)))
                return rc;
        }
    }
    // the tick's one host wait: every rank's row counts
    HIP_TRY(hipMemcpyAsync(h_tot, d_tot, (size_t)nchunks * R * 8, hipMemcpyDeviceToHost, xstream));
    HIP_TRY(hipStreamSynchronize(xstream));
    for (uint32_t c = 0; c < nchunks; c++) {
        for (uint32_t r = 0; r < R; r++) {
            uint64_t& cap = xcap[(size_t)r * kMaxChunks + c];
            const uint64_t tot = h_tot[(size_t)c * R + r];
            if (tot <= cap) continue;
            // second round (identical decision on every rank): rows [cap, tot) of rank r, chunk c
            uint64_t rlo, rhi;
            uint32_t rwl;
            geom(r, c, &rlo, &rhi, &rwl);
            const DevLayout L = dev_layout(rhi - rlo, ntw, rwl);
            const uint64_t words = 16ull * (tot - cap);
            if (r == row_rank) {
                if ((rc = pack_dev(t, rlo, rhi, rwl, xstream))) return rc;  // (d_msg held a later chunk)
                COMM_TRY(ncclBroadcast(d_msg + L.rows + 16ull * cap, d_msg + L.rows + 16ull * cap, words, ncclUint64,
                                       (int)r, comm, xstream));
                exchange_bytes_out += words * 8;
            } else {
                if ((rc = ensure_dev(d_ovf, ovf_cap, words))) return rc;
                COMM_TRY(ncclBroadcast(d_ovf, d_ovf, words, ncclUint64, (int)r, comm, xstream));
                exchange_bytes_in += words * 8;
                if ((rc = unpack_dev(t, rlo, rhi, rwl, d_recv_msgs + at[(size_t)c * R + r], d_ovf, cap, tot, false,
                                     xstream)))
                    return rc;
                HIP_TRY(hipStreamSynchronize(xstream));  // (d_ovf is reused by the next overflow)
            }
            x_overflow_rounds++;
        }
        for (uint32_t r = 0; r < R; r++) {  // capacities: 1.25x the largest count seen (rows),
            uint64_t& cap = xcap[(size_t)r * kMaxChunks + c];  // at most every tile row of the chunk
            const uint64_t tot = h_tot[(size_t)c * R + r];
            uint64_t rlo, rhi;
            uint32_t rwl;
            geom(r, c, &rlo, &rhi, &rwl);
            if (tot > cap) cap = std::min<uint64_t>(tot + tot / 4 + 16, (rhi - rlo) * (hw / kTileWords));
        }
    }
    return GOSSIP_OK;
}

// Fused row partition: one rank's FT slice message (dense_kernel.h k_ft_pack), u32 words
uint64_t gossip_engine::ft_words(uint32_t wact) const {
    return (uint64_t)wact * 64u * ft_smax() + 2ull * (wact / 4u) * snz_nstw + 2ull * wact;
}

// The fused tick's exchange over RCCL: every rank packs its FT_next slice, stage masks and partial
// liveness, one all-gather (the north star's frontier all-gather: W shares x n bits in total, 32 MiB
// per hop at C5), and each rank unpacks the others' into its FT_next, stage masks and liveness --
// on the engine stream, after the tick's births, before the liveness read-back.  F_next rows and
// occupancy words stay per rank (nothing reads another rank's: the next fused tick reads FT).
int gossip_engine::ft_pack(int64_t t) {
    const uint32_t wact = hw;
    const uint64_t words = ft_words(wact);
    uint64_t* m = reinterpret_cast<uint64_t*>(d_ftmsg);
    int rc = ensure_dev(m, ftmsg_cap, (words + 1) / 2);
    d_ftmsg = reinterpret_cast<uint32_t*>(m);
    if (rc) return rc;
    const uint32_t g = (uint32_t)std::min<uint64_t>((words + 255) / 256, 8192);
    k_ft_pack<<<g, 256, 0, stream>>>(d_FT[fcur ^ 1], n_pad / 32u, row_lo[row_rank] / 32u, ft_smax(),
                                     (uint32_t)((row_lo[row_rank + 1] - row_lo[row_rank] + 31) / 32), wact * 64u,
                                     d_snz[(t + 1) % 3], (wact / 4u) * snz_nstw, d_live[t % 3], wact, d_ftmsg);
    HIP_TRY(hipGetLastError());
    exchange_bytes_out += words * 4;
    return GOSSIP_OK;
}
int gossip_engine::ft_unpack(int64_t t, uint32_t r, const uint32_t* msg) {
    const uint32_t wact = hw;
    const uint64_t words = ft_words(wact);
    const uint32_t g = (uint32_t)std::min<uint64_t>((words + 255) / 256, 8192);
    k_ft_unpack<<<g, 256, 0, stream>>>(d_FT[fcur ^ 1], n_pad / 32u, row_lo[r] / 32u, ft_smax(),
                                       (uint32_t)((row_lo[r + 1] - row_lo[r] + 31) / 32), wact * 64u, msg,
                                       d_snz[(t + 1) % 3], (wact / 4u) * snz_nstw, d_live[t % 3], wact);
    HIP_TRY(hipGetLastError());
    exchange_bytes_in += words * 4;
    return GOSSIP_OK;
}
uint32_t gossip_engine::ft_smax() const {
    uint64_t smax = 0;
    for (uint32_t r = 0; r < row_count; r++) smax = std::max<uint64_t>(smax, (row_lo[r + 1] - row_lo[r] + 31) / 32);
    return (uint32_t)smax;
}
int gossip_engine::exchange_ft(int64_t t) {
    const uint32_t R = row_count;
    if (!hw) return GOSSIP_OK;
    const uint64_t words = ft_words(hw);
    uint64_t* rv = reinterpret_cast<uint64_t*>(d_ftrecv);
    int rc = ensure_dev(rv, ftrecv_cap, (words * R + 1) / 2);
    d_ftrecv = reinterpret_cast<uint32_t*>(rv);
    if (rc) return rc;
    if ((rc = ft_pack(t))) return rc;
    COMM_TRY(ncclAllGather(d_ftmsg, d_ftrecv, words, ncclUint32, comm, stream));
    for (uint32_t r = 0; r < R; r++)
        if (r != row_rank && (rc = ft_unpack(t, r, d_ftrecv + words * r))) return rc;
    return GOSSIP_OK;
}

int gossip_engine::tick_step_b(int64_t t) {
    const int lv = (int)(t % 3);
    const uint32_t wact = hw;
    const int nxt = fcur ^ 1;
    if (comm && fused_rows) {
        int rc = exchange_ft(t);
        if (rc) return rc;
    } else if (comm) {
        int rc = exchange_rccl(t);
        if (rc) return rc;
    } else if (opt_rehearse_rows > 1 && !young && hw) {
        int rc = rehearse_exchange(t);
        if (rc) return rc;
    }
    if (xstream) {  // the unpacked rows and liveness precede the read-back and the next pull
        HIP_TRY(hipEventRecord(ev_xdone, xstream));
        HIP_TRY(hipStreamWaitEvent(stream, ev_xdone, 0));
    }
    // 6. liveness read-back (consumed kLag ticks later)
    {
        const int ls = (int)(t % kRing);
        // Words at or beyond wact were allocated after this tick, so their last_inject is
        // later than t and retire_from() never reads their (uncopied) entries.
        if (wact) HIP_TRY(hipMemcpyAsync(h_live[ls], d_live[lv], (size_t)wact * 8, hipMemcpyDeviceToHost, stream));
        HIP_TRY(hipEventRecord(live_done[ls], stream));
        live_pending[ls] = true;
        live_tick[ls] = t;
    }
    // 7. snapshot bases: totals over ticks < snap.tick (the partial of snap.tick, if any,
    //    is accumulated by that tick's pull/births through ctl.snap)
    for (size_t s = 0; s < snaps.size() && !batch; s++) {
        if (snaps[s].tick == t + 1) {
            k_sum_u32<<<256, 256, 0, stream>>>(d_recv, d_effgen, n, d_scalars + 2 + 2 * s);
            HIP_TRY(hipGetLastError());
        }
    }
    fcur = nxt;
    ticks++;
    if (trace) {
        int rc = decode_trace(t);
        if (rc) return rc;
    }
    return GOSSIP_OK;
}

int gossip_engine::decode_trace(int64_t t) {
    HIP_TRY(hipStreamSynchronize(stream));
    if (hw == 0) return GOSSIP_OK;
    std::vector<uint64_t> F((size_t)n * stride);
    HIP_TRY(hipMemcpy(F.data(), d_F[fcur], F.size() * 8, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> nz;
    if (d_nz[fcur]) {
        nz.resize((size_t)n * ntw);
        HIP_TRY(hipMemcpy(nz.data(), d_nz[fcur], nz.size() * 8, hipMemcpyDeviceToHost));
    }
    // young tiles: F_{t+1} of the write-sparse tiles lives in the slots (unless overflowed)
    std::vector<uint8_t> ws_tile(stride / kTileWords, 0);
    if (young && !wt_last.empty()) {
        for (uint32_t tl : wt_last) ws_tile[tl] = 1;
        std::vector<uint16_t> S((size_t)n * kSlotU16);
        HIP_TRY(hipMemcpy(S.data(), d_slot[fcur], S.size() * 2, hipMemcpyDeviceToHost));
        for (uint32_t v = v0; v < v1; v++) {
            const uint16_t* sv = S.data() + (size_t)v * kSlotU16;
            if (sv[0] == kSlotOverflow) continue;  // dense rows valid
            for (uint32_t tl : wt_last)
                for (uint32_t q = 0; q < kTileWords; q++) F[(size_t)v * stride + tl * kTileWords + q] = 0ull;
            for (uint32_t k = 1; k <= sv[0]; k++) {
                const uint32_t e = sv[k];
                if (e == kSlotTomb || (e >> 10) >= wt_last.size()) continue;
                F[(size_t)v * stride + wt_last[e >> 10] * kTileWords + ((e >> 6) & 15u)] |= 1ull << (e & 63u);
            }
        }
    }
    for (uint32_t v = v0; v < v1; v++)
        for (uint32_t w = 0; w < hw; w++) {
            const uint32_t tl = w >> 4;
            if (!nz.empty() && !ws_tile[tl] && !((nz[(size_t)v * ntw + (tl >> 6)] >> (tl & 63u)) & 1ull)) continue;  // stale row
            uint64_t x = F[(size_t)v * stride + w];
            while (x) {
                const int b = __builtin_ctzll(x);
                x &= x - 1;
                const uint32_t src = col_src[(size_t)w * 64 + b];
                if (src == UINT32_MAX) continue;
                const gossip_gen_event& e = ev[src];
                const int64_t bt = e.ns / L;
                const bool birth = (e.node == v && bt == t);
                const int64_t dl = link_timing ? ev_delta[src] : 0;
                const int64_t real_t = batch ? (ev_orig_ns[src] + (t - bt) * (L + dl)) / L : t;
                tr.push_back(Tr{v, e.share_id, real_t, (uint32_t)(t - bt), (uint8_t)(birth ? 0 : 1)});
            }
        }
    return GOSSIP_OK;
}

extern "C" {

int gossip_engine_create(const gossip_config* cfg, gossip_engine** out) {
    if (!cfg || !out) return set_error(GOSSIP_EINVAL, "NULL argument");
    *out = nullptr;
    if (cfg->latency_ns <= 0 || cfg->latency_ns >= 2000000000ll)
        return set_error(GOSSIP_EINVAL,
                         "latency must be in (0, 2 s): generation intervals are U(2,5) s "
                         "(p2pnode.cc:99) and the engine allows one generation per node per tick");
    if (cfg->t_cut_ns <= 0) return set_error(GOSSIP_EINVAL, "t_cut must be positive");
    if (cfg->shard_count > 1 && cfg->shard_rank >= cfg->shard_count)
        return set_error(GOSSIP_EINVAL, "shard_rank >= shard_count");
    if (cfg->mode != GOSSIP_MODE_AUTO && cfg->mode != GOSSIP_MODE_CSR && cfg->mode != GOSSIP_MODE_DENSE)
        return set_error(GOSSIP_EINVAL, "unsupported mode");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_error(GOSSIP_EHIP, "no HIP device: the engine has no CPU fallback");
    if (cfg->device < 0 || cfg->device >= ndev) return set_error(GOSSIP_EINVAL, "bad device ordinal");
    try {
        auto e = std::make_unique<gossip_engine>();
        e->cfg = *cfg;
        e->device = cfg->device;
        HIP_TRY(hipSetDevice(e->device));
        HIP_TRY(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
        HIP_TRY(hipDeviceGetAttribute(&e->num_cus, hipDeviceAttributeMultiprocessorCount, e->device));
        if (cfg->flags & GOSSIP_F_TIMING)  // timed phases: no event creation inside a tick's launches
            for (int k = 0; k < 256; k++) {
                hipEvent_t ev = nullptr;
                HIP_TRY(hipEventCreate(&ev));
                e->event_pool.push_back(ev);
            }
        e->L = cfg->latency_ns;
        e->t0 = cfg->t_start_ns;
        e->tick0 = cfg->t_start_ns / e->L;
        e->cut_tick = cfg->t_cut_ns / e->L;
        e->cut_r = cfg->t_cut_ns % e->L;
        e->tick_end = e->cut_r ? e->cut_tick + 1 : e->cut_tick;
        if (e->tick_end < e->tick0) e->tick_end = e->tick0;
        e->cur = e->tick0;
        e->opt_pull_nt = env_option("GOSSIP_PULL_NT", -1);
        e->opt_pull_grid = env_option("GOSSIP_PULL_GRID", 0);
        e->opt_dense_min_tiles = env_option("GOSSIP_DENSE_MIN_TILES", 512);
        e->opt_dense_fused = env_option("GOSSIP_DENSE_FUSED", 1);
        e->dense_rounds = env_option("GOSSIP_DENSE_ROUNDS", -1);
        e->dense_gm = std::max<int64_t>(1, env_option("GOSSIP_DENSE_GM", 4));
        e->opt_young = env_option("GOSSIP_YOUNG", -1);
        e->opt_young_age = env_option("GOSSIP_YOUNG_AGE", 5);
        e->opt_young_cap = env_option("GOSSIP_YOUNG_CAP", 127);
        e->opt_young_overlap = env_option("GOSSIP_YOUNG_OVERLAP", 1);
        e->opt_young_grid = env_option("GOSSIP_YOUNG_GRID", 0);
        e->opt_pull_gate = env_option("GOSSIP_PULL_GATE", 1);
        e->opt_pull_tiles = env_option("GOSSIP_PULL_TILES", 1);
        e->opt_pull_tile_order = env_option("GOSSIP_PULL_TILE_ORDER", 1);
        e->opt_young_nt = env_option("GOSSIP_YOUNG_NT", 1);
        e->opt_young_skip = env_option("GOSSIP_YOUNG_SKIP", -1);
        e->opt_pull_push = env_option("GOSSIP_PULL_PUSH", -1);
        e->opt_young_idle = env_option("GOSSIP_YOUNG_IDLE", 1);
        e->opt_mem_limit = env_option("GOSSIP_MEM_LIMIT", 0);
        e->opt_xchunks = env_option("GOSSIP_XCHUNKS", 4);
        e->opt_late_age = env_option("GOSSIP_LATE_AGE", -1);
        e->opt_pull_sat = env_option("GOSSIP_PULL_SAT", 1);
        e->opt_dense_rows = env_option("GOSSIP_DENSE_ROWS", -1);
        e->trace = (cfg->flags & GOSSIP_F_TRACE) != 0;
        e->dense = cfg->mode == GOSSIP_MODE_DENSE;
        e->handshake = (cfg->flags & GOSSIP_F_HANDSHAKE) != 0;
        e->batch = (cfg->flags & GOSSIP_F_HOP_BATCH) != 0;
        if (e->batch && e->handshake)
            return set_error(GOSSIP_EINVAL, "GOSSIP_F_HOP_BATCH and GOSSIP_F_HANDSHAKE are exclusive");
        if (e->handshake) {
            if (e->dense) return set_error(GOSSIP_EINVAL, "GOSSIP_F_HANDSHAKE: CSR mode only");
            if (e->t0 < 0 || e->t0 % e->L != 0)
                return set_error(GOSSIP_EINVAL, "GOSSIP_F_HANDSHAKE: t_start must be a multiple of the latency");
            if (cfg->t_cut_ns < e->t0 + 3 * e->L)
                return set_error(GOSSIP_EINVAL, "GOSSIP_F_HANDSHAKE: t_cut must be >= t_start + 3 latency");
        }
        *out = e.release();
        return GOSSIP_OK;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
}

int gossip_engine_set_graph(gossip_engine* e, uint32_t num_nodes, const int64_t* row_ptr,
                            const int32_t* col, const uint8_t* mult) {
    if (!e || !row_ptr || (!col && row_ptr[num_nodes] > 0)) return set_error(GOSSIP_EINVAL, "NULL argument");
    if (e->have_graph) return set_error(GOSSIP_ESTATE, "graph already set");
    if (num_nodes != e->cfg.num_nodes) return set_error(GOSSIP_EINVAL, "num_nodes mismatch with config");
    HIP_TRY(hipSetDevice(e->device));
    try {
        e->n = num_nodes;
        // row partition: rank r owns [row_lo[r], row_lo[r+1]), blocks of 512 rows (dense tiles
        // and 64-node pull waves both divide it)
        e->row_lo.assign(e->row_count + 1, num_nodes);
        const uint64_t rpr = ((uint64_t)(num_nodes + e->row_count - 1) / e->row_count + 511) / 512 * 512;
        for (uint32_t r = 0; r < e->row_count; r++) e->row_lo[r] = (uint32_t)std::min<uint64_t>(num_nodes, r * rpr);
        if (e->row_count > 1 && e->row_lo[e->row_count - 1] >= num_nodes)
            return set_error(GOSSIP_EINVAL, "row partition: fewer than one 512-row block per rank");
        e->v0 = e->row_lo[e->row_rank];
        e->v1 = e->row_lo[e->row_rank + 1];
        e->nnz = (uint64_t)row_ptr[num_nodes];
        if (e->nnz >= (1ull << 31)) return set_error(GOSSIP_EINVAL, "more than 2^31 adjacency entries");
        e->h_rowptr.assign(row_ptr, row_ptr + num_nodes + 1);
        e->h_col.assign(col, col + e->nnz);
        e->h_peers.assign(num_nodes, 0);
        e->h_sockets.assign(num_nodes, 0);
        for (uint32_t v = 0; v < num_nodes; v++) {
            if (row_ptr[v + 1] < row_ptr[v]) return set_error(GOSSIP_EINVAL, "row_ptr not monotone");
            uint32_t p = 0;
            for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; j++) {
                if (col[j] < 0 || (uint32_t)col[j] >= num_nodes) return set_error(GOSSIP_EINVAL, "col out of range");
                p += mult ? mult[j] : 1u;
            }
            e->h_peers[v] = p;
            e->h_sockets[v] = (uint32_t)(row_ptr[v + 1] - row_ptr[v]);
        }
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    HIP_TRY(hipMalloc(&e->d_rowptr, ((size_t)e->n + 1) * 8));
    HIP_TRY(hipMalloc(&e->d_col, std::max<size_t>(e->nnz, 1) * 4));
    HIP_TRY(hipMalloc(&e->d_deg, (size_t)std::max<uint32_t>(e->n, 1) * 4));
    HIP_TRY(hipMemcpy(e->d_rowptr, row_ptr, ((size_t)e->n + 1) * 8, hipMemcpyHostToDevice));
    if (e->nnz) HIP_TRY(hipMemcpy(e->d_col, col, e->nnz * 4, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(e->d_deg, e->h_peers.data(), (size_t)e->n * 4, hipMemcpyHostToDevice));
    if (e->cfg.mode == GOSSIP_MODE_AUTO) e->dense = auto_dense(e->n, e->nnz, e->handshake);
    if (e->dense) {
        // A[v][u] = [u in peers(v)] as bits (multiplicity only scales a count the pull does not
        // need), rows/cols padded to kDensePad with zeros.  Inc stays exact in int32 below 2^19
        // columns (dense_kernel.h), far above any adjacency that fits in HBM as bits.
        e->n_pad = (e->n + kDensePad - 1u) / kDensePad * kDensePad;
        const uint64_t kw = e->n_pad / 32u;
        const uint64_t bytes = (uint64_t)e->n_pad * kw * 4u;
        size_t freeb = 0, totalb = 0;
        HIP_TRY(hipMemGetInfo(&freeb, &totalb));
        if (bytes * 2 > (uint64_t)freeb)
            return set_error(GOSSIP_ENOMEM, "DENSE mode: the " + std::to_string(bytes) +
                                                "-byte adjacency does not fit; use GOSSIP_MODE_CSR");
        HIP_TRY(hipMalloc(&e->d_Ab, bytes));
        const uint64_t rows_per = std::max<uint64_t>(1, (256ull << 20) / (kw * 4u));
        std::vector<uint32_t> buf;
        try {
            buf.resize(rows_per * kw);
        } catch (const std::bad_alloc&) {
            return set_error(GOSSIP_ENOMEM, "host allocation failed");
        }
        for (uint64_t r0 = 0; r0 < e->n_pad; r0 += rows_per) {
            const uint64_t r1 = std::min<uint64_t>(e->n_pad, r0 + rows_per);
            std::fill(buf.begin(), buf.begin() + (r1 - r0) * kw, 0u);
            const uint64_t rn = std::min<uint64_t>(r1, e->n) > r0 ? std::min<uint64_t>(r1, e->n) - r0 : 0;
            const int th = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
            gossip::parallel_for(rn, th, [&](uint64_t lo, uint64_t hi) {
                for (uint64_t i = lo; i < hi; i++) {
                    const uint64_t v = r0 + i;
                    uint32_t* row = buf.data() + i * kw;
                    for (int64_t j = row_ptr[v]; j < row_ptr[v + 1]; j++)
                        row[(uint32_t)col[j] >> 5] |= 1u << ((uint32_t)col[j] & 31u);
                }
            });
            HIP_TRY(hipMemcpy(e->d_Ab + r0 * kw, buf.data(), (r1 - r0) * kw * 4u, hipMemcpyHostToDevice));
        }
    }
    e->have_graph = true;
    return GOSSIP_OK;
}

int gossip_engine_set_topology(gossip_engine* e, const gossip_topology* t) {
    if (!t) return set_error(GOSSIP_EINVAL, "NULL topology");
    int rc = gossip_engine_set_graph(e, t->n, t->row_ptr.data(), t->col.data(), t->mult.data());
    if (rc) return rc;
    try {
        gossip::cached_topology_components(t, &e->comp);  // same graph: reuse the labels if built
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    if (!e->handshake) return rc;
    // Handshake window: key (a,b) puts b in peers(a) at makeconnections (p2pnetwork.cc:144-145)
    // and a in peers(b) only when REGISTER arrives (p2pnode.cc:185-186).  Until then v sends
    // to its |keys (v,*)| connector-side peers, and the shares that get through (sent in
    // [t_start + 2L, t_start + 3L)) travel a -> b only: a CSR of those edges, rows b.
    try {
        const uint32_t n = t->n;
        std::vector<int64_t> rp((size_t)n + 1, 0);
        e->h_degc.assign(n, 0);
        for (size_t k = 0; k < t->la.size(); k++) {
            e->h_degc[t->la[k]]++;
            rp[(size_t)t->lb[k] + 1]++;
        }
        for (uint32_t v = 0; v < n; v++) rp[v + 1] += rp[v];
        std::vector<int32_t> col((size_t)rp[n]);
        std::vector<int64_t> pos(rp.begin(), rp.end() - 1);
        for (size_t k = 0; k < t->la.size(); k++) col[(size_t)pos[t->lb[k]]++] = (int32_t)t->la[k];
        HIP_TRY(hipMalloc(&e->d_rowptr_c, ((size_t)n + 1) * 8));
        HIP_TRY(hipMalloc(&e->d_col_c, std::max<size_t>(col.size(), 1) * 4));
        HIP_TRY(hipMalloc(&e->d_degc, (size_t)std::max<uint32_t>(n, 1) * 4));
        HIP_TRY(hipMemcpy(e->d_rowptr_c, rp.data(), rp.size() * 8, hipMemcpyHostToDevice));
        if (!col.empty()) HIP_TRY(hipMemcpy(e->d_col_c, col.data(), col.size() * 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(e->d_degc, e->h_degc.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    return GOSSIP_OK;
}

int gossip_engine_add_snapshot(gossip_engine* e, int64_t t_ns) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (e->have_sched) return set_error(GOSSIP_ESTATE, "add snapshots before the schedule");
    gossip_engine::Snap s{t_ns, t_ns / e->L, t_ns % e->L, 0, 0};
    for (const auto& o : e->snaps)
        if (o.tick == s.tick) return set_error(GOSSIP_EINVAL, "two snapshots in one tick");
    e->snaps.push_back(s);
    return GOSSIP_OK;
}

int gossip_engine_set_row_partition(gossip_engine* e, uint32_t rank, uint32_t count) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (e->have_graph) return set_error(GOSSIP_ESTATE, "set the row partition before the graph");
    if (count == 0 || rank >= count) return set_error(GOSSIP_EINVAL, "row partition: rank >= count");
    if (e->handshake) return set_error(GOSSIP_EINVAL, "row partition: not with GOSSIP_F_HANDSHAKE");
    if (count > 1 && e->opt_rehearse_rows > 1)  // (either order of the two calls is refused)
        return set_error(GOSSIP_EINVAL, "row partition: not on a rehearse_rows engine");
    e->row_rank = rank;
    e->row_count = count;
    return GOSSIP_OK;
}

int gossip_rccl_unique_id(uint8_t* out, uint32_t len) {
    if (!out || len < sizeof(ncclUniqueId)) return set_error(GOSSIP_EINVAL, "unique id buffer too small");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return GOSSIP_OK;
}

int gossip_engine_abort(gossip_engine* e) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    bool expected = false;
    // the flag first: the engine's own thread checks it before every collective (COMM_TRY); then
    // wait until no collective is being enqueued on the communicator, and free it.  The wait has a
    // deadline: an issue can block inside RCCL on a peer that already failed (lazy
    // connection setup on the first collective), and unblocking exactly that is ncclCommAbort's job
    if (e->aborted.compare_exchange_strong(expected, true) && e->comm) {
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(kAbortWaitS);
        while (e->comm_issuing.load() != 0 && std::chrono::steady_clock::now() < deadline)
            std::this_thread::yield();
        ncclCommAbort(e->comm);
    }
    return GOSSIP_OK;
}

int gossip_engine_connect_rccl(gossip_engine* e, const uint8_t* id, uint32_t len) {
    if (!e || !id || len < sizeof(ncclUniqueId)) return set_error(GOSSIP_EINVAL, "bad argument");
    if (e->comm) return set_error(GOSSIP_ESTATE, "already connected");
    HIP_TRY(hipSetDevice(e->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    NCCL_TRY(ncclCommInitRank(&e->comm, (int)e->row_count, uid, (int)e->row_rank));
    return GOSSIP_OK;
}

// One device, one thread: the engines of one row partition step in
// lockstep and exchange rows with device copies -- the rehearsal backend of the RCCL exchange.
int gossip_engine_group_run(gossip_engine** es, uint32_t count, int64_t tick_end) {
    if (!es || count == 0) return set_error(GOSSIP_EINVAL, "NULL argument");
    for (uint32_t r = 0; r < count; r++) {
        gossip_engine* e = es[r];
        if (!e || !e->have_sched) return set_error(GOSSIP_ESTATE, "set graph and schedule first");
        if (e->aborted.load()) return set_error(GOSSIP_ESTATE, "engine aborted (gossip_engine_abort)");
        if (e->row_count != count || e->row_rank != r) return set_error(GOSSIP_EINVAL, "engines must be ranks 0..count-1 of one partition");
        if (e->comm) return set_error(GOSSIP_EINVAL, "group run is the non-RCCL backend");
        // the unpack kernels read the other ranks' messages in place: one device only
        if (e->device != es[0]->device)
            return set_error(GOSSIP_EINVAL, "group run: every engine must be on the same device (no peer access)");
    }
    gossip_engine* e0 = es[0];
    for (uint32_t r = 0; r < count; r++) es[r]->group_mode = true;
    if (tick_end > e0->tick_end) tick_end = e0->tick_end;
    try {
        while (e0->cur < tick_end) {
            if (e0->batch && e0->cur > e0->last_birth_tick &&
                std::find(e0->tile_alloc.begin(), e0->tile_alloc.end(), (uint8_t)1) == e0->tile_alloc.end()) {
                for (uint32_t r = 0; r < count; r++) es[r]->done = true;
                break;
            }
            const int64_t t = e0->cur;
            // ranks run one after another (each stands for its own GPU: its kernel times are
            // then its own, not shared with the other ranks' concurrent kernels)
            for (uint32_t r = 0; r < count; r++) {
                HIP_TRY(hipSetDevice(es[r]->device));
                int rc = es[r]->tick_step_a(t);
                if (rc) return rc;
                HIP_TRY(hipStreamSynchronize(es[r]->stream));
            }
            for (uint32_t r = 1; r < count; r++)
                if (es[r]->hw != e0->hw || es[r]->stride != e0->stride || es[r]->fcur != e0->fcur)
                    return set_error(GOSSIP_EINVAL, "row partition engines diverged (different inputs?)");
            // the RCCL backend's exchange, chunk by chunk, with device-to-device copies in place of
            // the collectives (the ranks already ran one after another, so nothing overlaps here):
            // the same device-sized messages, capacities and second rounds as exchange_rccl
            for (uint32_t r = 1; r < count; r++)
                if (es[r]->nchunks != e0->nchunks || es[r]->fused_rows != e0->fused_rows)
                    return set_error(GOSSIP_EINVAL, "ranks use different xchunks / dense_fused options");
            // the fused tick's FT slice exchange (exchange_ft): every rank packs, then every rank
            // unpacks the others' messages in place (one device)
            if (e0->fused_rows && e0->hw) {
                for (uint32_t r = 0; r < count; r++) {
                    int rc = es[r]->ft_pack(t);
                    if (rc) return rc;
                    HIP_TRY(hipStreamSynchronize(es[r]->stream));
                }
                for (uint32_t d = 0; d < count; d++) {
                    for (uint32_t r = 0; r < count; r++) {
                        if (r == d) continue;
                        int rc = es[d]->ft_unpack(t, r, es[r]->d_ftmsg);
                        if (rc) return rc;
                    }
                    HIP_TRY(hipStreamSynchronize(es[d]->stream));
                }
            }
            for (uint32_t c = 0; c < e0->nchunks && !e0->fused_rows; c++) {
                auto geom = [&](uint32_t r, uint64_t* lo, uint64_t* hi, uint32_t* wl) {
                    e0->chunk_rows(r, c, lo, hi);
                    *wl = (c + 1 >= e0->nchunks) ? e0->hw : 0u;
                };
                for (uint32_t r = 0; r < count; r++) {
                    gossip_engine* e = es[r];
                    if (e->xcap.size() != (size_t)count * gossip_engine::kMaxChunks)
                        e->xcap.assign((size_t)count * gossip_engine::kMaxChunks, 0ull);
                    uint64_t lo, hi;
                    uint32_t wl;
                    geom(r, &lo, &hi, &wl);
                    int rc = e->pack_dev(t, lo, hi, wl, e->stream);
                    if (rc) return rc;
                    HIP_TRY(hipStreamSynchronize(e->stream));
                }
                std::vector<unsigned long long> tot(count);
                for (uint32_t r = 0; r < count; r++)  // (the all-gather of the row counts)
                    HIP_TRY(hipMemcpy(&tot[r], es[r]->d_msg, 8, hipMemcpyDeviceToHost));
                for (uint32_t d = 0; d < count; d++) {
                    gossip_engine* e = es[d];
                    for (uint32_t r = 0; r < count; r++) {
                        if (r == d) continue;
                        uint64_t lo, hi;
                        uint32_t wl;
                        geom(r, &lo, &hi, &wl);
                        const DevLayout L = dev_layout(hi - lo, e->ntw, wl);
                        const uint64_t cap = e->xcap[(size_t)r * gossip_engine::kMaxChunks + c];
                        int rc = e->ensure_dev(e->d_recv_msgs, e->recv_cap, L.rows + 16ull * cap);
                        if (rc) return rc;
                        // first round: prefix + the first `cap` rows (the header caps the unpack)
                        HIP_TRY(hipMemcpyAsync(e->d_recv_msgs, es[r]->d_msg, (L.rows + 16ull * cap) * 8,
                                               hipMemcpyDeviceToDevice, e->stream));
                        if ((rc = e->unpack_dev(t, lo, hi, wl, e->d_recv_msgs, e->d_recv_msgs + L.rows, 0, cap, true,
                                                e->stream)))
                            return rc;
                        if (tot[r] > cap) {  // second round: rows [cap, tot)
                            const uint64_t words = 16ull * (tot[r] - cap);
                            if ((rc = e->ensure_dev(e->d_ovf, e->ovf_cap, words))) return rc;
                            HIP_TRY(hipMemcpyAsync(e->d_ovf, es[r]->d_msg + L.rows + 16ull * cap, words * 8,
                                                   hipMemcpyDeviceToDevice, e->stream));
                            if ((rc = e->unpack_dev(t, lo, hi, wl, e->d_recv_msgs, e->d_ovf, cap, tot[r], false,
                                                    e->stream)))
                                return rc;
                            e->x_overflow_rounds++;
                        }
                        HIP_TRY(hipStreamSynchronize(e->stream));  // (receive buffers are reused)
                    }
                    for (uint32_t r = 0; r < count; r++) {  // (at most every tile row of the chunk)
                        uint64_t& cap = e->xcap[(size_t)r * gossip_engine::kMaxChunks + c];
                        uint64_t lo, hi;
                        uint32_t wl;
                        geom(r, &lo, &hi, &wl);
                        if (tot[r] > cap)
                            cap = std::min<uint64_t>(tot[r] + tot[r] / 4 + 16, (hi - lo) * (e->hw / kTileWords));
                    }
                }
            }
            for (uint32_t r = 0; r < count; r++) {
                HIP_TRY(hipSetDevice(es[r]->device));
                int rc = es[r]->tick_step_b(t);
                if (rc) return rc;
                es[r]->cur++;
            }
        }
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    return GOSSIP_OK;
}

int gossip_engine_set_option(gossip_engine* e, const char* name, int64_t value) {
    if (!e || !name) return set_error(GOSSIP_EINVAL, "NULL argument");
    const std::string k(name);
    if (k == "pull_nt") {
        if (value < -1 || value > 1) return set_error(GOSSIP_EINVAL, "pull_nt: -1 (auto), 0 or 1");
        e->opt_pull_nt = value;
    } else if (k == "pull_grid") {
        if (value < 0 || value > (1ll << 24)) return set_error(GOSSIP_EINVAL, "pull_grid: 0 (auto) .. 2^24 blocks");
        e->opt_pull_grid = value;
    } else if (k == "young") {
        if (value < -1 || value > 1) return set_error(GOSSIP_EINVAL, "young: -1 (auto), 0 or 1");
        if (e->have_sched) return set_error(GOSSIP_ESTATE, "young: set before the schedule");
        e->opt_young = value;
    } else if (k == "young_age") {
        if (value < 1 || value > 64) return set_error(GOSSIP_EINVAL, "young_age: 1 .. 64 hops");
        e->opt_young_age = value;
    } else if (k == "young_cap") {
        if (value < 1 || value > (int64_t)kSlotU16 - 1) return set_error(GOSSIP_EINVAL, "young_cap: 1 .. 127 entries");
        e->opt_young_cap = value;
    } else if (k == "young_overlap") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "young_overlap: 0 or 1");
        e->opt_young_overlap = value;
    } else if (k == "pull_tile_order") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "pull_tile_order: 0 or 1");
        e->opt_pull_tile_order = value;
    } else if (k == "pull_tiles") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "pull_tiles: 0 or 1");
        e->opt_pull_tiles = value;
    } else if (k == "pull_sat") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "pull_sat: 0 or 1");
        e->opt_pull_sat = value;
    } else if (k == "dense_rows") {
        if (value < -1 || value > 1) return set_error(GOSSIP_EINVAL, "dense_rows: -1 (auto), 0 or 1");
        e->opt_dense_rows = value;
    } else if (k == "pull_gate") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "pull_gate: 0 or 1");
        e->opt_pull_gate = value;
    } else if (k == "young_list_cap") {
        if (value < 1 || value > (int64_t)kListU16 - 1) return set_error(GOSSIP_EINVAL, "young_list_cap: 1 .. 127 entries");
        e->opt_young_list_cap = value;
    } else if (k == "young_nt") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "young_nt: 0 or 1");
        e->opt_young_nt = value;
    } else if (k == "young_idle") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "young_idle: 0 or 1");
        e->opt_young_idle = value;
    } else if (k == "pull_push") {
        if (value < -1 || value > 1) return set_error(GOSSIP_EINVAL, "pull_push: -1 (auto), 0 or 1");
        e->opt_pull_push = value;
    } else if (k == "young_skip") {
        if (value < -1 || value > 1) return set_error(GOSSIP_EINVAL, "young_skip: -1 (auto), 0 or 1");
        e->opt_young_skip = value;
    } else if (k == "young_grid") {
        if (value < 0 || value > (1 << 20)) return set_error(GOSSIP_EINVAL, "young_grid: 0 .. 2^20 blocks");
        e->opt_young_grid = value;
    } else if (k == "mem_limit") {
        if (value < 0) return set_error(GOSSIP_EINVAL, "mem_limit >= 0 bytes");
        if (e->have_sched) return set_error(GOSSIP_ESTATE, "mem_limit: set before the schedule");
        e->opt_mem_limit = value;
    } else if (k == "late_age") {
        if (value < -1 || value > 1000) return set_error(GOSSIP_EINVAL, "late_age: -1 (auto), 0 (off) .. 1000 ticks");
        e->opt_late_age = value;
    } else if (k == "xchunks") {
        if (value < 1 || value > (int64_t)gossip_engine::kMaxChunks) return set_error(GOSSIP_EINVAL, "xchunks: 1 .. 16 row chunks");
        if (e->tick_open) return set_error(GOSSIP_ESTATE, "xchunks: not between tick_begin and tick_end");
        if (e->comm) return set_error(GOSSIP_ESTATE, "xchunks: set before gossip_engine_connect_rccl");
        e->opt_xchunks = value;
    } else if (k == "rehearse_rows") {
        if (value < 0 || value > 64) return set_error(GOSSIP_EINVAL, "rehearse_rows: 0 (off) .. 64 row ranges");
        if (e->have_sched) return set_error(GOSSIP_ESTATE, "rehearse_rows: set before the schedule");
        if (value > 1 && e->row_count > 1)
            return set_error(GOSSIP_EINVAL, "rehearse_rows: an unpartitioned CSR engine");
        e->opt_rehearse_rows = value;
    } else if (k == "dense_fused") {
        if (value < 0 || value > 1) return set_error(GOSSIP_EINVAL, "dense_fused: 0 or 1");
        e->opt_dense_fused = value;
    } else if (k == "dense_min_tiles") {
        if (value < 1) return set_error(GOSSIP_EINVAL, "dense_min_tiles >= 1");
        e->opt_dense_min_tiles = value;
    } else {
        return set_error(GOSSIP_EINVAL, "unknown option '" + k + "'");
    }
    return GOSSIP_OK;
}

int gossip_engine_get_option(const gossip_engine* e, const char* name, int64_t* value) {
    if (!e || !name || !value) return set_error(GOSSIP_EINVAL, "NULL argument");
    const std::string k(name);
    const std::pair<const char*, int64_t> opts[] = {
        {"pull_nt", e->opt_pull_nt}, {"pull_grid", e->opt_pull_grid},
        {"young", e->opt_young}, {"young_age", e->opt_young_age},
        {"young_cap", e->opt_young_cap}, {"young_overlap", e->opt_young_overlap},
        {"pull_tile_order", e->opt_pull_tile_order}, {"pull_tiles", e->opt_pull_tiles},
        {"pull_sat", e->opt_pull_sat}, {"dense_rows", e->opt_dense_rows}, {"pull_gate", e->opt_pull_gate},
        {"young_list_cap", e->opt_young_list_cap}, {"young_nt", e->opt_young_nt},
        {"young_skip", e->opt_young_skip}, {"pull_push", e->opt_pull_push}, {"young_idle", e->opt_young_idle}, {"young_grid", e->opt_young_grid}, {"mem_limit", e->opt_mem_limit}, {"late_age", e->opt_late_age},
        {"xchunks", e->opt_xchunks}, {"rehearse_rows", e->opt_rehearse_rows},
        {"dense_fused", e->opt_dense_fused}, {"dense_min_tiles", e->opt_dense_min_tiles}};
    for (const auto& o : opts)
        if (k == o.first) {
            *value = o.second;
            return GOSSIP_OK;
        }
    return set_error(GOSSIP_EINVAL, "unknown option '" + k + "'");
}

// Host-staged exchange (any transport): tick_begin -> export own message -> import every other
// rank's -> tick_end.
static int check_stepping(gossip_engine* e) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (e->aborted.load()) return set_error(GOSSIP_ESTATE, "engine aborted (gossip_engine_abort)");
    if (!e->have_sched) return set_error(GOSSIP_ESTATE, "set graph and schedule first");
    if (e->comm) return set_error(GOSSIP_ESTATE, "host-staged stepping is not for an RCCL-connected engine");
    return GOSSIP_OK;
}

int gossip_engine_tick_begin(gossip_engine* e) {
    int rc = check_stepping(e);
    if (rc) return rc;
    if (e->tick_open) return set_error(GOSSIP_ESTATE, "tick_begin twice without tick_end");
    HIP_TRY(hipSetDevice(e->device));
    try {
        if (e->cur >= e->tick_end) return 1;
        if (e->batch && e->cur > e->last_birth_tick &&
            std::find(e->tile_alloc.begin(), e->tile_alloc.end(), (uint8_t)1) == e->tile_alloc.end()) {
            e->done = true;
            return 1;
        }
        // enqueued only: the exports wait for their row chunks (ev_chunk) on the exchange stream
        if ((rc = e->tick_step_a(e->cur))) return rc;
        if ((rc = e->ensure_xstream())) return rc;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    e->packed_tick = -1;
    e->tick_open = true;
    return GOSSIP_OK;
}

int gossip_engine_exchange_chunks(const gossip_engine* e) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    return e->row_count > 1 ? (int)std::min<int64_t>(gossip_engine::kMaxChunks, std::max<int64_t>(1, e->opt_xchunks)) : 1;
}

static int export_message(gossip_engine* e, uint32_t chunk, void* buf, uint64_t cap_bytes, uint64_t* bytes) {
    int rc = check_stepping(e);
    if (rc) return rc;
    if (!e->tick_open) return set_error(GOSSIP_ESTATE, "exchange_export outside tick_begin/tick_end");
    if (chunk != gossip_engine::kWholeRows && chunk >= e->nchunks)
        return set_error(GOSSIP_EINVAL, "exchange_export_chunk: chunk >= gossip_engine_exchange_chunks");
    HIP_TRY(hipSetDevice(e->device));
    if (e->packed_tick != e->cur || e->packed_chunk != chunk) {  // pack once per (tick, chunk)
        const uint32_t after = chunk == gossip_engine::kWholeRows ? e->nchunks - 1u : chunk;
        HIP_TRY(hipStreamWaitEvent(e->xstream, e->ev_chunk[after], 0));
        if ((rc = e->pack_rows(e->cur, chunk, e->xstream))) return rc;
        e->packed_tick = e->cur;
        e->packed_chunk = chunk;
    }
    if (bytes) *bytes = e->msg_words * 8;
    if (!buf) return GOSSIP_OK;
    if (cap_bytes < e->msg_words * 8) return set_error(GOSSIP_EINVAL, "export buffer too small");
    HIP_TRY(hipMemcpyAsync(buf, e->d_msg, e->msg_words * 8, hipMemcpyDeviceToHost, e->xstream));
    HIP_TRY(hipStreamSynchronize(e->xstream));
    return GOSSIP_OK;
}

static int import_message(gossip_engine* e, uint32_t rank, uint32_t chunk, const void* buf, uint64_t bytes) {
    int rc = check_stepping(e);
    if (rc) return rc;
    if (!e->tick_open) return set_error(GOSSIP_ESTATE, "exchange_import outside tick_begin/tick_end");
    if (rank >= e->row_count || rank == e->row_rank || !buf || bytes % 8)
        return set_error(GOSSIP_EINVAL, "exchange_import: bad rank or buffer");
    if (chunk != gossip_engine::kWholeRows && chunk >= e->nchunks)
        return set_error(GOSSIP_EINVAL, "exchange_import_chunk: chunk >= gossip_engine_exchange_chunks");
    HIP_TRY(hipSetDevice(e->device));
    if ((rc = e->ensure_dev(e->d_recv_msgs, e->recv_cap, std::max<uint64_t>(bytes / 8, 1)))) return rc;
    // The unpack ORs liveness into d_live and writes F_next / nz_next rows that this tick's
    // engine-stream work clears first (tick_step_a's memsets): order it after the chunk, even
    // when the caller imports before exporting its own message.
    {
        const uint32_t after = chunk == gossip_engine::kWholeRows ? e->nchunks - 1u : chunk;
        HIP_TRY(hipStreamWaitEvent(e->xstream, e->ev_chunk[after], 0));
    }
    HIP_TRY(hipMemcpyAsync(e->d_recv_msgs, buf, bytes, hipMemcpyHostToDevice, e->xstream));
    if ((rc = e->unpack_rows(e->cur, rank, chunk, e->d_recv_msgs, bytes / 8, e->xstream))) return rc;
    HIP_TRY(hipStreamSynchronize(e->xstream));  // (the receive buffer is reused by the next import)
    return GOSSIP_OK;
}

int gossip_engine_exchange_export(gossip_engine* e, void* buf, uint64_t cap_bytes, uint64_t* bytes) {
    return export_message(e, gossip_engine::kWholeRows, buf, cap_bytes, bytes);
}

int gossip_engine_exchange_import(gossip_engine* e, uint32_t rank, const void* buf, uint64_t bytes) {
    return import_message(e, rank, gossip_engine::kWholeRows, buf, bytes);
}

int gossip_engine_exchange_export_chunk(gossip_engine* e, uint32_t chunk, void* buf, uint64_t cap_bytes,
                                        uint64_t* bytes) {
    return export_message(e, chunk, buf, cap_bytes, bytes);
}

int gossip_engine_exchange_import_chunk(gossip_engine* e, uint32_t rank, uint32_t chunk, const void* buf,
                                        uint64_t bytes) {
    return import_message(e, rank, chunk, buf, bytes);
}

int gossip_engine_tick_end(gossip_engine* e) {
    int rc = check_stepping(e);
    if (rc) return rc;
    if (!e->tick_open) return set_error(GOSSIP_ESTATE, "tick_end without tick_begin");
    HIP_TRY(hipSetDevice(e->device));
    try {
        if ((rc = e->tick_step_b(e->cur))) return rc;
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    e->cur++;
    e->tick_open = false;
    return GOSSIP_OK;
}

int gossip_engine_set_link_timing(gossip_engine* e, int64_t ns_per_byte, uint32_t header_bytes,
                                  int64_t send_defer_ns) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (e->have_sched) return set_error(GOSSIP_ESTATE, "set link timing before the schedule");
    if (!e->batch)
        return set_error(GOSSIP_EINVAL, "link timing needs GOSSIP_F_HOP_BATCH (per-share cut masks)");
    if (ns_per_byte < 0 || send_defer_ns < 0) return set_error(GOSSIP_EINVAL, "negative link timing");
    // (any delay keeps hop order: it is the same at every hop of a share; the bound only
    // keeps hop * (L + delay) far inside int64)
    if (ns_per_byte > 1000000000ll || send_defer_ns > 1000000000ll)
        return set_error(GOSSIP_EINVAL, "link timing above 1 s per byte / per send");
    e->link_timing = true;
    e->link_npb = ns_per_byte;
    e->link_hdr = header_bytes;
    e->link_defer = send_defer_ns;
    return GOSSIP_OK;
}

int gossip_engine_set_schedule(gossip_engine* e, uint64_t num_events, const gossip_gen_event* ev) {
    if (!e || (num_events && !ev)) return set_error(GOSSIP_EINVAL, "NULL argument");
    if (!e->have_graph) return set_error(GOSSIP_ESTATE, "set the graph first");
    if (e->have_sched) return set_error(GOSSIP_ESTATE, "schedule already set");
    HIP_TRY(hipSetDevice(e->device));
    try {
        e->ev.assign(ev, ev + num_events);
        for (const auto& x : e->ev) {
            if (x.node >= e->n) return set_error(GOSSIP_EINVAL, "event node out of range");
            if (x.ns < e->cfg.t_start_ns || x.ns >= e->cfg.t_cut_ns)
                return set_error(GOSSIP_EINVAL, "event outside [t_start, t_cut): not a counted generation");
        }
        std::stable_sort(e->ev.begin(), e->ev.end(), [](const gossip_gen_event& a, const gossip_gen_event& b) {
            return a.ns != b.ns ? a.ns < b.ns : a.node < b.node;
        });
        for (uint64_t k = 1; k < e->ev.size(); k++)
            if (e->ev[k].node == e->ev[k - 1].node && e->ev[k].ns == e->ev[k - 1].ns)
                return set_error(GOSSIP_EINVAL, "duplicate generation event");
        if (e->handshake && e->h_degc.empty())
            return set_error(GOSSIP_ESTATE, "GOSSIP_F_HANDSHAKE needs the link keys: use gossip_engine_set_topology");
        // GenerateAndGossipShare's peers.empty() branch (p2pnode.cc:108-113): a generation at a
        // node without peers is not counted (before REGISTER only connector-side peers exist).
        {
            const int64_t t_reg = e->t0 + 3 * e->L;
            size_t o = 0;
            for (size_t k = 0; k < e->ev.size(); k++) {
                const gossip_gen_event& x = e->ev[k];
                const bool no_peers = e->h_peers[x.node] == 0 ||
                                      (e->handshake && x.ns < t_reg && e->h_degc[x.node] == 0);
                if (!no_peers) e->ev[o++] = x;
            }
            e->ev.resize(o);
        }
        if (e->handshake) {
            // A share sent before t_start + 2L is lost with its REGISTER segment and floods
            // nothing; its id must not belong to another generation the engine would merge.
            const int64_t t_est = e->t0 + 2 * e->L;
            std::vector<uint32_t> ids(e->ev.size());
            for (size_t k = 0; k < e->ev.size(); k++) ids[k] = e->ev[k].share_id;
            std::sort(ids.begin(), ids.end());
            for (const auto& x : e->ev) {
                if (x.ns >= t_est) break;  // sorted by ns
                const auto r = std::equal_range(ids.begin(), ids.end(), x.share_id);
                if (r.second - r.first > 1)
                    return set_error(GOSSIP_EINVAL, "GOSSIP_F_HANDSHAKE: a share lost in the handshake "
                                                    "window shares its id with another generation");
            }
        }
        if (e->batch) {
            // Shares are independent floods when no two generations share an id (the seen set
            // is keyed by id, p2pnode.cc:189), so each can run at any tick: generation g of a
            // node moves to tick tick0 + 1 + g with its phase.  Exact: counts depend only on
            // hops, and the cut / snapshots are applied per column from the real times.
            if (gossip::any_id_collision(e->ev.size(), e->ev.data()))
                return set_error(GOSSIP_EINVAL, "GOSSIP_F_HOP_BATCH needs unique share ids (n <= 128,849)");
            std::vector<uint32_t> gi(e->n, 0);
            std::vector<std::pair<gossip_gen_event, int64_t>> rm(e->ev.size());
            for (size_t k = 0; k < e->ev.size(); k++) {
                gossip_gen_event x = e->ev[k];
                const int64_t orig = x.ns;
                x.ns = (e->tick0 + 1 + (int64_t)gi[x.node]++) * e->L + orig % e->L;
                rm[k] = {x, orig};
            }
            std::stable_sort(rm.begin(), rm.end(), [](const auto& a, const auto& b) {
                return a.first.ns != b.first.ns ? a.first.ns < b.first.ns : a.first.node < b.first.node;
            });
            e->ev_orig_ns.resize(rm.size());
            for (size_t k = 0; k < rm.size(); k++) {
                e->ev[k] = rm[k].first;
                e->ev_orig_ns[k] = rm[k].second;
            }
            if (e->link_timing) {
                // per-share hop delay: the message is the same string at every hop
                e->ev_delta.resize(rm.size());
                for (size_t k = 0; k < rm.size(); k++) {
                    const uint32_t len = gossip_share_message_length(e->ev[k].node, e->ev[k].share_id,
                                                                     e->ev_orig_ns[k]);
                    e->ev_delta[k] = e->link_defer + ((int64_t)len + e->link_hdr) * e->link_npb;
                }
            }
            e->last_birth_tick = e->ev.empty() ? e->tick0 : e->ev.back().ns / e->L;
            e->cut_tick = -1;  // per-column cut instead
            e->tick_end = e->last_birth_tick + 1;
        }
        int rc = e->prepare_instances();
        if (rc) return rc;
        for (auto& s : e->snaps) {
            uint64_t g = 0, own = 0;
            for (size_t k = 0; k < e->ev.size(); k++)
                if ((e->batch ? e->ev_orig_ns[k] : e->ev[k].ns) < s.t_ns) {
                    g++;
                    own += e->ev[k].node >= e->v0 && e->ev[k].node < e->v1;
                }
            s.gen_total = g;
            s.own_gen_total = own;
        }
        rc = e->alloc_device();
        if (rc) return rc;
        if (e->batch) e->tick_end = INT64_MAX / 4;  // runs until every flood has retired
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    e->have_sched = true;
    return GOSSIP_OK;
}

int gossip_engine_set_schedule_obj(gossip_engine* e, const gossip_schedule* s) {
    if (!s) return set_error(GOSSIP_EINVAL, "NULL schedule");
    return gossip_engine_set_schedule(e, s->ev.size(), s->ev.data());
}

int64_t gossip_engine_first_tick(const gossip_engine* e) { return e ? e->tick0 : -1; }
int gossip_engine_mode(const gossip_engine* e) {
    if (!e) return GOSSIP_EINVAL;
    if (!e->have_graph && e->cfg.mode == GOSSIP_MODE_AUTO) return GOSSIP_MODE_AUTO;
    return e->dense ? GOSSIP_MODE_DENSE : GOSSIP_MODE_CSR;
}
int64_t gossip_engine_end_tick(const gossip_engine* e) { return e ? e->tick_end : -1; }
int64_t gossip_engine_current_tick(const gossip_engine* e) { return e ? e->cur : -1; }

int gossip_engine_run(gossip_engine* e, int64_t tick_end) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (e->aborted.load()) return set_error(GOSSIP_ESTATE, "engine aborted (gossip_engine_abort)");
    if (!e->have_sched) return set_error(GOSSIP_ESTATE, "set graph and schedule first");
    if (e->row_count > 1 && !e->comm)
        return set_error(GOSSIP_ESTATE, "row-partitioned engine: gossip_engine_connect_rccl or gossip_engine_group_run "
                                        "(or host-staged gossip_engine_tick_begin/exchange/tick_end)");
    HIP_TRY(hipSetDevice(e->device));
    if (tick_end > e->tick_end) tick_end = e->tick_end;
    try {
        while (e->cur < tick_end) {
            if (e->batch && e->cur > e->last_birth_tick &&
                std::find(e->tile_alloc.begin(), e->tile_alloc.end(), (uint8_t)1) == e->tile_alloc.end()) {
                e->done = true;
                break;
            }
            int rc = e->tick_step(e->cur);
            if (rc) return rc;
            e->cur++;
        }
    } catch (const std::bad_alloc&) {
        return set_error(GOSSIP_ENOMEM, "host allocation failed");
    }
    return GOSSIP_OK;
}

int gossip_engine_sync(gossip_engine* e) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    return GOSSIP_OK;
}

int gossip_engine_get_stats(gossip_engine* e, uint32_t* gen, uint32_t* recv, uint32_t* fwd,
                            uint64_t* sent, uint32_t* processed, uint32_t* peers,
                            uint32_t* sockets) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (!e->have_sched) return set_error(GOSSIP_ESTATE, "no schedule");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const size_t n = e->n;
    std::vector<uint32_t> r(n), g(n), eg(n);
    HIP_TRY(hipMemcpy(r.data(), e->d_recv, n * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(g.data(), e->d_gen, n * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(eg.data(), e->d_effgen, n * 4, hipMemcpyDeviceToHost));
    if (sent) {  // births' sends + deg x recv (header comment)
        HIP_TRY(hipMemcpy(sent, e->d_sent, n * 8, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) sent[i] += (uint64_t)r[i] * e->h_peers[i];
    }
    if (gen) std::memcpy(gen, g.data(), n * 4);
    if (recv) std::memcpy(recv, r.data(), n * 4);
    if (fwd) std::memcpy(fwd, r.data(), n * 4);  // sharesForwarded++ beside sharesReceived++
    if (processed)
        for (size_t i = 0; i < n; i++) processed[i] = r[i] + eg[i];
    if (peers) std::memcpy(peers, e->h_peers.data(), n * 4);
    if (sockets) std::memcpy(sockets, e->h_sockets.data(), n * 4);
    return GOSSIP_OK;
}

int gossip_engine_get_snapshot(gossip_engine* e, uint32_t k, int64_t* t_ns, uint64_t* total_gen,
                               uint64_t* total_processed) {
    if (!e || k >= e->snaps.size()) return set_error(GOSSIP_EINVAL, "bad snapshot index");
    if (!e->have_sched) return set_error(GOSSIP_ESTATE, "no schedule");
    const auto& s = e->snaps[k];
    HIP_TRY(hipSetDevice(e->device));
    if (t_ns) *t_ns = s.t_ns;
    if (total_gen) *total_gen = s.gen_total;
    if (e->batch && !e->done) return set_error(GOSSIP_ESTATE, "hop-batched snapshots need the complete run");
    if (s.t_ns > e->cfg.t_cut_ns) {
        // After PrintStatistics + StopAllNodes: counters frozen at t_cut (the caller reports
        // zero socket connections, p2pnode.cc:55-69).
        if (!e->batch && e->cur < e->tick_end) return set_error(GOSSIP_ESTATE, "snapshot after t_cut needs the full run");
        HIP_TRY(hipMemsetAsync(e->d_scalars, 0, 8, e->stream));
        k_sum_u32<<<256, 256, 0, e->stream>>>(e->d_recv, e->d_effgen, e->n, e->d_scalars);
        HIP_TRY(hipGetLastError());
        unsigned long long v = 0;
        HIP_TRY(hipMemcpyAsync(&v, e->d_scalars, 8, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (total_processed) *total_processed = v;
        return GOSSIP_OK;
    }
    if (!e->batch && e->cur <= s.tick - (s.r ? 0 : 1) && s.tick >= e->tick0)
        return set_error(GOSSIP_ESTATE, "snapshot time not simulated yet");
    HIP_TRY(hipStreamSynchronize(e->stream));
    unsigned long long v[2] = {0, 0};
    HIP_TRY(hipMemcpy(v, e->d_scalars + 2 + 2 * k, 16, hipMemcpyDeviceToHost));
    if (e->batch) {  // generations before T (all effective: unique ids) + arrivals before T
        if (total_processed) *total_processed = s.own_gen_total + v[1];
        return GOSSIP_OK;
    }
    if (total_processed) *total_processed = (s.tick <= e->tick0 && s.r == 0) ? 0 : (v[0] + v[1]);
    return GOSSIP_OK;
}

int gossip_engine_get_counters(gossip_engine* e, gossip_counters* c) {
    if (!e || !c) return set_error(GOSSIP_EINVAL, "NULL argument");
    std::memset(c, 0, sizeof(*c));
    c->ticks = e->ticks;
    c->pull_launches = e->pull_launches;
    c->pull_bytes = e->pull_bytes;
    c->words_hw = e->hw;
    c->words_cap = e->stride;
    c->device_bytes = e->device_bytes;
    if (!e->have_sched) return GOSSIP_OK;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    double ms = e->pull_ms_done;
    for (auto& p : e->timers) {
        float x = 0.f;
        HIP_TRY(hipEventElapsedTime(&x, p.first, p.second));
        ms += x;
        e->event_pool.push_back(p.first);
        e->event_pool.push_back(p.second);
    }
    e->timers.clear();
    e->pull_ms_done = ms;
    c->pull_ms = ms;
    HIP_TRY(hipMemsetAsync(e->d_scalars, 0, 16, e->stream));
    k_sum_sent<<<256, 256, 0, e->stream>>>(e->d_sent, e->d_recv, e->d_deg, e->n, e->d_scalars);
    k_sum_u32<<<256, 256, 0, e->stream>>>(e->d_recv, nullptr, e->n, e->d_scalars + 1);
    HIP_TRY(hipGetLastError());
    unsigned long long v[2];
    HIP_TRY(hipMemcpyAsync(v, e->d_scalars, 16, hipMemcpyDeviceToHost, e->stream));
    std::vector<unsigned long long> rep((size_t)kAcctSlots * kAcctReplicas, 0ull);
    HIP_TRY(hipMemcpyAsync(rep.data(), e->d_acct, rep.size() * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    unsigned long long acct[kAcctSlots] = {0};
    for (uint32_t r = 0; r < kAcctReplicas; r++)
        for (uint32_t q = 0; q < kAcctSlots; q++) acct[q] += rep[(size_t)r * kAcctSlots + q];
    c->edge_events = v[0];
    c->receptions = v[1];
    // Bytes k_pull actually had to move (work-skipping aware): peer-row pairs (16 B),
    // col indices of the node passes that pulled (4 B), own-row seen reads/writes and F_next
    // writes (16 B each), row_ptr and the per-node counters.
    c->pull_bytes_moved = 16ull * acct[0] + 4ull * acct[1] + 16ull * (acct[2] + acct[3] + acct[4]) +
                          8ull * acct[7] + e->pull_launches * (8ull * (e->n + 1) + 16ull * e->n + 8ull * e->n * e->ntw) +
                          16ull * e->n * std::min<uint32_t>(2u, e->ntw) * e->sat_launches +  // sat words r + w
                          8ull * acct[32] + (((uint64_t)e->n + 63) / 64 * 8) * e->mark_launches;  // push marks set / read
    c->pull_pair_edges = acct[0];
    c->dense_ops = acct[5];  // k_dense_gemm adds 2*M*N*K of every tile-split it computes
    c->dense_tiles_skipped = acct[6];
    c->pull_col_ids = acct[1];
    c->pull_seen_reads = acct[2];
    c->pull_seen_writes = acct[3];
    c->pull_f_writes = acct[4];
    c->pull_nz_reads = acct[7];
    c->pull_nt = e->last_nt;
    c->pull_grid = e->last_grid;
    {
        double yms = e->young_ms_done;
        for (auto& p : e->timers_young) {
            float x = 0.f;
            HIP_TRY(hipEventElapsedTime(&x, p.first, p.second));
            yms += x;
            e->event_pool.push_back(p.first);
            e->event_pool.push_back(p.second);
        }
        e->timers_young.clear();
        e->young_ms_done = yms;
        c->young_ms = yms;
        double pms = e->phase_ms_done;
        if (e->dense && e->d_phase_ts) {  // device-stamped DENSE spans (100 MHz ticks)
            unsigned long long ts[4];
            HIP_TRY(hipMemcpy(ts, e->d_phase_ts, sizeof(ts), hipMemcpyDeviceToHost));
            pms += (double)ts[2] * 1e-5;
        }
        for (auto& p : e->timers_phase) {
            float x = 0.f;
            HIP_TRY(hipEventElapsedTime(&x, p.first, p.second));
            pms += x;
            e->event_pool.push_back(p.first);
            e->event_pool.push_back(p.second);
        }
        e->timers_phase.clear();
        e->phase_ms_done = pms;
        c->pull_phase_ms = pms;
    }
    c->young_launches = e->young_launches;
    c->exchange_bytes_sent = e->exchange_bytes_out;
    c->exchange_bytes_received = e->exchange_bytes_in;
    c->young_slot_lines = acct[8];
    c->young_col_ids = acct[9];
    c->young_fallback_rows = acct[10];
    c->young_seen_reads = acct[11];
    c->young_seen_writes = acct[12];
    c->young_rows_written = acct[13];
    c->young_slot_writes = acct[14];
    // k_pull_young's bytes: 128 B per slot line / fallback row / row written / slot written,
    // 5 B per peer (id + second-line hint), 8 B per own seen word, row_ptr + counters per node
    // and launch
    c->young_line2_misses = acct[15];
    c->pull_late_age = (uint32_t)e->late_age_now();
    c->pull_tiles = e->pt_used ? 1u : 0u;
    c->young_bytes_moved = 128ull * (acct[8] + acct[10] + acct[13] + acct[14] + acct[15] + acct[17] + acct[18] + acct[19]) +
                           5ull * acct[9] +
                           8ull * (acct[11] + acct[12]) + e->young_launches * (8ull * (e->n + 1) + 16ull * e->n);
    c->young_fresh_lines = acct[19];
#ifdef DENSE_STAMPS
    fprintf(stderr, "dense_stamps_cycles");
    for (int k = 22; k < 32; k++) fprintf(stderr, " %llu", (unsigned long long)acct[k]);  // (30, 31: block time)
    fprintf(stderr, "\n");
#endif
#ifdef YOUNG_STAMPS
    fprintf(stderr, "young_stamps_cycles");
    for (int k = 22; k < 30; k++) fprintf(stderr, " %llu", (unsigned long long)acct[k]);  // (20, 21: k_pull items)
    fprintf(stderr, "\n");
#endif
    c->young_list_lines = acct[17] + acct[18];
    c->pull_lpw = e->last_lpw;
    c->pull_dense_tiles = e->last_dense_tiles;
    c->pull_sat_skips = acct[16];
    c->pull_items = acct[20];
    c->pull_gather_items = acct[21];
    c->dense_fused_launches = e->fused_launches;
    c->young_grid = e->last_young_grid;
    c->young_skip_ticks = (uint32_t)e->skip_ticks;
    c->young_idle_ticks = e->idle_ticks;
    c->pull_push_tiles = e->push_tiles;
    c->pull_pushw_tiles = e->pushw_tiles;
    c->pull_marks = acct[32];
    c->pull_sat = e->sat_used ? 1u : 0u;
    c->window_early_retires = e->early_retires;
    uint64_t g = 0;
    const uint64_t done = (uint64_t)std::max<int64_t>(0, std::min(e->cur, e->tick_end) - e->tick0);
    if (!e->tick_lo.empty()) g = e->tick_lo[std::min<uint64_t>(done, e->tick_lo.size() - 1)];
    c->generations = g;
    return GOSSIP_OK;
}

int gossip_engine_get_rehearsal(gossip_engine* e, uint32_t ranges, double* pull_ms, double* pack_ms,
                                double* unpack_ms, uint64_t* msg_bytes, uint64_t* ticks) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    if (e->opt_rehearse_rows < 2 || ranges != (uint32_t)e->opt_rehearse_rows)
        return set_error(GOSSIP_EINVAL, "get_rehearsal: ranges must equal the rehearse_rows option");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    e->rehearse_harvest();
    for (uint32_t r = 0; r < ranges; r++) {
        if (pull_ms) pull_ms[r] = e->rr_ms[0][r];
        if (pack_ms) pack_ms[r] = e->rr_ms[1][r];
        if (unpack_ms) unpack_ms[r] = e->rr_ms[2][r];
        if (msg_bytes) msg_bytes[r] = r < e->rr_bytes.size() ? e->rr_bytes[r] : 0;
    }
    if (ticks) *ticks = e->rr_ticks;
    return GOSSIP_OK;
}

int gossip_engine_get_rehearsal_peak(gossip_engine* e, uint32_t ranges, uint64_t* msg_bytes_max) {
    if (!e || !msg_bytes_max) return set_error(GOSSIP_EINVAL, "NULL argument");
    if (e->opt_rehearse_rows < 2 || ranges != (uint32_t)e->opt_rehearse_rows)
        return set_error(GOSSIP_EINVAL, "get_rehearsal_peak: ranges must equal the rehearse_rows option");
    for (uint32_t r = 0; r < ranges; r++) msg_bytes_max[r] = r < e->rr_bytes_max.size() ? e->rr_bytes_max[r] : 0;
    return GOSSIP_OK;
}

int gossip_engine_reset_timing(gossip_engine* e) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (auto& p : e->timers) {
        e->event_pool.push_back(p.first);
        e->event_pool.push_back(p.second);
    }
    e->timers.clear();
    e->pull_ms_done = 0.0;
    e->pull_launches = 0;
    e->pull_bytes = 0;
    for (auto& p : e->timers_young) {
        e->event_pool.push_back(p.first);
        e->event_pool.push_back(p.second);
    }
    e->timers_young.clear();
    e->young_ms_done = 0.0;
    e->young_launches = 0;
    e->skip_ticks = 0;
    e->idle_ticks = 0;
    e->push_tiles = 0;
    e->pushw_tiles = 0;
    e->mark_launches = 0;
    e->sat_launches = 0;
    for (auto& p : e->timers_phase) {
        e->event_pool.push_back(p.first);
        e->event_pool.push_back(p.second);
    }
    e->timers_phase.clear();
    e->phase_ms_done = 0.0;
    if (e->d_phase_ts) HIP_TRY(hipMemsetAsync(e->d_phase_ts + 2, 0, 16, e->stream));
    e->rehearse_harvest();  // (row-partition rehearsal: restart the per-range sums)
    for (auto& v : e->rr_ms) std::fill(v.begin(), v.end(), 0.0);
    std::fill(e->rr_bytes.begin(), e->rr_bytes.end(), 0ull);
    std::fill(e->rr_bytes_max.begin(), e->rr_bytes_max.end(), 0ull);
    e->rr_ticks = 0;
    if (e->d_acct) {
        HIP_TRY(hipMemsetAsync(e->d_acct, 0, kAcctSlots * kAcctReplicas * 8, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    return GOSSIP_OK;
}

uint64_t gossip_engine_trace_size(const gossip_engine* e) { return e ? e->tr.size() : 0; }

int gossip_engine_get_trace(const gossip_engine* e, uint32_t* node, uint32_t* share_id,
                            int64_t* tick, uint32_t* hop, uint8_t* via_recv) {
    if (!e) return set_error(GOSSIP_EINVAL, "NULL engine");
    for (size_t k = 0; k < e->tr.size(); k++) {
        const auto& r = e->tr[k];
        if (node) node[k] = r.node;
        if (share_id) share_id[k] = r.id;
        if (tick) tick[k] = r.tick;
        if (hop) hop[k] = r.hop;
        if (via_recv) via_recv[k] = r.via;
    }
    return GOSSIP_OK;
}

void gossip_engine_destroy(gossip_engine* e) {
    if (!e) return;
    hipSetDevice(e->device);
    delete e;
}

}  // extern "C"
