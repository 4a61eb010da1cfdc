// pull_kernel.h -- k_pull, the CSR pull over the bit-sliced frontier (included by engine.hip,
// which defines WordCtl, PullArgs and group_fix).
//
// One tick of P2PNode::HandleRead -> processedShares check -> ReceiveShare ->
// GossipShareToPeers (p2pnode.cc:127-199) for every node at once:
//     inc = OR_{u in peers(v)} F_cur[u];  new = inc & ~seen[v] & keep;  seen |= new;
//     F_next[v] = new;  recv[v] += popcount(new)   (sent[v] += |peers(v)| * popcount(new) is
//     derived: engine.hip, sent = births' sends + deg x recv)
//
// Lane layout: a node is served by GRP = LPW x EPN lanes.  Word-lane wl owns the 16-B word pair
// [2wl, 2wl+1] of every 2*LPW-word pass; edge-lane el takes every EPN-th peer.  Wide windows
// (sparse graphs) use EPN = 1, LPW = 32: a wave serves two nodes and reads 512 B of one peer
// row of each per instruction (LPW = 64, one node and 1 KiB per instruction, measured 4-9 %
// slower on C3/C4 and 20 % slower when a window ends in a half pass; engine.hip).
// Narrow windows on dense graphs use EPN > 1: lanes split the peer list, then OR-reduce.
// A launch covers the words [wbase, wbase + wact) of every row (wact <= kPullLdsWords).
//
// Per-word state shared by all nodes (last tick's liveness, the word flags) is staged in LDS
// once per block, so a work item carries only its own seen pair between pipeline stages.
//
// Latency structure.  The pull is a dependent-load chain per node (row_ptr -> peer ids ->
// peer occupancy words -> peer rows), so the kernel pipelines it: a wave owns 64 consecutive
// nodes and loads their row_ptr once; work items (node, pass) run in order, and in iteration k
// the kernel issues the own seen pair of item k+1, the peer ids of item k+2 and the peer
// occupancy words of item k+1 before the peer-row gathers of item k, so one round trip per
// item covers the whole chain.  Peer rows are gathered kInflight at a time (16 B per lane each).
//
// Work skipping (bytes the pull never moves):
//   dead pair  -- no column of the two words had a frontier bit anywhere last tick
//                 (live_prev == 0): nothing can arrive;
//   saturated  -- the node has seen every live column of the pair: peer rows not read;
//   empty row  -- a peer's 16-word tile row with no frontier bit (its occupancy bit in
//                 nz_cur is clear) is not read: young tiles are mostly empty rows;
//   covered    -- once the peer rows read so far hold every bit the node can still take
//                 (live last tick, unseen, kept) in all words of a tile, the tile's remaining
//                 peer rows cannot change `new` and are not read (bottom-up early exit, for
//                 tiles flagged WF_LATE: every tile by default, option late_age);
//   F_next tile rows are written only when some word of the tile got a bit (and the tile's
//   occupancy bit set); rows left unwritten hold stale bits that no reader ever loads.
//   saturated  -- (round 4, option pull_sat) a tile whose every live column the node has seen
//                 stays so until a birth lands in the tile (live columns only die: every
//                 incoming bit lies in live_prev), so k_pull keeps a per-node bit per tile
//                 (`sat`, written whole per occupancy word like nz_next) and skips the tile at
//                 that node -- no own-seen read, no peer row, no occupancy word -- while the host
//                 trusts the bit (tmask: listed last tick, no birth since, not re-allocated);
//   push marks -- (round 6, option pull_push) direction-optimising BFS's top-down step for tiles
//                 whose frontier sits on few nodes (the previous generation's stragglers, a
//                 tile's first hops): the tick before, every node that writes a non-empty row of
//                 such a tile (TM_PUSHW) sets its peers' bits in a per-node mark bitmap, and this
//                 tick the tile (TM_PUSH) is skipped at every UNMARKED node as if saturated -- none
//                 of its peers holds a row of it, so nothing can arrive.  The sat bits of TM_PUSH
//                 tiles are written back as 0 (an unmarked node's skip says nothing about them);
//   dense rows -- (round 4, option dense_rows) tiles whose frontier rows are dense everywhere
//                 (C4: F_cur at hops 5-7, ~100-760 bits per 1,024-share row) are read WITHOUT
//                 occupancy words: their writer of the last tick wrote every node's row (WF_DW,
//                 zeros included), so a peer's row is valid whatever its occupancy bit, and a
//                 node whose other listed tiles are all saturated or dense loads no occupancy
//                 word at all.  The random 8-B occupancy loads cost a line fetch each (C4: 282M
//                 per shard-tick, ~36 GB of the 37 GB of k_pull traffic above its algorithmic
//                 bytes, profiles/pmc_C4.json).
#pragma once

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long x) {
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

// Lanes of the wave for which c holds (a wave-uniform value: traffic accounting in SGPRs).
__device__ __forceinline__ uint32_t wave_count(bool c) { return (uint32_t)__popcll(__ballot(c)); }

// OR over aligned groups of G lanes.  Up to 16 lanes with DPP moves -- quad permutes, then the
// row half-mirror (lane i <-> 7 - i of each 8) and the row mirror (i <-> 15 - i of each 16) -- which
// are VALU operations; a __shfl_xor is a ds_bpermute through the LDS crossbar with a round trip
// per step, and k_pull runs several of these reductions per work item.  Beyond 16 lanes the last
// steps are shuffles.  Every lane of a group must be active (group-uniform control flow).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_or_step(uint32_t x) {
    return x | (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
template <int G>
__device__ __forceinline__ uint32_t group_or(uint32_t x, uint32_t lane) {  // lane: the caller's (G >= 32)
    static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "group size");
    if constexpr (G >= 2) x = dpp_or_step<0xB1>(x);   // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (G >= 4) x = dpp_or_step<0x4E>(x);   // quad_perm [2,3,0,1]: lane ^ 2
    if constexpr (G >= 8) x = dpp_or_step<0x141>(x);  // row_half_mirror: the other quad of the 8
    if constexpr (G >= 16) x = dpp_or_step<0x140>(x); // row_mirror: the other 8 of the row
    if constexpr (G >= 32) x |= lane_get(x, lane ^ 16u);
    if constexpr (G >= 64) x |= lane_get(x, lane ^ 32u);
    return x;
}
template <int G>
__device__ __forceinline__ unsigned long long group_or64(unsigned long long x, uint32_t lane) {
    return (unsigned long long)group_or<G>((uint32_t)x, lane) |
           ((unsigned long long)group_or<G>((uint32_t)(x >> 32), lane) << 32);
}
// Sum over aligned groups of G lanes (every lane of a group active), DPP up to 16 lanes.
template <int G>
__device__ __forceinline__ uint32_t group_add(uint32_t x, uint32_t lane) {
    if constexpr (G >= 2) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
    if constexpr (G >= 4) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
    if constexpr (G >= 8) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);
    if constexpr (G >= 16) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);
    if constexpr (G >= 32) x += lane_get(x, lane ^ 16u);
    if constexpr (G >= 64) x += lane_get(x, lane ^ 32u);
    return x;
}

// WF_YOUNG: the word belongs to a young tile, which k_pull_young owns this tick (young_kernel.h)
// WF_LATE: the word's tile is old enough (option late_age) for the bottom-up early exit
// WF_DW: write every node's F_next row of the tile, zeros included (its readers of the next tick
//        read it without occupancy words: dense rows, above)
enum : uint32_t { WF_CLEAR = 1u, WF_GROUP = 2u, WF_KEEP = 4u, WF_SNAP = 8u, WF_YOUNG = 16u, WF_LATE = 32u,
                  WF_DW = 64u, WF_BIRTH = 128u };  // WF_BIRTH: a generation lands in the word this tick (k_dense_fused)
// PullArgs::tmask, per occupancy word tw: [5 tw] dense-row tiles (read without occupancy words),
// [5 tw + 1] tiles whose sat bits are trusted this tick, [5 tw + 2] listed tiles that need occupancy,
// [5 tw + 3] push tiles (skipped at unmarked nodes), [5 tw + 4] push-write tiles (rows mark peers)
enum : uint32_t { TM_DENSE = 0, TM_SATOK = 1, TM_NZ = 2, TM_PUSH = 3, TM_PUSHW = 4, TM_WORDS = 5 };
constexpr uint32_t kTmSlots = 16;  // LDS words for the launch's (<= 2) occupancy words of tmask

constexpr uint32_t kPullLdsWords = 2048;  // words per launch: LDS liveness, new liveness, flags
#ifndef PULL_INFLIGHT
// 6 peer-row loads in flight per lane: k_pull<32,1> then holds 93 VGPRs, 5 waves per SIMD (8 in
// flight: 100 VGPRs, 4 waves); C4 shard, same box: k_pull alone 53.0 -> 50.0 ms, the early exit
// tested every 6 peers reads 5 % fewer rows (profiles/r03/ab/r3p2_*).  A/B builds: make variants
#define PULL_INFLIGHT 6
#endif
constexpr int kInflight = PULL_INFLIGHT;  // peer-row loads in flight per lane
// Non-temporal row accesses: a template switch of k_pull<LPW,1>, chosen at launch by bitmap size
// (engine.hip, kPullNtBytes).  On C4 (97 GB bitmaps) every row access non-temporal ran 128.6 ms
// per launch against 132.1 ms; on C3 (2 GB bitmaps) 3.59 ms against 3.31 ms
// (profiles/r01/nt_ab.json) -- so large windows stream, small ones keep the caches.
template <bool NT>
__device__ __forceinline__ ulonglong2 load_row16(const uint64_t* p) {
    if constexpr (NT) {
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        return make_ulonglong2(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1));
    } else {
        return *reinterpret_cast<const ulonglong2*>(p);
    }
}
template <bool NT>
__device__ __forceinline__ void store_row16(uint64_t* p, uint64_t x, uint64_t y) {
    if constexpr (NT) {
        unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
        __builtin_nontemporal_store((unsigned long long)x, q);
        __builtin_nontemporal_store((unsigned long long)y, q + 1);
    } else {
        *reinterpret_cast<ulonglong2*>(p) = make_ulonglong2(x, y);
    }
}

// + the keep masks of the launch's words when some word has WF_KEEP (the cut tick): read from
// LDS, a flagged word's mask never makes the wave wait on a global load
__host__ __device__ constexpr size_t pull_lds_bytes(uint32_t wact, bool keep = false, uint32_t nptile = 0) {
    return (size_t)wact * 16u + (((size_t)wact + 15u) & ~(size_t)15u) + (keep ? (size_t)wact * 8u : 0u) +
           (((size_t)nptile * 2u + 15u) & ~(size_t)15u);
}
// + (option pull_sat) the launch's two occupancy words of tmask and every wave's sat words of its
// 64 nodes (2 per node), the passes' live-tile masks and forced passes, every wave's per-step pass
// masks (empty items skipped), behind the rest
constexpr uint32_t kPullMaxPasses = 32;  // passes of a listed launch: kPullLdsWords / 16 / 4 tiles
constexpr size_t kPullSatLds = kTmSlots * 8u + 4u * 64u * 2u * 8u + kPullMaxPasses * 8u + 16u + 4u * kPullMaxPasses * 4u + 4u * 8u;
// + (push marks) every wave's forced push bits of its 64 nodes (2 occupancy words each)
constexpr size_t kPullPushLds = 4u * 64u * 2u * 8u;
static_assert(2u * TM_WORDS <= kTmSlots, "tmask words of a launch fit their LDS slot");
constexpr uint32_t kNoWord = 0xffffffffu;

// Peer ids of the first GRP peers of item k's node (0xffffffff past the list).
template <int LPW, int EPN>
__device__ __forceinline__ uint32_t pull_cid_load(const PullArgs& a, uint32_t step, uint64_t c0,
                                                  int64_t rp, int64_t rp_end, uint32_t gl,
                                                  uint32_t slot) {
    constexpr int NPW = 64 / (LPW * EPN);
    const uint32_t idx = step * NPW + slot;
    const int32_t beg = (int32_t)lane_get((uint32_t)rp, idx);
    const int32_t nx = (int32_t)lane_get((uint32_t)rp, (idx + 1u) & 63u);
    const int32_t end = (idx + 1u < 64u) ? nx : (int32_t)rp_end;
    const int32_t jj = beg + (int32_t)gl;
    return (c0 + idx < a.n && jj < end) ? (uint32_t)a.col[jj] : 0xffffffffu;
}

// SP (the C4 launch, engine.hip launch_pull_t): tile lists with dense-row tiles, saturation bits,
// empty-item skipping and the own-seen gate all on and no diagnostic no-skip -- compile-time
// flags instead of runtime ones (each runtime flag held a 64-bit SGPR mask; the kernel spilled
// SGPRs into VGPR lanes, and every reload in the item loop is a VALU instruction)
// PUSH (SP only): push marks on (PullArgs::mark_cur / mark_next; engine.hip launch_pull_t)
template <int LPW, int EPN, bool NT = false, bool SP = false, bool PUSH = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SP ? 5 : 1))) void k_pull(PullArgs a) {
    static_assert(SP || !PUSH, "push marks run in the SP instantiation");
    const bool noskip = SP ? false : a.noskip != 0u;
    constexpr int GRP = LPW * EPN;  // lanes per node
    constexpr int NPW = 64 / GRP;   // nodes per wave step
    static_assert(GRP <= 64 && (64 % GRP) == 0, "lane layout");
    extern __shared__ unsigned long long smem[];
    unsigned long long* s_lp = smem;             // live_prev of this launch's words
    unsigned long long* s_new = smem + a.wact;   // liveness of this tick (OR of new bits)
    uint8_t* s_wf = reinterpret_cast<uint8_t*>(smem + 2u * a.wact);
    unsigned long long* s_keep = smem + 2u * a.wact + ((a.wact + 15u) & ~15u) / 8u;
    uint16_t* s_pt = reinterpret_cast<uint16_t*>(s_keep + (a.keep_lds ? a.wact : 0u));
    for (uint32_t i = threadIdx.x; i < a.wact; i += 256) {
        const uint8_t f = a.wflags[a.wbase + i];
        // a young word is k_pull_young's: dead here, no clear, no write
        s_lp[i] = (f & WF_YOUNG) ? 0ull : (a.live_prev && !noskip) ? a.live_prev[a.wbase + i] : ~0ull;
        s_new[i] = 0ull;
        s_wf[i] = (f & WF_YOUNG) ? (uint8_t)0 : f;
        if (a.keep_lds) s_keep[i] = (f & WF_KEEP) ? a.ctl[a.wbase + i].keep : ~0ull;
    }
    for (uint32_t i = threadIdx.x; i < a.nptile; i += 256) s_pt[i] = a.ptile[i];
    // saturation bits and dense-row tiles (the gathering pull over tile lists only)
    const bool tm_on = SP || (EPN == 1 && a.tmask != nullptr && a.ptile != nullptr);  // dense rows (+ sat)
    const bool sat_on = SP || (tm_on && a.sat != nullptr);
    unsigned long long* s_tm = reinterpret_cast<unsigned long long*>(
        reinterpret_cast<char*>(smem) + pull_lds_bytes(a.wact, a.keep_lds != 0, a.nptile));
    unsigned long long* s_sat = s_tm + kTmSlots;  // [wave][node of the chunk][occupancy word of the launch]
    unsigned long long* s_plm = s_sat + 4u * 128u;  // [pass] live tiles (bits by tile in its nz word)
    uint32_t* s_pforce = reinterpret_cast<uint32_t*>(s_plm + kPullMaxPasses);  // passes every node runs
    uint32_t* s_smask = s_pforce + 4;  // [wave][step] passes some node of the step has work in
    // [wave] nodes of the chunk whose rows of push-write tiles mark their peers (push marks)
    unsigned long long* s_mkw = reinterpret_cast<unsigned long long*>(s_smask + 4u * kPullMaxPasses) + wave_in_block();
    if (PUSH && (threadIdx.x & 63u) == 0u) *s_mkw = 0ull;
    // [wave][node][occupancy word]: push tiles an unmarked node skips that its trusted sat bits did
    // not already cover -- removed from the sat words written back (the skip says nothing about
    // them; a trusted bit stays true: the node receives nothing in a push tile, live columns only die)
    unsigned long long* s_psk = s_mkw - wave_in_block() + 4u + (uint64_t)wave_in_block() * 128u;
    if (threadIdx.x < 2u * TM_WORDS) {
        const uint32_t twg = (a.wbase >> 10) + threadIdx.x / TM_WORDS;
        s_tm[threadIdx.x] = (tm_on && twg < a.ntw) ? a.tmask[twg * TM_WORDS + threadIdx.x % TM_WORDS] : 0ull;
    }
    // Empty items (tile lists with tmask): an item (node, pass) whose every tile is saturated at
    // the node (a trusted sat bit) or dead (no live column) moves nothing and changes nothing, so
    // the item sequence skips it.  Passes holding a tile that must be written or cleared anyway
    // (WF_CLEAR, WF_DW, WF_KEEP) are never skipped, and a node with any item runs the last pass of
    // each occupancy word (its nz and sat words are written back there, its counters after the
    // last pass).  A node with no item at all (round 6: on the sparse ticks of an 8-shard rank,
    // ~95 % of the nodes) runs none: its sat words are written back before the items.
    constexpr uint32_t TPP_ = LPW >= 8 ? (uint32_t)LPW / 8u : 1u;
    const bool skip_on = SP || (tm_on && a.nptile / TPP_ <= kPullMaxPasses);
    __syncthreads();  // (s_lp, s_wf, s_pt written)
    if (skip_on && threadIdx.x < 64u) {
        const uint32_t p = threadIdx.x, np = a.nptile / TPP_;
        unsigned long long lm = 0ull;
        bool force = false, last = p + 1u == np;
        if (p < np) {
            for (uint32_t k = 0; k < TPP_; k++) {
                const uint32_t t = s_pt[p * TPP_ + k];
                if (t == 0xffffu) continue;
                unsigned long long lv = 0ull;
                uint32_t fl = 0u;
                for (uint32_t q = 0; q < 16u; q++) {
                    lv |= s_lp[t * 16u + q];
                    fl |= s_wf[t * 16u + q];
                }
                if (lv) lm |= 1ull << (((a.wbase >> 4) + t) & 63u);
                if (fl & (WF_CLEAR | WF_DW | WF_KEEP)) force = true;
            }
            if (p + 1u < np && ((a.wbase + (uint32_t)s_pt[(p + 1u) * TPP_] * 16u) >> 10) !=
                                   ((a.wbase + (uint32_t)s_pt[p * TPP_] * 16u) >> 10))
                last = true;
            s_plm[p] = lm;
        }
        const unsigned long long fm = __ballot(p < np && force), lmk = __ballot(p < np && last);
        // the launch's occupancy words that hold a pass (bit q: tw_base + q)
        const unsigned long long tq = __ballot(p < np && ((a.wbase + (uint32_t)s_pt[p * TPP_] * 16u) >> 10) != (a.wbase >> 10));
        const unsigned long long t0 = __ballot(p < np && ((a.wbase + (uint32_t)s_pt[p * TPP_] * 16u) >> 10) == (a.wbase >> 10));
        if (threadIdx.x == 0) {
            s_pforce[0] = (uint32_t)fm;   // passes every node runs
            s_pforce[1] = (uint32_t)lmk;  // the last pass of each occupancy word (nodes with items)
            s_pforce[2] = (t0 ? 1u : 0u) | (tq ? 2u : 0u);
        }
    }
    __syncthreads();
    const uint32_t lane_id = threadIdx.x & 63u;
    // lane geometry, recomputed inside the loops from an opaque lane id (engine.hip, opaque)
#define PULL_LANES                                                                             \
    const uint32_t lane = opaque(lane_id);                                                    \
    const uint32_t gl = lane % GRP, wl = gl % LPW, el = gl / LPW, slot = lane / GRP;          \
    (void)el;
    const uint64_t stride = a.stride;
    const uint64_t n = a.n;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + wave_in_block();
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    // Pass geometry: consecutive 2 LPW-word passes, or (pull_tiles) LPW / 8 listed tiles per pass
    constexpr uint32_t TPP = LPW >= 8 ? (uint32_t)LPW / 8u : 1u;
    const bool listed = SP || a.ptile != nullptr;
    const uint32_t npass = listed ? a.nptile / TPP : (a.wact + 2u * LPW - 1u) / (2u * LPW);
    // launch-local word of this lane's pair in pass p (kNoWord: none)
    auto lw_of = [&](uint32_t p, uint32_t wl) -> uint32_t {
        if (!listed) {
            const uint32_t x = p * 2u * LPW + 2u * wl;
            return x < a.wact ? x : kNoWord;
        }
        const uint32_t t = s_pt[p * TPP + (wl >> 3)];
        return t == 0xffffu ? kNoWord : t * 16u + 2u * (wl & 7u);
    };
    // the occupancy word (1,024 words) of pass p: one per pass (listed groups never straddle one)
    auto tw_of = [&](uint32_t p) -> uint32_t {
        return listed ? (a.wbase + (uint32_t)s_pt[p * TPP] * 16u) >> 10 : (a.wbase + p * 2u * LPW) >> 10;
    };
    // bit k = the occupancy bit of pass p's k-th tile in the nz word nzw (a peer's, of tw_of(p))
    auto pass_bits = [&](unsigned long long nzw, uint32_t p) -> uint32_t {
        if (!listed) return (uint32_t)(nzw >> (((a.wbase + p * 2u * LPW) >> 4) & 63u)) & 0xffu;
        uint32_t r = 0;
#pragma unroll
        for (uint32_t k = 0; k < TPP; k++) {
            const uint32_t t = s_pt[p * TPP + k];
            if (t != 0xffffu) r |= (uint32_t)((nzw >> (((a.wbase >> 4) + t) & 63u)) & 1ull) << k;
        }
        return r;
    };
    const uint32_t nsteps = 64u / NPW;
    unsigned long long snap_local = 0ull;
    uint32_t t_pe = 0, t_col = 0, t_srd = 0, t_swr = 0, t_fwr = 0, t_nz = 0, t_sk = 0;  // wave-uniform
    uint32_t t_it = 0, t_gi = 0;  // node items, node items that gathered
    uint32_t t_mk = 0;            // push marks set (one 8-B atomic each)
    unsigned long long nzacc = 0ull;
    const bool gather = EPN == 1;  // the pipelined id/occupancy loads
    const uint32_t tw_base = a.wbase >> 10;  // the launch's first occupancy word
    unsigned long long* s_satw = s_sat + (uint64_t)wave_in_block() * 128u;
    // the trusted saturated tiles of the chunk's node idx in occupancy word tw
    auto satv_of = [&](uint32_t idx, uint32_t tw) -> unsigned long long {
        return sat_on ? s_satw[idx * 2u + (tw - tw_base)] : 0ull;
    };
    // does node idx need its peers' occupancy words of tw (some listed tile that is neither
    // dense-row nor saturated at the node)?
    auto nz_needed = [&](uint32_t idx, uint32_t tw) -> bool {
        return !tm_on || (s_tm[(tw - tw_base) * TM_WORDS + TM_NZ] & ~satv_of(idx, tw)) != 0ull;
    };

    for (uint64_t c0 = a.v0 + wave * 64u; npass && c0 < n; c0 += nwaves * 64u) {
        PULL_LANES
        const int64_t rp = a.rowptr[min(c0 + lane, n)];
        const int64_t rp_end = a.rowptr[min(c0 + 64u, n)];
        if (sat_on) {  // the chunk's sat words, trusted bits only (waited for below)
            const uint64_t vj = c0 + lane;
            // push tiles are skipped at an unmarked node like saturated ones (header comment)
            const bool unmarked = PUSH && a.mark_cur && vj < n && !((a.mark_cur[vj >> 6] >> (vj & 63u)) & 1ull);
#pragma unroll
            for (uint32_t q = 0; q < 2u; q++) {
                const uint32_t twg = tw_base + q;
                const unsigned long long tr = (vj < n && twg < a.ntw) ? a.sat[vj * a.ntw + twg] & s_tm[q * TM_WORDS + TM_SATOK] : 0ull;
                const unsigned long long pk = (unmarked && vj < n && twg < a.ntw) ? s_tm[q * TM_WORDS + TM_PUSH] & ~tr : 0ull;
                s_satw[lane * 2u + q] = tr | pk;
                if (PUSH) s_psk[lane * 2u + q] = pk;
            }
        }
        // per step, the passes some node of the step has work in (skip_on; else every pass)
        uint32_t* s_sm = s_smask + wave_in_block() * kPullMaxPasses;
        if (skip_on) {
            uint32_t m = 0u;
            const uint64_t vj = c0 + lane;
            if (vj < n) {
                for (uint32_t p = 0; p < npass; p++) {
                    const uint32_t twp = tw_of(p) - tw_base;
                    // (s_satw: this lane's node, written above by this lane)
                    if ((s_plm[p] & ~(sat_on ? s_satw[lane * 2u + twp] : 0ull)) != 0ull) m |= 1u << p;
                }
                m |= s_pforce[0];
                if (m || !PUSH) {  // (the idle-node skip runs in the PUSH instantiation only)
                    m |= s_pforce[1];
                } else if (sat_on) {  // no item: the node's sat words now (nz_next was zeroed)
                    const uint32_t tq = s_pforce[2];
#pragma unroll
                    for (uint32_t q = 0; q < 2u; q++)
                        if ((tq >> q) & 1u)
                            a.sat[vj * a.ntw + tw_base + q] = s_satw[lane * 2u + q] & ~(PUSH ? s_psk[lane * 2u + q] : 0ull);
                }
            }
            m = group_or<NPW>(m, lane);  // (the NPW nodes of a step are adjacent lanes)
            if (lane % NPW == 0u) s_sm[lane / NPW] = m;
            __builtin_amdgcn_wave_barrier();
        }
        // the item after (step, pass): the step's next pass with work, else the next step's first
        auto next_item = [&](uint32_t st, uint32_t ps, uint32_t& st1, uint32_t& ps1) {
            if (!skip_on) {
                st1 = ps + 1u < npass ? st : st + 1u;
                ps1 = ps + 1u < npass ? ps + 1u : 0u;
                return;
            }
            const uint32_t m = ps + 1u < 32u ? s_sm[st] & ~((2u << ps) - 1u) : 0u;
            if (m) {
                st1 = st;
                ps1 = (uint32_t)__builtin_ctz(m);
            } else {
                st1 = st + 1u;
                if constexpr (PUSH)
                    while (st1 < nsteps && s_sm[st1] == 0u) st1++;  // (steps without an item)
                ps1 = st1 < nsteps ? (uint32_t)__builtin_ctz(s_sm[st1]) : 0u;
            }
        };
        // item k = (step, pass): node c0 + step * NPW + slot, the lane's word pair lw_of(pass)
        uint32_t step = 0, pass = 0u;
        if (skip_on) {
            if constexpr (PUSH)
                while (step < nsteps && s_sm[step] == 0u) step++;
            pass = step < nsteps ? (uint32_t)__builtin_ctz(s_sm[step]) : 0u;
        }
        uint32_t first_step = 0xffffffffu;  // the step whose peer range beg/end holds
        ulonglong2 s2c = make_ulonglong2(0ull, 0ull);
        if (step < nsteps) {
            const uint64_t v = c0 + step * NPW + slot;
            const uint32_t lw = lw_of(pass, wl);
            if (v < n && lw != kNoWord && (s_lp[lw] | s_lp[lw + 1u]) != 0ull &&
                !((satv_of(step * NPW + slot, tw_of(pass)) >> (((a.wbase + lw) >> 4) & 63u)) & 1ull))
                s2c = load_row16<NT>(a.seen + v * stride + a.wbase + lw);
        }
        uint32_t cid0 = 0xffffffffu, cid1 = 0xffffffffu;
        unsigned long long nz0 = 0ull;
        if (gather && step < nsteps) {
            uint32_t s1, p1;
            next_item(step, pass, s1, p1);
            cid0 = pull_cid_load<LPW, EPN>(a, step, c0, rp, rp_end, gl, slot);
            cid1 = s1 == step ? cid0 : s1 < nsteps ? pull_cid_load<LPW, EPN>(a, s1, c0, rp, rp_end, gl, slot) : 0xffffffffu;
            const bool ld = cid0 != 0xffffffffu && nz_needed(step * NPW + slot, tw_of(pass));
            nz0 = ld ? a.nz_cur[(uint64_t)cid0 * a.ntw + tw_of(pass)] : 0ull;
            t_nz += wave_count(ld);
        }
        uint32_t cnt = 0;
        // Occupancy gate of the own-seen loads: nzor = OR over the node's peers of their
        // occupancy word (recomputed when the word changes); a tile no peer holds a row of
        // receives nothing, so its seen pair is not read (s2 gated: no gather, no write).
        // Only for nodes whose peers fit in one lane group, and only for the next item of the
        // same node and occupancy word (whose nz word is already in registers).
        unsigned long long nzor = 0ull;
        bool nz_new = true, s2c_gated = false;
        int32_t beg = 0, end = 0;  // the current node's peer range (read once per node)
        const bool gate = gather && (SP || (!noskip && a.gate_seen));
        // the first item's loads have landed before the item loop: inside it, every load is
        // then waited for by the item that issued it or the next (a loop header that merged a
        // pending first-item load would make every item wait for its own prefetches)
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
        while (step < nsteps) {
            PULL_LANES
            // ---- geometry of this item and the next two ----
            uint32_t step1, pass1, step2, pass2;
            next_item(step, pass, step1, pass1);
            if (step1 < nsteps)
                next_item(step1, pass1, step2, pass2);
            else
                step2 = nsteps;
            (void)pass2;
            const uint32_t idx = step * NPW + slot;
            const uint32_t v = (uint32_t)(c0 + idx);
            const uint32_t lw0 = lw_of(pass, wl);
            const uint32_t w = a.wbase + (lw0 == kNoWord ? 0u : lw0);
            const bool act = c0 + idx < n && lw0 != kNoWord;
            if (step != first_step) {  // (uniform) a new node: its peer range, with the whole wave active
                first_step = step;
                beg = (int32_t)lane_get((uint32_t)rp, idx);
                const int32_t nxb = (int32_t)lane_get((uint32_t)rp, (idx + 1u) & 63u);
                end = (idx + 1u < 64u) ? nxb : (int32_t)rp_end;
            }
            const uint32_t tw = tw_of(pass);  // (uniform: the pass's occupancy word)
            // dense-row tiles of the pass's occupancy word: every peer holds a valid row (uniform)
            const unsigned long long drm = tm_on ? s_tm[(tw - tw_base) * TM_WORDS + TM_DENSE] : 0ull;
            // ---- stage loads: own seen pair of item k+1, ids of k+2, occupancy of k+1 ----
            ulonglong2 s2n = make_ulonglong2(0ull, 0ull);
            bool s2n_gated = false;
            if (gate && nz_new) {  // (uniform) this item starts a new occupancy word
                unsigned long long x = nz0;
                x = group_or64<GRP>(x, lane);
                nzor = x | drm;
                nz_new = false;
            }
            if (step1 < nsteps) {
                // (a dead pair's seen words are never needed: only cleared, never merged)
                const uint64_t v1 = c0 + step1 * NPW + slot;
                const uint32_t lw1 = lw_of(pass1, wl);
                // this item's peer range was read with the whole wave active (a shuffle inside
                // the branch below would read the row pointers of lanes whose own pair is dead --
                // inactive lanes give no data -- so a node with more peers than one lane group
                // could pass the one-group test below and be gated on a partial occupancy OR)
                const int32_t b0 = beg, e0 = end;  // (this item's node)
                if (v1 < n && lw1 != kNoWord && (s_lp[lw1] | s_lp[lw1 + 1u]) != 0ull) {
                    // same node and occupancy word as this item, peers in one lane group
                    s2n_gated = gate && step1 == step && tw_of(pass1) == tw && e0 - b0 <= GRP &&
                                !((nzor >> (((a.wbase + lw1) >> 4) & 63u)) & 1ull);
                    // a saturated tile (trusted sat bit) needs nothing: not even its seen words
                    s2n_gated |= ((satv_of(step1 * NPW + slot, tw_of(pass1)) >> (((a.wbase + lw1) >> 4) & 63u)) & 1ull) != 0ull;
                    if (!s2n_gated) s2n = load_row16<NT>(a.seen + v1 * stride + a.wbase + lw1);
                }
            }
            uint32_t cid2 = 0xffffffffu;
            unsigned long long nz1 = 0ull;
            if (gather) {
                if (step2 < nsteps)
                    cid2 = step2 == step1 ? cid1 : pull_cid_load<LPW, EPN>(a, step2, c0, rp, rp_end, gl, slot);
                if (step1 < nsteps) {
                    const uint32_t tw1 = tw_of(pass1);
                    if (step1 == step && tw1 == tw) {
                        nz1 = nz0;  // same node, same occupancy word
                    } else {
                        const bool ld = cid1 != 0xffffffffu && nz_needed(step1 * NPW + slot, tw1);
                        nz1 = ld ? a.nz_cur[(uint64_t)cid1 * a.ntw + tw1] : 0ull;
                        t_nz += wave_count(ld);
                    }
                }
            }
            // ---- decide: is any peer row worth reading for this pair? ----
            uint32_t f0 = 0, f1 = 0;
            uint64_t lp0 = 0ull, lp1 = 0ull;
            if (act) {
                const uint32_t lw = w - a.wbase;
                const uint16_t fl = *reinterpret_cast<const uint16_t*>(s_wf + lw);
                f0 = fl & 0xffu;
                f1 = fl >> 8;
                lp0 = s_lp[lw];
                lp1 = s_lp[lw + 1u];
            }
            // a tile saturated at this node is a dead pair here: no seen read or write, nothing new
            const unsigned long long tbit = 1ull << ((w >> 4) & 63u);
            const bool sk = act && (satv_of(idx, tw) & tbit) != 0ull;
            if (sk) {
                lp0 = 0ull;
                lp1 = 0ull;
            }
            t_sk += wave_count(sk && (wl & 7u) == 0u);
            const bool dead = (lp0 | lp1) == 0ull;
            ulonglong2 s2 = s2c;
            if (f0 & WF_CLEAR) s2.x = 0ull;
            if (f1 & WF_CLEAR) s2.y = 0ull;
            uint64_t k0 = ~0ull, k1 = ~0ull;
            if (act && (f0 & WF_KEEP)) k0 = s_keep[w - a.wbase];
            if (act && (f1 & WF_KEEP)) k1 = s_keep[w + 1 - a.wbase];
            // Bits that can still become new (direction-optimising BFS, bottom-up): every F_cur
            // bit -- so every incoming bit -- lies inside live_prev, and seen / not-kept bits are
            // masked out of `new`, so new = incoming & want (and peers beyond covering `want`
            // add nothing).  Only `want` is carried past the gather.
            const uint64_t want0 = lp0 & ~s2.x & k0, want1 = lp1 & ~s2.y & k1;
            const bool need = act && !dead && !s2c_gated && (noskip || (want0 | want1) != 0ull);
            // Columns are allocated in 16-word tiles (one 128-B line per row, engine.hip), so the
            // read decision is made per tile: the 8 word-lanes of a tile load together and every
            // fetched line is fully used.
            int tn = need ? 1 : 0;
            tn = (int)group_or<8>((uint32_t)tn, lane);  // per tile (8 word-lanes)
            const bool tneed = tn != 0 && act;
            int gneed = tn;
            gneed = (int)group_or<GRP>((uint32_t)gneed, lane);
            t_it += wave_count(gl == 0 && c0 + idx < n);
            t_gi += wave_count(gl == 0 && gneed != 0);
            // ---- gather peer rows ----
            uint64_t acc0 = 0ull, acc1 = 0ull;
            if (gneed) {  // uniform inside the node group
                const uint64_t* Fw = a.Fcur + w;
                if constexpr (EPN == 1) {
                    // late tiles (WF_LATE, set by the host from the tile's age): dense frontier
                    // rows, few unseen bits -- stop at the first batch that covers them all
                    const bool late = ((f0 | f1) & WF_LATE) != 0u;
                    // one lane group's worth of peers (ids in `cid`, occupancy words in `nzw`)
                    auto gchunk = [&](uint32_t cid, unsigned long long nzw, int rem) {
                        t_col += wave_count((int)gl < rem);
                        // the <= 8 occupancy bits of this pass's tiles, tested per lane by tile
                        // (a dense-row tile: every peer's row, whatever its occupancy word says)
                        const uint32_t nzp = pass_bits(nzw | drm, pass);
                        for (int t0 = 0; t0 < rem; t0 += kInflight) {
                            int open = (noskip || !late)
                                           ? 1 : (((want0 & ~acc0) | (want1 & ~acc1)) != 0ull);
                            open = (int)group_or<8>((uint32_t)open, lane);  // per tile (8 word-lanes)
                            int gopen = open;
                            gopen = (int)group_or<GRP>((uint32_t)gopen, lane);
                            if (!gopen) break;  // uniform inside the node group
                            uint32_t u[kInflight], z[kInflight];
#pragma unroll
                            for (int t = 0; t < kInflight; t++) {
                                const uint32_t src = (lane & ~(uint32_t)(GRP - 1)) | ((uint32_t)(t0 + t) & (GRP - 1u));
                                u[t] = lane_get(cid, src);
                                z[t] = lane_get(nzp, src);
                            }
                            ulonglong2 q[kInflight];
#pragma unroll
                            for (int t = 0; t < kInflight; t++) {
                                q[t] = make_ulonglong2(0ull, 0ull);
                                const bool issue = open && tneed && t0 + t < rem && ((z[t] >> (wl >> 3)) & 1u);
                                if (issue) q[t] = load_row16<NT>(Fw + (uint64_t)u[t] * stride);
                                t_pe += wave_count(issue);
                            }
#pragma unroll
                            for (int t = 0; t < kInflight; t++) {
                                acc0 |= q[t].x;
                                acc1 |= q[t].y;
                            }
                        }
                    };
                    // the first lane group of peers is straight-line code (its ids and occupancy
                    // came with the previous item), so no loop header makes the wave wait for
                    // the loads this item just issued for the next ones
                    gchunk(cid0, nz0, min(GRP, end - beg));
                    for (int32_t cb = beg + GRP; cb < end; cb += GRP) {  // more peers (rare)
                        const int rem = min(GRP, end - cb);
                        const int32_t jj = cb + (int32_t)gl;
                        const uint32_t cid = (jj < end) ? (uint32_t)a.col[jj] : 0u;
                        const bool ld = (int)gl < rem && nz_needed(idx, tw);
                        const unsigned long long nzw = ld ? a.nz_cur[(uint64_t)cid * a.ntw + tw] : 0ull;
                        t_nz += wave_count(ld);
                        gchunk(cid, nzw, rem);
                    }
                } else {
                    // edge-lane el walks peers beg+el, beg+el+EPN, ...; 8 in flight
                    for (int32_t j0 = beg + (int32_t)el; j0 < end; j0 += 8 * EPN) {
                        uint32_t u[8];
                        unsigned long long z[8];
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            const int32_t j = j0 + t * EPN;
                            u[t] = (tneed && j < end) ? (uint32_t)a.col[j] : 0xffffffffu;
                            t_col += wave_count(wl == 0 && u[t] != 0xffffffffu);
                        }
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            z[t] = 0ull;
                            if (u[t] != 0xffffffffu) z[t] = a.nz_cur[(uint64_t)u[t] * a.ntw + tw];
                            t_nz += wave_count(u[t] != 0xffffffffu);
                        }
                        ulonglong2 q[8];
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            q[t] = make_ulonglong2(0ull, 0ull);
                            const bool issue = u[t] != 0xffffffffu && (z[t] & tbit) != 0ull;
                            if (issue) q[t] = *reinterpret_cast<const ulonglong2*>(Fw + (uint64_t)u[t] * stride);
                            t_pe += wave_count(issue);
                        }
#pragma unroll
                        for (int t = 0; t < 8; t++) {
                            acc0 |= q[t].x;
                            acc1 |= q[t].y;
                        }
                    }
                }
            }
            if constexpr (EPN > 1) {
#pragma unroll
                for (int off = LPW; off < GRP; off <<= 1) {
                    const uint32_t src = lane ^ (uint32_t)off;
                    acc0 |= (uint64_t)lane_get((uint32_t)acc0, src) | ((uint64_t)lane_get((uint32_t)(acc0 >> 32), src) << 32);
                    acc1 |= (uint64_t)lane_get((uint32_t)acc1, src) | ((uint64_t)lane_get((uint32_t)(acc1 >> 32), src) << 32);
                }
            }
            // Everything this item loaded -- the gather's rows and the next items' prefetches -- has
            // landed before its stores issue: gfx950 counts stores in vmcnt, and the pipeline's
            // hand-over at the loop latch (s2c = s2n, nz0 = nz1, the ids) would otherwise wait with
            // the item's stores outstanding (vmcnt(0): a write round trip per item)
            __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
            // ---- dedup ----
            uint64_t n0 = 0ull, n1 = 0ull;
            if (act && el == 0 && !dead) {
                n0 = acc0 & want0;
                n1 = acc1 & want1;
                if (f0 & WF_GROUP) n0 = group_fix(n0, s2.x, a.ctl[w].gmask, a.ctl[w].gstart);
                if (f1 & WF_GROUP) n1 = group_fix(n1, s2.y, a.ctl[w + 1].gmask, a.ctl[w + 1].gstart);
            }
            // tile occupancy of F_next: the 8 word-lanes of a tile agree on writing the row
            // (NOSKIP diagnostic: every tile row is written and marked occupied, so the pull
            // reads every peer row -- the dense-pull byte count)
            int ta = (n0 | n1) != 0ull || (noskip && act);
            ta = (int)group_or<8>((uint32_t)ta, lane);
            // a WF_DW tile's row is written at every node (zeros too): read as a dense row next tick
            const bool trow = ta || (act && (f0 & WF_DW));
            // ---- push marks: a non-empty row of a push-write tile marks every peer of the node,
            //      after the chunk's items (the node's bit in the wave's LDS word meanwhile) ----
            if (PUSH && a.mark_next && ta && act && (wl & 7u) == 0u &&
                ((s_tm[(tw - tw_base) * TM_WORDS + TM_PUSHW] & tbit) != 0ull))
                atomicOr(s_mkw, 1ull << idx);
            // ---- saturation bit of the tile: every live column of it seen, after this tick ----
            // (want = live & unseen & kept, so want & ~new are the live columns still unseen; a
            // keep-masked word's dropped columns are unseen too: never saturated on a keep tick)
            // The bit is updated in place in the node's LDS sat word, which the occupancy word's
            // last item writes back whole.
            if (sat_on) {
                int un = ((want0 & ~n0) | (want1 & ~n1)) != 0ull || ((f0 | f1) & WF_KEEP) != 0u;
                un = (int)group_or<8>((uint32_t)un, lane);
                if (act && (wl & 7u) == 0u) {
                    unsigned long long* sw = s_satw + idx * 2u + (tw - tw_base);
                    if (un)
                        atomicAnd(sw, ~tbit);
                    else
                        atomicOr(sw, tbit);
                }
            }
            // ---- state, counters (one lane per word pair) ----
            const bool own = act && el == 0;
            const bool swr = own && (dead ? ((f0 | f1) & WF_CLEAR) != 0u
                                          : ((n0 | n1) != 0ull || ((f0 | f1) & WF_CLEAR) != 0u));
            t_fwr += wave_count(own && trow);
            t_srd += wave_count(own && !dead && !s2c_gated);
            t_swr += wave_count(swr);
            if (own) {
                uint64_t* sp = a.seen + (uint64_t)v * stride + w;
                uint64_t* fp = a.Fnext + (uint64_t)v * stride + w;
                if (trow) store_row16<NT>(fp, n0, n1);
                if (swr) {
                    if (dead && !((f0 & f1) & WF_CLEAR))
                        sp[(f0 & WF_CLEAR) ? 0 : 1] = 0ull;
                    else
                        store_row16<NT>(sp, s2.x | n0, s2.y | n1);
                }
                if (!dead) {
                    cnt += (uint32_t)(__popcll(n0) + __popcll(n1));
                    if (a.snap) {
                        if (f0 & WF_SNAP) snap_local += (unsigned long long)__popcll(n0 & a.ctl[w].snap);
                        if (f1 & WF_SNAP) snap_local += (unsigned long long)__popcll(n1 & a.ctl[w + 1].snap);
                    }
                    if (n0) atomicOr(&s_new[w - a.wbase], (unsigned long long)n0);
                    if (n1) atomicOr(&s_new[w + 1 - a.wbase], (unsigned long long)n1);
                }
            }
            // ---- occupancy word of this node, written whole once per nz word index ----
            {
                unsigned long long nb = (ta && own && (wl & 7u) == 0u) ? tbit : 0ull;
                nb = group_or64<GRP>(nb, lane);
                nzacc |= nb;
                const bool last_of_tw = pass + 1u == npass || tw_of(pass + 1u) != tw;
                if (last_of_tw) {
                    if (gl == 0 && c0 + idx < n) {
                        if (!a.shared_out)
                            a.nz_next[(uint64_t)v * a.ntw + tw] = nzacc;
                        else if (nzacc)
                            atomicOr(&a.nz_next[(uint64_t)v * a.ntw + tw], nzacc);
                        if (sat_on)
                            a.sat[(uint64_t)v * a.ntw + tw] = s_satw[idx * 2u + (tw - tw_base)] &
                                                              ~(PUSH ? s_psk[idx * 2u + (tw - tw_base)] : 0ull);
                    }
                    nzacc = 0ull;
                }
            }
            // ---- per-node counters after the node's last pass ----
            // (a no-return atomic: nothing waits on it -- a read-modify-write, or a load of the
            // node's |peers| here, would wait with the item's stores outstanding, vmcnt(0), and
            // drain the pipeline's prefetches once per node.  sent is not touched: every reception
            // sends |peers| copies, so the engine derives sent = births' sends + deg x recv)
            if (pass + 1u == npass) {
                const uint32_t c = group_add<GRP>(cnt, lane);
                if (gl == 0 && c) atomicAdd(&a.recv[v], c);
                cnt = 0;
            }
            // ---- advance the pipeline ----
            s2c = s2n;
            s2c_gated = s2n_gated;
            cid0 = cid1;
            cid1 = cid2;
            nz_new = step1 != step || tw_of(pass1) != tw;
            nz0 = nz1;
            step = step1;
            pass = pass1;
        }
        if (PUSH && a.mark_next) {  // (uniform) the chunk's marking nodes: every peer's bit (rare by the
            __builtin_amdgcn_wave_barrier();  //  host's choice of push-write tiles)
            unsigned long long mk = *s_mkw;
            __builtin_amdgcn_wave_barrier();
            if (lane_id == 0) *s_mkw = 0ull;
            uint32_t nm = 0;
            while (mk) {
                const uint32_t j = (uint32_t)__builtin_ctzll(mk);
                mk &= mk - 1ull;
                const int32_t b = (int32_t)lane_read((uint32_t)rp, j);
                const int32_t e = j + 1u < 64u ? (int32_t)lane_read((uint32_t)rp, j + 1u) : (int32_t)rp_end;
                for (int32_t q = b + (int32_t)lane_id; q < e; q += 64) {
                    const uint32_t u = (uint32_t)a.col[q];
                    atomicOr(&a.mark_next[u >> 6], 1ull << (u & 63u));
                    nm++;
                }
            }
            t_mk += wave_sum32(nm);
        }
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane_id == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.acct && lane_id == 0) {
        const uint32_t tv[10] = {t_pe, t_col, t_srd, t_swr, t_fwr, t_nz, t_sk, t_it, t_gi, t_mk};
        const int slot_of[10] = {0, 1, 2, 3, 4, 7, 16, 20, 21, 32};
#pragma unroll
        for (int q = 0; q < 10; q++)
            if (tv[q]) acct_add(a.acct, (uint32_t)slot_of[q], (unsigned long long)tv[q]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.wact; i += 256) {
        const unsigned long long x = s_new[i];
        if (x) atomicOr(&a.live[a.wbase + i], x);
    }
#undef PULL_LANES
}

// Diagnostic build only (Makefile engine_sk.o; results are WRONG there): tiles at least
// GOSSIP_DIAG_SKIP_AGE ticks old are left out of k_pull's lists, to price the passes over the
// previous generations' straggler tiles.  The product build leaves the lists as they are.
#ifdef PULL_DIAG_SKIP_ENV
#include <cstdlib>
static inline bool diag_skip_tile(int64_t age) {
    static const long a = std::getenv("GOSSIP_DIAG_SKIP_AGE") ? std::atol(std::getenv("GOSSIP_DIAG_SKIP_AGE")) : 0;
    return a > 0 && age >= a;
}
#define PULL_DIAG_SKIP(tl) || diag_skip_tile(t - tile_first[tl])
#else
#define PULL_DIAG_SKIP(tl)
#endif
