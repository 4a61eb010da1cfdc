// young_kernel.h -- k_pull_young: the pull for YOUNG frontier tiles, whose rows hold a handful of
// bits (included by engine.hip after pull_kernel.h).
//
// Why.  A share at hop h has reached ~deg^h nodes, so a 1024-share tile of age <= 4 holds a few
// bits per node row (C4: ~7 of 1,024 at age 4, < 1 at age 3) -- yet k_pull reads the whole
// 128-B row of every peer that has one bit, and the HBM cost of a random gather is per 128-B line
// (tools/gather_probe: 64-B rows give half the GB/s of 128-B rows).  At C4, ages 1-4 are ~40 % of
// the peer-row lines k_pull reads.
//
// Representation.  Next to the dense rows, every node has a SLOT of 256 B (two lines) per
// frontier buffer: u16[0] = number of entries c (or kSlotOverflow), u16[1..c] = the node's
// frontier bits in the tick's WRITE-SPARSE tiles, one entry per bit: (w_idx << 10) | bit, with
// w_idx the tile's index in that tick's write-sparse list (< 63; 0xffff is a tombstone).  ~47
// entries per node at C4, so a peer costs one line read instead of ~9 row reads.  A node with
// more entries than the capacity is OVERFLOWED: its slot says so and its dense rows of every
// write-sparse tile are written (zeros included); readers fall back to those rows.
//
// Which tiles (host, engine.hip tick_step_a): a tile is write-sparse at tick t while its oldest
// shares are at most `young_age` hops old in F_{t+1}; read-sparse at t iff it was write-sparse at
// t-1.  This kernel owns the words of every read-sparse tile (k_pull skips them: WF_YOUNG) and of
// fresh write-sparse tiles; the tiles leaving the young set (read-sparse, write-dense) are written
// back as dense rows with their occupancy bits, for k_pull to read next tick.
//
// Per node (one wave; dependent round trips: slot lines -- peer ids are prefetched a node ahead,
// hinted second lines come with the first -- then the own seen words): gather the peers' slots
// (8 lanes x 16 B per peer, 24 peers per batch) and scatter their entries into a per-wave LDS
// accumulator of the read-sparse words; compact the touched words into a list; dedup them against
// the own seen words (the same WordCtl masks as k_pull: keep, id groups, snapshot), counters, the
// output slot (wave prefix sum of the entry counts) and the dense rows of the tiles leaving the
// young set.  64 VGPRs (round 3: lane values recomputed per node, explicit-lane shuffles) and ~5
// KiB of LDS per wave, so that 6-8 waves per SIMD hide the round trips (an explicitly pipelined
// variant measured no faster: the loop-carried registers forced vmcnt(0) waits, profiles/r02/).
// The young words' liveness is reported as all-ones (a young tile is alive by definition; it
// retires after it leaves the young set, through k_pull's exact liveness).
//
// Seen lists (round 4).  A node's processedShares bits in its young tiles are few (C4: ~53 of the
// ~36k shares of the young tiles, hops <= 4), yet in the dense seen rows every one of them cost an
// 8-B read and an 8-B write a few per 128-B line (1.3x the bytes), and every fresh tile a 128-B
// clear per node (8 GB per C4 shard-tick).  So each node keeps them as a LIST of 256 B (header +
// 127 u16 entries (yid << 10) | (word << 6) | bit, yid = the tile's young id, stable while the tile
// is young), read with the first batch of peer slots (no dependent seen round trip), applied to
// the accumulator as AND-NOT, and rewritten in whole lines.  An id group's bits enter the list all
// together (any seen bit of a group blocks the group, group_fix: holding all of them is the same
// test).  A tile leaving the young set gets its dense seen rows MATERIALISED (list entries | this
// tick's new bits, whole 128-B lines: the stale rows of the tile's previous life are overwritten,
// so fresh tiles need no clear).  A list that would exceed kListCap entries (or k_births' append)
// OVERFLOWS: the node's dense seen rows of its young tiles are materialised and used from then on
// (dense words read and written as before, fresh tiles cleared at that node).
// Header: (kept << 7) | total; entries [1, kept] are the kept entries of earlier ticks, (kept,
// total] this tick's arrivals (and births): k_births tests an id group against the former only.
#pragma once

constexpr uint32_t kSlotU16 = 128;           // 256 B per node per frontier buffer
constexpr uint32_t kSlotOverflow = 0xffffu;  // header: the node's dense rows are valid
constexpr uint32_t kSlotTomb = 0xffffu;      // entry: removed (id-group birth beat an arrival)
constexpr uint32_t kYoungMax = 48;           // tiles per launch
constexpr uint32_t kYoungWriteMax = 40;      // write-sparse tiles per tick (w_idx < 40 <= 62)
constexpr int kYoungQ = 3;  // slot-line loads per batch: 24 peers (C4: P(deg > 24) ~ 2 %)
constexpr uint32_t kListU16 = 128;           // seen list: 256 B per node (header + 127 entries)
constexpr uint32_t kListOverflow = 0xffffu;  // header: the dense seen rows of the young tiles are valid
constexpr uint32_t kListReserve = 8;         // entries left for k_births' appends after k_pull_young
constexpr uint32_t kListCap = kListU16 - 1u - kListReserve;  // k_pull_young overflows a list beyond this
constexpr uint32_t kYidNone = 0xffu;
__host__ __device__ constexpr uint32_t list_header(uint32_t kept, uint32_t total) { return (kept << 7) | total; }
// YT_DW (a leaving tile): write every node's dense row, zeros too -- k_pull reads the tile next
// tick as dense rows, without occupancy words (pull_kernel.h)
enum : uint32_t { YT_READ = 1u, YT_WRITE = 2u, YT_DW = 4u };

struct YoungTile {
    uint32_t tile;
    uint8_t flags;  // YT_READ: F_cur holds this tile in slots; YT_WRITE: F_next goes to slots
    uint8_t r_idx;  // w_idx of this tile in F_cur's entries (YT_READ)
    uint8_t w_idx;  // index written into F_next's entries (YT_WRITE)
    uint8_t yid;    // young id: the tile's index in the seen lists' entries while it is young
};

// yt order (host): [0, nr) the read-sparse tiles BY THEIR INDEX IN F_cur's ENTRIES (so an entry
// (r << 10) | (word << 6) | bit lands in accumulator word (r << 4) | word = entry >> 6, with no
// lookup), then [nr, ny) the fresh write-sparse tiles (no input).  A read tile is leaving
// (YT_READ only: dense output) or staying (YT_READ | YT_WRITE); lv[0, nt) lists the leaving
// positions by tile.  Every unused entry of a written slot line is a tombstone, so readers
// scatter whole lines without looking at the count (tombstones land in spare words).
struct YoungArgs {
    const int64_t* rowptr;
    const int32_t* col;
    const uint64_t* Fcur;
    uint64_t* Fnext;
    uint64_t* seen;
    const uint16_t* slot_cur;
    uint16_t* slot_next;
    const WordCtl* ctl;
    const uint8_t* wflags;
    uint32_t* recv;
    unsigned long long* live;
    unsigned long long* snap;  // nullable
    unsigned long long* acct;  // nullable
    unsigned long long* nz_next;
    uint32_t ntw;
    const YoungTile* yt;
    uint32_t ny, nr, nt;
    const uint8_t* lv;  // [nt] positions in yt of the leaving tiles, by tile
    uint32_t n, v0, stride, cap;
    // Second-line hints (per CSR entry): hint_cur[j] == stamp_cur says that the slot of peer
    // col[j] holds more than 63 entries this tick, so its second line is loaded together with the
    // first; a writer with a two-line slot marks every reverse entry rev[j] of its own list in
    // hint_next with stamp_next.  A hint is only a hint: a peer whose header says two lines
    // without one is fetched on demand (acct[15]).
    const uint8_t* hint_cur;
    uint8_t* hint_next;
    const int32_t* rev;
    uint32_t stamp_cur, stamp_next;
    // Empty-slot skipping (round 6, option young_skip).  On the ticks after a shard's births most
    // slots are EMPTY (C4, one rank of 8: the births tick's slots hold ~34k of 10M nodes' entries,
    // the next tick's ~5 %), yet every node read its ~16 peers' slot lines -- 25 GB per launch for
    // nothing.  When the host expects the slots written this tick to be sparse (sparse_wr), every
    // writer of a NON-EMPTY slot (here and in k_births) also stamps its reverse entries, with
    // stamp1_next for one line (stamp_next still means two lines), and the next tick's readers
    // (sparse_rd) load only the peers whose hint byte carries one of the two stamps: an unstamped
    // peer's slot is empty (a stale byte that happens to match costs one useless line, never a
    // result).  The hint bytes ride with the peer ids, so skipping adds no round trip.
    uint32_t stamp1_cur, stamp1_next;
    uint32_t sparse_rd, sparse_wr;
    // Idle nodes (round 6): with nothing to read but stamped slots (sparse_rd, or no read tile) and
    // no young tile leaving or gone (every seen-list entry stays), a node none of whose peers holds
    // a stamped slot gets no bit and keeps its list: per 64-node chunk, one pass over the chunk's
    // hint bytes finds the nodes with work, and the others only get an empty slot and their list
    // header's this-tick part folded into `kept` -- no per-node walk (~800 VALU each).
    uint32_t fast;
    unsigned long long* work;  // fast: per 64-node chunk from v0, its nodes with work (k_young_idle)
    uint32_t slot_nt;  // option young_nt: non-temporal slot-line loads (C4 shard, young alone 21.1 -> 19.0 ms)
    uint16_t* list;        // n x kListU16 seen lists
    const uint8_t* ymap;   // [64] young id -> position in yt (0xff: none)
    uint32_t list_cap;     // entries a list may keep (kListCap; option young_list_cap for tests)
};

constexpr uint32_t kYoungSpare = 32;  // spare accumulator words per wave (tombstones land here)

__host__ __device__ constexpr size_t young_lds_bytes(uint32_t ny, uint32_t nr) {
    // 4 waves x (accumulator 8 B per read word + spares, touched list 2 B per read word, a slot
    // and a seen-list staging buffer), tiles, read-word flags, leaving positions, young ids
    return 4u * ((size_t)nr * 16u + kYoungSpare) * 8u + 4u * (size_t)nr * 16u * 2u + 4u * kSlotU16 * 2u +
           4u * kListU16 * 2u + (size_t)ny * sizeof(YoungTile) + (size_t)nr * 16u + 64u + 64u;
}

// x with every id group it touches made whole (gm / gs: the word's group bits and group starts;
// groups are contiguous runs, group_fix's layout)
__device__ __forceinline__ uint64_t group_expand(uint64_t x, uint64_t gm, uint64_t gs) {
    uint64_t todo = x & gm, out = x;  // (the groups holding a bit of x, group_fix)
    while (todo) {
        const uint64_t grp = group_of((uint32_t)__builtin_ctzll(todo), gm, gs);
        out |= grp;
        todo &= ~grp;
    }
    return out;
}

// Inclusive prefix sum over the wave (every lane active), DPP only: row shifts inside each row of
// 16, then the row broadcasts of lanes 15 and 31 (a ds_bpermute chain costs an LDS round trip a step)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Entry j (0..7) of a lane's 16-B piece of a slot line.
__device__ __forceinline__ uint32_t slot_entry(const ulonglong2& q, int j) {
    const uint64_t word = j < 4 ? q.x : q.y;
    return (uint32_t)(word >> (16 * (j & 3))) & 0xffffu;
}

// Set bits of m below the calling lane (v_mbcnt: 2 VALU, no 64-bit shift of a lane mask).
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Diagnostic build YOUNG_STAMPS: shader cycles per phase of the node loop (s_memtime), summed
// over waves into acct[22..29] (engine.hip prints them with the counters); no output depends on them
#ifdef YOUNG_STAMPS
#define YSTAMP(k)                                              \
    do {                                                       \
        const uint64_t ys_t = __builtin_amdgcn_s_memtime();    \
        ycyc[k] += ys_t - ylast;                               \
        ylast = ys_t;                                          \
    } while (0)
#elif defined(YOUNG_MARKS)
#define YSTAMP(k) asm volatile(";YMARK " #k ::)
#else
#define YSTAMP(k) \
    do {          \
    } while (0)
#endif

// Measurement build YOUNG_DUP=k (tools/ab: instruction counts per segment by PMC): segment k of the
// node loop runs twice on the same data -- the first launch's count difference is its cost.  Its
// outputs are wrong by design (counters double); never a product build.
#ifndef YOUNG_DUP
#define YOUNG_DUP 0
#endif
#if YOUNG_DUP
#define YDUP(k) for (int ydup_ = 0; ydup_ < (YOUNG_DUP == (k) ? 2 : 1); ydup_++)
#else
#define YDUP(k)  // (the product build: no wrapper at all -- a one-trip loop still moved register allocation)
#endif

// 256-thread blocks; the register budget of 4 waves per SIMD (A/B build: YOUNG_MIN_WAVES)
#ifndef YOUNG_MIN_WAVES
#define YOUNG_MIN_WAVES 4
#endif
// SPARSE: the instantiation of the sparse ticks (engine.hip launch_young: empty-slot skipping, the
// idle-node pass's work masks, no read tile); the other one keeps the dense ticks' register
// allocation (SGPR spills 54 vs 72: ~0.5 ms per C4 shard-tick, profiles/r06/)
template <bool SPARSE>
__global__ __launch_bounds__(256, YOUNG_MIN_WAVES) void k_pull_young(YoungArgs a) {
    extern __shared__ unsigned long long smem[];
    const uint32_t nrw = a.nr * 16u;  // accumulated words
    const uint32_t accw = nrw + kYoungSpare;
    const uint32_t lane_id = threadIdx.x & 63u, wv = wave_in_block();
    unsigned long long* s_acc = smem + wv * accw;
    uint16_t* s_list = reinterpret_cast<uint16_t*>(smem + 4u * accw) + wv * nrw;
    uint16_t* s_out = reinterpret_cast<uint16_t*>(smem + 4u * accw) + 4u * nrw + wv * kSlotU16;  // 16-B aligned
    uint16_t* s_lst = reinterpret_cast<uint16_t*>(smem + 4u * accw) + 4u * nrw + 4u * kSlotU16 + wv * kListU16;
    YoungTile* s_yt = reinterpret_cast<YoungTile*>(reinterpret_cast<uint16_t*>(smem + 4u * accw) + 4u * nrw +
                                                   4u * kSlotU16 + 4u * kListU16);
    uint8_t* s_wf = reinterpret_cast<uint8_t*>(s_yt + a.ny);
    uint8_t* s_lv = s_wf + nrw;
    uint8_t* s_ymap = s_lv + 64;
    for (uint32_t i = threadIdx.x; i < a.ny; i += 256) s_yt[i] = a.yt[i];
    if (threadIdx.x < a.nt) s_lv[threadIdx.x] = a.lv[threadIdx.x];
    if (threadIdx.x < 64u) s_ymap[threadIdx.x] = a.ymap[threadIdx.x];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nrw; i += 256) s_wf[i] = a.wflags[s_yt[i >> 4].tile * 16u + (i & 15u)];
    for (uint32_t i = lane_id; i < accw; i += 64) s_acc[i] = 0ull;
    if (blockIdx.x == 0)  // young tiles are alive by definition (see above)
        for (uint32_t i = threadIdx.x; i < a.ny * 16u; i += 256)
            if (s_yt[i >> 4].flags) a.live[s_yt[i >> 4].tile * 16u + (i & 15u)] = ~0ull;
    __syncthreads();
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + wv;
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t stride = a.stride;
    unsigned long long snap_local = 0ull;
    // traffic (wave-uniform): slot lines, peer ids, dense fallback rows, seen r/w, row/slot writes,
    // unhinted second lines, seen-list lines read / written, seen rows materialised / cleared
    uint32_t t_sl = 0, t_col = 0, t_fb = 0, t_srd = 0, t_swr = 0, t_rw = 0, t_slw = 0, t_miss = 0;
    uint32_t t_lr = 0, t_lw = 0, t_mat = 0;
#ifdef YOUNG_STAMPS
    uint64_t ycyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t ylast = __builtin_amdgcn_s_memtime();
#endif

    for (uint64_t c0 = a.v0 + wave * 64u; c0 < a.n; c0 += nwaves * 64u) {
        const uint32_t lane = opaque(lane_id);
        const uint32_t cnt_nodes = (uint32_t)min<uint64_t>(64u, a.n - c0);
        const int64_t rp = a.rowptr[c0 + min(lane, cnt_nodes)];
        const int64_t rp_end = a.rowptr[c0 + cnt_nodes];
        // peer ids of node j (lane p = peer p of its first 64), one node ahead of the gather
        // (the peer's id and its hint byte, combined only when the node's gather starts: bit 31
        // of the id says the peer's slot has a second line -- ids are < 2^31)
        auto load_ids = [&](uint32_t j, uint32_t& hint, int32_t& rv) -> uint32_t {
            const int32_t b = (int32_t)lane_read((uint32_t)rp, j & 63u);
            const int32_t nx = (int32_t)lane_read((uint32_t)rp, (j + 1u) & 63u);
            const int32_t e = j + 1u < 64u ? nx : (int32_t)rp_end;
            hint = 0u;
            rv = -1;
            if (!(j < cnt_nodes && (int32_t)lane < e - b)) return 0xffffffffu;
            hint = a.hint_cur[b + (int32_t)lane];
            rv = a.rev[b + (int32_t)lane];  // (for the node's second-line hints, if it writes two lines)
            return (uint32_t)a.col[b + (int32_t)lane];
        };
        auto with_hint = [&](uint32_t id, uint32_t hint) -> uint32_t {
            if (id == 0xffffffffu) return id;
            if (hint == a.stamp_cur) return id | 0x80000000u;
            return (SPARSE && a.sparse_rd && hint != a.stamp1_cur) ? 0xffffffffu : id;  // (an empty slot: skipped)
        };
        // sparse_rd: the peers left after with_hint, moved to the front of the wave (lane p = the
        // p-th peer with a stamped slot), so the gather's batches cover them only (np0 = their number)
        auto compact = [&](uint32_t id, uint32_t lane) -> uint32_t {
            const unsigned long long m = __ballot(id != 0xffffffffu);
            uint32_t* sc = reinterpret_cast<uint32_t*>(s_out);  // (free until the node's dedup)
            if (id != 0xffffffffu) sc[lanes_below(m)] = id;
            __builtin_amdgcn_wave_barrier();
            const uint32_t r = lane < (uint32_t)__popcll(m) ? sc[lane] : 0xffffffffu;
            __builtin_amdgcn_wave_barrier();
            return r;
        };
        // the chunk's nodes with work: every node, unless k_young_idle found the idle ones (fast)
        const unsigned long long work = (SPARSE && a.fast) ? a.work[(c0 - a.v0) >> 6]
                                                           : cnt_nodes >= 64u ? ~0ull : ((1ull << cnt_nodes) - 1ull);
        uint32_t h_cur = 0u;
        int32_t rv_cur = -1;
        uint32_t jn = SPARSE ? (work ? (uint32_t)__builtin_ctzll(work) : 64u) : 0u;
        uint32_t cid_cur = load_ids(jn, h_cur, rv_cur);
        cid_cur = with_hint(cid_cur, h_cur);
        for (; jn < cnt_nodes;) {
            // the next node with work (64: none)
            const unsigned long long wn = (SPARSE && jn + 1u < 64u) ? work & ~((2ull << jn) - 1ull) : 0ull;
            const uint32_t jnext = !SPARSE ? jn + 1u : wn ? (uint32_t)__builtin_ctzll(wn) : 64u;
            const uint32_t lane = opaque(lane_id);
            const uint64_t v = c0 + jn;
            // the 8 entries of a lane's 16-B piece of a slot line; `hdr`: entry 0 is the line's header
            const uint32_t spare_h = 2u * (nrw + (lane & (kYoungSpare - 1u)));  // (half-word index)
            auto scatter8 = [&](const ulonglong2& q, bool hdr) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t e = (j == 0 && hdr) ? kSlotTomb : slot_entry(q, j);
                    // 32-bit LDS atomics on the half word holding the bit, e >> 5 (half the data moved
                    // per lane, one mask register); a tombstone's half word (> every real one) is
                    // clamped into the lane's spare word.  4 VALU per entry: extract, clamp,
                    // address, mask
                    atomicOr(reinterpret_cast<uint32_t*>(s_acc) + min(e >> 5, spare_h), 1u << (e & 31u));
                }
            };
            const int32_t beg = (int32_t)lane_read((uint32_t)rp, jn);
            const int32_t nx = (int32_t)lane_read((uint32_t)rp, (jn + 1u) & 63u);
            const int32_t end = jn + 1u < 64u ? nx : (int32_t)rp_end;
            // ---- gather: peers' slots -> accumulator, in batches of 8 kYoungQ peers ----
            // (the first batch is straight-line code: its loads go out before the next node's id
            // prefetch, and no loop header makes the wave wait for that prefetch)
            ulonglong2 q[kYoungQ], q2[kYoungQ];
            auto issue = [&](uint32_t cid, int32_t pb) {
#pragma unroll
                for (int k = 0; k < kYoungQ; k++) {
                    const uint32_t p = (uint32_t)pb + (uint32_t)k * 8u + (lane >> 3);
                    const uint32_t u = lane_get(cid, p);
                    q[k] = make_ulonglong2(~0ull, ~0ull);  // tombstones: nothing to scatter
                    q2[k] = make_ulonglong2(~0ull, ~0ull);
                    if (p < 64u && u != 0xffffffffu) {
                        const uint16_t* sl = a.slot_cur + (uint64_t)(u & 0x7fffffffu) * kSlotU16 + (lane & 7u) * 8u;
                        // (option young_nt: peers' slot lines are read once per reader and never
                        // reused from the caches -- non-temporal, like k_pull's rows)
                        if (a.slot_nt) {
                            q[k] = load_row16<true>(reinterpret_cast<const uint64_t*>(sl));
                            if (u & 0x80000000u) q2[k] = load_row16<true>(reinterpret_cast<const uint64_t*>(sl + 64u));
                        } else {
                            q[k] = *reinterpret_cast<const ulonglong2*>(sl);
                            if (u & 0x80000000u) q2[k] = *reinterpret_cast<const ulonglong2*>(sl + 64u);
                        }
                    }
                }
            };
            // bit p of ovf: peer p of the 64-peer chunk overflowed (its dense rows are read)
            auto consume = [&](uint32_t cid, int32_t pb, int32_t np, unsigned long long& ovf) {
                uint32_t missk = 0u;  // bit k: group k's peer has a second line nobody announced
#pragma unroll
                for (int k = 0; k < kYoungQ; k++) {
                    if (pb + k * 8 >= np) break;  // (uniform) no peer in this group of 8
                    const uint32_t p = (uint32_t)pb + (uint32_t)k * 8u + (lane >> 3);
                    const uint32_t u = lane_get(cid, p);
                    const bool valid = p < 64u && u != 0xffffffffu;
                    const bool hinted = valid && (u & 0x80000000u);
                    const uint32_t hdr = valid ? lane_get((uint32_t)(q[k].x & 0xffffull), lane & ~7u) : 0u;
                    t_sl += wave_count(valid && (lane & 7u) == 0u) + wave_count(hinted && (lane & 7u) == 0u);
                    // an overflowed slot's entries are a subset of its dense rows (read below)
                    scatter8(q[k], (lane & 7u) == 0u);
                    const bool two = hdr != kSlotOverflow && hdr > 63u;
                    if (__ballot(two || hinted)) {  // (uniform) some second line in this group
                        if (two && !hinted) missk |= 1u << k;  // fetched after the batch
                        if (!two) q2[k] = make_ulonglong2(~0ull, ~0ull);  // stale hint
                        scatter8(q2[k], false);
                    }
                    const unsigned long long mo = __ballot((lane & 7u) == 0u && valid && hdr == kSlotOverflow);
                    if (mo) {
#pragma unroll
                        for (int g = 0; g < 8; g++)
                            if ((mo >> (8 * g)) & 1ull) ovf |= 1ull << (((uint32_t)pb + (uint32_t)k * 8u + (uint32_t)g) & 63u);
                    }
                }
                if (__ballot(missk != 0u)) {  // (uniform, rare) unannounced second lines
                    for (int k = 0; k < kYoungQ; k++) {
                        const bool miss = (missk >> k) & 1u;
                        if (!__ballot(miss)) continue;
                        const uint32_t p = (uint32_t)pb + (uint32_t)k * 8u + (lane >> 3);
                        const uint32_t u = lane_get(cid, p) & 0x7fffffffu;
                        ulonglong2 x = make_ulonglong2(~0ull, ~0ull);
                        if (miss) x = *reinterpret_cast<const ulonglong2*>(a.slot_cur + (uint64_t)u * kSlotU16 + 64u + (lane & 7u) * 8u);
                        t_miss += wave_count(miss && (lane & 7u) == 0u);
                        scatter8(x, false);
                    }
                }
            };
            auto fallback = [&](uint32_t cid, unsigned long long ovf) {
                while (ovf) {  // overflowed peers: their dense rows of every read-sparse tile
                    const int p = __builtin_ctzll(ovf);
                    ovf &= ovf - 1ull;
                    const uint32_t u = lane_read(cid, (uint32_t)p) & 0x7fffffffu;
                    for (uint32_t i = lane; i < nrw; i += 64) {
                        if (!s_yt[i >> 4].flags) continue;  // a position whose tile is gone
                        const uint64_t x = a.Fcur[(uint64_t)u * stride + s_yt[i >> 4].tile * 16u + (i & 15u)];
                        if (x) s_acc[i] |= x;  // this lane owns word i here
                    }
                    t_fb += a.nr;
                }
            };
            // (sparse_rd: only the stamped peers, compacted; nr == 0 -- no read tile, e.g. a births
            //  tick after a tick without young tiles -- nothing to gather at all)
            if (SPARSE && a.nr == 0u)
                cid_cur = 0xffffffffu;
            else if (SPARSE && a.sparse_rd)
                cid_cur = compact(cid_cur, lane);
            const int32_t np0 = !SPARSE ? min(64, end - beg)
                                : a.nr == 0u ? 0 : a.sparse_rd ? (int32_t)wave_count(cid_cur != 0xffffffffu) : min(64, end - beg);
            t_col += (uint32_t)max(0, end - beg);
            unsigned long long ovf = 0ull;
            YDUP(7) issue(cid_cur, 0);
            // own seen list (its two lines, 2 entries per lane), with the first batch
            const uint32_t ql = reinterpret_cast<const uint32_t*>(a.list + v * kListU16)[lane];
            t_lr += 2u;
            uint32_t h_next = 0u;
            int32_t rv_next = -1;
            const uint32_t cid_next = load_ids(jnext, h_next, rv_next);  // the next node's peers
            YSTAMP(0);
            YDUP(1) consume(cid_cur, 0, np0, ovf);
            for (int32_t pb = 8 * kYoungQ; pb < np0; pb += 8 * kYoungQ) {  // degree > 8 kYoungQ
                issue(cid_cur, pb);
                consume(cid_cur, pb, np0, ovf);
            }
            fallback(cid_cur, ovf);
            for (int32_t cb = beg + 64; a.nr && cb < end; cb += 64) {  // peers beyond the first 64 (rare)
                const int32_t np = min(64, end - cb);
                uint32_t cid = 0xffffffffu;
                if ((int32_t)lane < np) cid = with_hint((uint32_t)a.col[cb + (int32_t)lane], a.hint_cur[cb + (int32_t)lane]);
                unsigned long long ovf2 = 0ull;
                for (int32_t pb = 0; pb < np; pb += 8 * kYoungQ) {
                    issue(cid, pb);
                    consume(cid, pb, np, ovf2);
                }
                fallback(cid, ovf2);
            }
            YSTAMP(1);
            // ---- seen list: clear the incoming bits the node already holds (p2pnode.cc:189) ----
            const uint32_t lhdr = lane_read(ql & 0xffffu, 0u);
            const bool lovf = lhdr == kListOverflow;  // (uniform) dense seen rows instead
            const uint32_t ltot = lovf ? 0u : (lhdr & 127u);
            // entry j (0, 1) of this lane's pair (kSlotTomb: none)
            auto lentry = [&](uint32_t j) -> uint32_t {
                const uint32_t idx = lane * 2u + j;
                const uint32_t e = (ql >> (16u * j)) & 0xffffu;
                return (idx == 0u || idx > ltot || e == kSlotTomb) ? kSlotTomb : e;
            };
            uint32_t keepm = 0u;  // bit j: entry j is kept into the new list (its tile stays young)
            reinterpret_cast<uint32_t*>(s_lst)[lane] = 0xffffffffu;  // tombstones
            __builtin_amdgcn_wave_barrier();
            YDUP(2) if (!lovf) {
#pragma unroll
                for (uint32_t j = 0; j < 2u; j++) {
                    const uint32_t e = lentry(j);
                    const uint32_t qp = e == kSlotTomb ? 0xffu : s_ymap[e >> 10];
                    if (qp >= a.ny) continue;  // (none, or a tile no longer young: dropped)
                    if (qp < a.nr)
                        atomicAnd(reinterpret_cast<uint32_t*>(s_acc + qp * 16u + ((e >> 6) & 15u)) + ((e >> 5) & 1u),
                                  ~(1u << (e & 31u)));
                    if (s_yt[qp].flags & YT_WRITE) keepm |= 1u << j;
                }
            }
            // kept entries -> s_lst[1, kept]
            uint32_t kept = 0;
            YDUP(10) {
                const uint32_t c = (uint32_t)__builtin_popcount(keepm);
                const uint32_t incl = wave_incl_scan(c);
                uint32_t pos = 1u + incl - c;
                kept = lane_read(incl, 63u);
                if (keepm & 1u) s_lst[pos++] = (uint16_t)(ql & 0xffffu);
                if (keepm & 2u) s_lst[pos] = (uint16_t)(ql >> 16);
            }
            YSTAMP(2);
            __builtin_amdgcn_wave_barrier();
            // ---- touched words -> list ----
            uint32_t ntouch = 0;
            YDUP(3) for (uint32_t i0 = (ntouch = 0u); i0 < nrw; i0 += 64) {
                const uint32_t i = i0 + lane;
                const bool hit = i < nrw && s_acc[i] != 0ull;
                const unsigned long long m = __ballot(hit);
                if (hit) s_list[ntouch + lanes_below(m)] = (uint16_t)i;
                ntouch += (uint32_t)__popcll(m);
            }
            __builtin_amdgcn_wave_barrier();
            YSTAMP(3);
            // ---- dedup against the seen list (or, an overflowed list -- rare -- the dense seen
            //      words; its own instantiation, so no other node waits on those loads); the
            //      staying tiles' slot entries and new list entries, positions by one wave scan ----
            reinterpret_cast<uint32_t*>(s_out)[lane] = 0xffffffffu;  // slot staging: tombstones
            __builtin_amdgcn_wave_barrier();
            uint32_t cnt = 0;            // new bits (this lane)
            uint32_t slot_total = 0;     // slot entries (uniform)
            uint32_t total = 1u + kept;  // next free entry of s_lst (uniform)
            auto dedup = [&](auto lovf_c) {
                constexpr bool LO = decltype(lovf_c)::value;
                for (uint32_t t0 = 0; t0 < ntouch; t0 += 64) {
                    const uint32_t t = t0 + lane;
                    const bool valid = t < ntouch;
                    const uint32_t i = valid ? s_list[t] : 0u;
                    const YoungTile yt = s_yt[i >> 4];
                    const uint32_t w = yt.tile * 16u + (i & 15u);
                    uint64_t x = 0ull, xe = 0ull;
                    if (valid) {
                        const uint32_t f = s_wf[i];
                        uint64_t sv = 0ull;
                        if constexpr (LO) sv = a.seen[v * stride + w];
                        // (a list holds every bit of a seen group: the accumulator has none of them)
                        x = s_acc[i] & ~sv;
                        if (f & WF_KEEP) x &= a.ctl[w].keep;  // (loaded and used in the branch)
                        if (f & WF_GROUP) x = group_fix(x, sv, a.ctl[w].gmask, a.ctl[w].gstart);
                        if constexpr (LO) {
                            if (x) a.seen[v * stride + w] = sv | x;
                        }
                        if (a.snap && (f & WF_SNAP)) snap_local += (unsigned long long)__popcll(x & a.ctl[w].snap);
                        s_acc[i] = x;  // the node's new bits, for the outputs below
                        if constexpr (!LO) xe = (f & WF_GROUP) ? group_expand(x, a.ctl[w].gmask, a.ctl[w].gstart) : x;
                    }
                    cnt += (uint32_t)__popcll(x);
                    if constexpr (LO) {
                        t_srd += wave_count(valid);
                        t_swr += wave_count(x != 0ull);
                    }
                    const bool stay = (yt.flags & YT_WRITE) != 0u;
                    const uint32_t cs = stay ? (uint32_t)__popcll(x) : 0u;
                    const uint64_t xl = stay ? xe : 0ull;
                    const uint32_t cl = (uint32_t)__popcll(xl);
                    if (__ballot((cs | cl) != 0u)) {  // (uniform)
                        const uint32_t pk = (cl << 16) | cs, incl = wave_incl_scan(pk), ex = incl - pk;
                        uint32_t ps = 1u + slot_total + (ex & 0xffffu), pl = total + (ex >> 16);
                        const uint32_t tot = lane_read(incl, 63u);
                        // (uniform) every lane's list bits are its slot bits (no id group among the
                        // words): one pass writes both entries, the list's at a uniform offset
                        const bool same = !LO && !__ballot(xl != (cs ? x : 0ull));
                        const uint32_t dl = total - 1u - slot_total;
                        slot_total += tot & 0xffffu;
                        total += tot >> 16;
                        if (same) {
                            const uint32_t sb = ((uint32_t)yt.w_idx << 10) | ((i & 15u) << 6);
                            const uint32_t lb = ((uint32_t)yt.yid << 10) | ((i & 15u) << 6);
                            for (uint64_t m = xl; m; m &= m - 1ull, ps++) {
                                const uint32_t bit = (uint32_t)__builtin_ctzll(m);
                                if (ps < kSlotU16) s_out[ps] = (uint16_t)(sb | bit);
                                if (ps + dl < kListU16) s_lst[ps + dl] = (uint16_t)(lb | bit);
                            }
                            continue;
                        }
                        for (uint64_t m = cs ? x : 0ull; m; m &= m - 1ull, ps++)
                            if (ps < kSlotU16)
                                s_out[ps] = (uint16_t)(((uint32_t)yt.w_idx << 10) | ((i & 15u) << 6) | (uint32_t)__builtin_ctzll(m));
                        for (uint64_t m = xl; m; m &= m - 1ull, pl++)
                            if (pl < kListU16)
                                s_lst[pl] = (uint16_t)(((uint32_t)yt.yid << 10) | ((i & 15u) << 6) | (uint32_t)__builtin_ctzll(m));
                    }
                }
            };
#if YOUNG_DUP
            const uint32_t ydc = cnt, yds = slot_total, ydt = total;
#endif
            YDUP(4) {
#if YOUNG_DUP
                cnt = ydc;  // (a repeated pass starts from the same state: same outputs)
                slot_total = yds;
                total = ydt;
#endif
                if (lovf)
                    dedup(std::true_type{});
                else
                    dedup(std::false_type{});
            }
            const uint32_t lcount = total - 1u;
            const bool lspill = !lovf && lcount > a.list_cap;  // (uniform) the list overflows now
            __builtin_amdgcn_wave_barrier();
            YSTAMP(4);
            cid_cur = with_hint(cid_next, h_next);  // (arrived long ago: the wait is before the stores)
            const int32_t rv = rv_cur;
            rv_cur = rv_next;
            // ---- output: the slot (staged above; an overflowed slot's entries are a subset of its
            //      dense rows), whole lines (no partial-line writes; unused entries are tombstones:
            //      readers scatter whole lines), dense rows (overflowed / leaving the young set) ----
            const bool overflow = slot_total > a.cap;
            uint16_t* out = a.slot_next + v * kSlotU16;
            if (lane == 0) s_out[0] = (uint16_t)(overflow ? kSlotOverflow : slot_total);
            __builtin_amdgcn_wave_barrier();
            YDUP(5) {
                const uint32_t lines = (!overflow && slot_total > 63u) ? 2u : 1u;
                if (lane < 8u * lines)
                    *reinterpret_cast<ulonglong2*>(out + lane * 8u) = *reinterpret_cast<const ulonglong2*>(s_out + lane * 8u);
                t_slw += lines;
                // announce a second line to the readers of the next tick -- and, sparse_wr, any
                // non-empty slot (an overflowed one too: its readers must see the header)
                if (lines == 2u || (a.sparse_wr && slot_total > 0u)) {
                    const uint8_t hv = (uint8_t)(lines == 2u ? a.stamp_next : a.stamp1_next);
                    if (rv >= 0) a.hint_next[rv] = hv;  // (the first 64 peers)
                    for (int32_t j = beg + 64 + (int32_t)lane; j < end; j += 64) {
                        const int32_t r = a.rev[j];
                        if (r >= 0) a.hint_next[r] = hv;
                    }
                }
            }
            YSTAMP(5);
            // dense rows: the leaving tiles (lv) always; every position if overflowed (leaving and
            // write-sparse tiles get rows)
            const uint32_t ndense = overflow ? a.ny : a.nt;
            unsigned long long nzw = 0ull;
            uint32_t nz_tw = 0xffffffffu;
            YDUP(6) for (uint32_t q0 = 0; q0 < ndense; q0 += 4) {
                const uint32_t qi = q0 + (lane >> 4), word = lane & 15u;
                const bool in = qi < ndense;
                const uint32_t q = !in ? 0u : overflow ? qi : (uint32_t)s_lv[qi];
                const YoungTile yt = s_yt[q];
                const bool leaving = in && (yt.flags & (YT_READ | YT_WRITE)) == YT_READ;  // (YT_DW or not)
                const bool dense_out = leaving || (in && (yt.flags & YT_WRITE));
                const uint64_t x = (in && q < a.nr) ? s_acc[q * 16u + word] : 0ull;
                const unsigned long long m = __ballot(in && x != 0ull);
                const bool tany = ((m >> (lane & ~15u)) & 0xffffull) != 0ull;
                // overflowed nodes write every write-sparse row (readers check no occupancy)
                const bool wr = dense_out && (tany || !leaving || (yt.flags & YT_DW));
                if (wr) a.Fnext[v * stride + yt.tile * 16u + word] = x;
                t_rw += wave_count(wr && word == 0u);
                if (leaving && tany && word == 0u) {
                    const uint32_t tw = yt.tile >> 6;
                    if (nz_tw != tw && nz_tw != 0xffffffffu) {
                        atomicOr(&a.nz_next[v * a.ntw + nz_tw], nzw);
                        nzw = 0ull;
                    }
                    nz_tw = tw;
                    nzw |= 1ull << (yt.tile & 63u);
                }
            }
            if (nzw) atomicOr(&a.nz_next[v * a.ntw + nz_tw], nzw);
            __builtin_amdgcn_wave_barrier();
            YSTAMP(6);
            // ---- seen rows materialised from the list: the tiles leaving the young set, or (the
            //      list overflows now) every young position; whole 128-B lines ----
            if (!lovf) {
                const uint32_t nm = lspill ? a.ny : a.nt;
                // (1) this tick's new bits stay single bits in the rows (k_births tests an id group
                //     against seen & ~arrivals: a whole group there would block a same-tick own
                //     generation that wins over the arrival); the old entries hold whole groups
                // (2) the old entries of those tiles
#pragma unroll
                for (uint32_t j = 0; j < 2u; j++) {
                    const uint32_t e = lentry(j);
                    const uint32_t qp = e == kSlotTomb ? 0xffu : s_ymap[e >> 10];
                    if (qp >= a.nr) continue;
                    const bool leaving = (s_yt[qp].flags & (YT_READ | YT_WRITE)) == YT_READ;
                    if (lspill || leaving)
                        atomicOr(reinterpret_cast<uint32_t*>(s_acc + qp * 16u + ((e >> 6) & 15u)) + ((e >> 5) & 1u),
                                 1u << (e & 31u));
                }
                __builtin_amdgcn_wave_barrier();
                // (3) write the rows (fresh positions: zeros), (4) reset their accumulator words
                for (uint32_t q0 = 0; q0 < nm; q0 += 4) {
                    const uint32_t qi = q0 + (lane >> 4), word = lane & 15u;
                    const uint32_t q = qi >= nm ? 0xffffffffu : lspill ? qi : (uint32_t)s_lv[qi];
                    if (q != 0xffffffffu && s_yt[q].flags) {
                        const uint64_t x = q < a.nr ? s_acc[q * 16u + word] : 0ull;
                        a.seen[v * stride + s_yt[q].tile * 16u + word] = x;
                        if (q < a.nr) s_acc[q * 16u + word] = 0ull;
                    }
                    t_mat += wave_count(q != 0xffffffffu && s_yt[q].flags && word == 0u);
                }
            }
            // ---- the new seen list: whole lines; an overflow marks the header ----
            YDUP(9) if (!lovf) {
                if (lane == 0) s_lst[0] = (uint16_t)(lspill ? kListOverflow : list_header(kept, lcount));
                __builtin_amdgcn_wave_barrier();
                const uint32_t lines = (!lspill && lcount > 63u) ? 2u : 1u;
                if (lane < 8u * lines)
                    *reinterpret_cast<ulonglong2*>(a.list + v * kListU16 + lane * 8u) =
                        *reinterpret_cast<const ulonglong2*>(s_lst + lane * 8u);
                t_lw += lines;
            }
            // ---- reset the touched accumulator words, counters ----
            YDUP(9) for (uint32_t t = lane; t < ntouch; t += 64) s_acc[s_list[t]] = 0ull;
            __builtin_amdgcn_wave_barrier();
            // fresh write-sparse tiles [nr, ny) of a node whose list overflowed (earlier): clear
            // their dense seen words (stale from the tiles' previous use; k_births sets this tick's
            // own-generation bits after this kernel).  A list node's fresh rows are written whole
            // when they leave the young set.
            if (lovf)
                for (uint32_t q0 = a.nr; q0 < a.ny; q0 += 4) {
                    const uint32_t qq = q0 + (lane >> 4);
                    if (qq < a.ny) a.seen[v * stride + s_yt[qq].tile * 16u + (lane & 15u)] = 0ull;
                    t_mat += wave_count(qq < a.ny && (lane & 15u) == 0u);
                }
            const uint32_t c = wave_sum32(cnt);
            if (lane == 0 && c) atomicAdd(&a.recv[v], c);  // no-return: nothing waits (sent: derived)
            YSTAMP(7);
            jn = jnext;
        }
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane_id == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
#ifdef YOUNG_STAMPS
    if (a.acct && lane_id == 0)
        for (int k = 0; k < 8; k++) acct_add(a.acct, 22u + (uint32_t)k, (unsigned long long)ycyc[k]);
#endif
    if (a.acct && lane_id == 0) {
        const uint32_t tv[11] = {t_sl, t_col, t_fb, t_srd, t_swr, t_rw, t_slw, t_miss, t_lr, t_lw, t_mat};
        const uint32_t slot_of[11] = {8, 9, 10, 11, 12, 13, 14, 15, 17, 18, 19};
#pragma unroll
        for (int q = 0; q < 11; q++)
            if (tv[q]) acct_add(a.acct, slot_of[q], (unsigned long long)tv[q]);
    }
}

// The idle-node pass of a `fast` tick (YoungArgs::fast), one lane per node, before k_pull_young on
// its stream: a node with work has a peer whose slot is stamped (its entries' hint bytes, 4 at a
// time) or an overflowed seen list while fresh tiles need clearing (k_pull_young's walk does that);
// every other node gets an empty slot and its list header's this-tick part folded into `kept`
// (k_births tests id groups against entries [1, kept] only).  Writes each chunk's work mask.
__global__ __launch_bounds__(256) void k_young_idle(YoungArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nchunks = ((uint64_t)a.n - a.v0 + 63u) / 64u;
    uint32_t t_lw = 0, t_idle = 0;
    for (uint64_t ch = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6); ch < nchunks; ch += (uint64_t)gridDim.x * 4u) {
        const uint64_t c0 = a.v0 + ch * 64u;
        const uint32_t cnt_nodes = (uint32_t)min<uint64_t>(64u, a.n - c0);
        const uint64_t v = c0 + lane;
        bool w = false;
        uint32_t lh = kListOverflow;
        if (lane < cnt_nodes) {
            if (a.nr) {  // some peer's slot is stamped (the hint bytes of this node's entries)
                const int32_t b = (int32_t)a.rowptr[v], e = (int32_t)a.rowptr[v + 1];
                const uint32_t p1 = a.stamp1_cur * 0x01010101u, p2 = a.stamp_cur * 0x01010101u;
                for (int32_t q = b & ~3; q < e; q += 4) {
                    const uint32_t x = *reinterpret_cast<const uint32_t*>(a.hint_cur + q);
                    uint32_t valid = 0xffffffffu;  // (the bytes inside [b, e))
                    if (q < b) valid <<= 8 * (b - q);
                    if (q + 4 > e) valid &= 0xffffffffu >> (8 * (q + 4 - e));
                    // a zero byte of x ^ stamp, by the borrow test (a false hit is only work)
                    const uint32_t z1 = x ^ p1, z2 = x ^ p2;
                    if ((((z1 - 0x01010101u) & ~z1) | ((z2 - 0x01010101u) & ~z2)) & 0x80808080u & valid) {
                        w = true;
                        break;
                    }
                }
            }
            lh = a.list[v * kListU16];
            if (lh == kListOverflow && a.ny > a.nr) w = true;  // (its fresh tiles' seen words)
        }
        const unsigned long long work = __ballot(w);
        if (lane == 0) a.work[ch] = work;
        if (lane < cnt_nodes && !w && lh != kListOverflow && (lh >> 7) != (lh & 127u)) {
            a.list[v * kListU16] = (uint16_t)list_header(lh & 127u, lh & 127u);
            t_lw++;
        }
#pragma unroll
        for (uint32_t i = 0; i < 8u; i++) {
            const uint32_t j = i * 8u + (lane >> 3);
            if (j < cnt_nodes && !((work >> j) & 1ull)) {
                ulonglong2 x = make_ulonglong2(~0ull, ~0ull);  // tombstones
                if ((lane & 7u) == 0u) x.x = ~0ull << 16;      // (entry 0: the header, 0)
                *reinterpret_cast<ulonglong2*>(a.slot_next + (c0 + j) * kSlotU16 + (lane & 7u) * 8u) = x;
            }
        }
        t_idle += cnt_nodes - (uint32_t)__popcll(work);
    }
    // idle nodes' slot lines written and header lines read (acct 14, 17), headers rewritten (18)
    const uint32_t lw = wave_sum32(t_lw);
    if (a.acct && lane == 0) {
        if (t_idle) {
            acct_add(a.acct, 14u, (unsigned long long)t_idle);
            acct_add(a.acct, 17u, (unsigned long long)t_idle);
        }
        if (lw) acct_add(a.acct, 18u, (unsigned long long)lw);
    }
}
