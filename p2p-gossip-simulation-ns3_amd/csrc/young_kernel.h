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
// Per node (one wave): gather the peers' slots (8 lanes x 16 B per peer, 32 peers in flight) and
// scatter their entries into a per-wave LDS accumulator of the young words; then dedup against
// the own seen words that got a bit (the same WordCtl masks as k_pull: clear, keep, id groups,
// snapshot), counters, and the output slot (wave prefix sum of the entry counts).
#pragma once

constexpr uint32_t kSlotU16 = 128;           // 256 B per node per frontier buffer
constexpr uint32_t kSlotOverflow = 0xffffu;  // header: the node's dense rows are valid
constexpr uint32_t kSlotTomb = 0xffffu;      // entry: removed (id-group birth beat an arrival)
constexpr uint32_t kYoungMax = 40;           // tiles per launch (LDS: 10 KiB per wave at 40)
constexpr uint32_t kYoungWriteMax = 34;      // write-sparse tiles per tick (w_idx < 34 <= 62)
constexpr int kYoungWpl = (int)(kYoungMax * 16 / 64);  // young words per lane (10)
constexpr int kYoungQ = 3;  // slot-line loads in flight per node: 24 peers (C4: P(deg > 24) ~ 2 %)
enum : uint32_t { YT_READ = 1u, YT_WRITE = 2u };

struct YoungTile {
    uint32_t tile;
    uint8_t flags;  // YT_READ: F_cur holds this tile in slots; YT_WRITE: F_next goes to slots
    uint8_t r_idx;  // w_idx of this tile in F_cur's entries (YT_READ)
    uint8_t w_idx;  // index written into F_next's entries (YT_WRITE)
    uint8_t pad;
};

struct YoungArgs {
    const int64_t* rowptr;
    const int32_t* col;
    const uint32_t* deg;
    const uint64_t* Fcur;
    uint64_t* Fnext;
    uint64_t* seen;
    const uint16_t* slot_cur;
    uint16_t* slot_next;
    const WordCtl* ctl;
    const uint8_t* wflags;
    uint32_t* recv;
    uint64_t* sent;
    unsigned long long* live;
    const unsigned long long* live_prev;  // nullable: all live
    unsigned long long* snap;             // nullable
    unsigned long long* acct;             // nullable
    unsigned long long* nz_next;
    uint32_t ntw;
    const YoungTile* yt;
    uint32_t ny;
    const uint8_t* rmap;  // [64] w_idx of F_cur entries -> position in yt (0xff: not read)
    uint32_t n, v0, stride, cap;
};

__host__ __device__ constexpr size_t young_lds_bytes(uint32_t ny) {
    // s_new + 4 waves x 2 accumulators (8 B per word each), tiles, word flags, rmap
    return (size_t)ny * 16u * 8u * 9u + (size_t)ny * sizeof(YoungTile) + (size_t)ny * 16u + 64u;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t lane) {
    uint32_t s = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)s, off, 64);
        if (lane >= (uint32_t)off) s += y;
    }
    return s - x;
}

// Entry j (0..7) of a lane's 16-B piece of a slot line.
__device__ __forceinline__ uint32_t slot_entry(const ulonglong2& q, int j) {
    const uint64_t word = j < 4 ? q.x : q.y;
    return (uint32_t)(word >> (16 * (j & 3))) & 0xffffu;
}

// Pipeline (one wave, 64 consecutive nodes per chunk, like k_pull): in the step of node k the
// wave issues the slot lines of node k+1 and the peer ids of node k+2, scatters node k's entries
// into LDS accumulator k&1 and issues node k's own seen words, then finishes node k-1 (dedup,
// seen, counters, output) from accumulator (k-1)&1 and the seen words that arrived meanwhile.
__global__ __launch_bounds__(256, 3) void k_pull_young(YoungArgs a) {
    extern __shared__ unsigned long long smem[];
    const uint32_t nw = a.ny * 16u;
    unsigned long long* s_new = smem;
    unsigned long long* s_accw = smem + nw + (threadIdx.x >> 6) * 2u * nw;  // this wave's 2 buffers
    YoungTile* s_yt = reinterpret_cast<YoungTile*>(smem + 9u * nw);
    uint8_t* s_wf = reinterpret_cast<uint8_t*>(s_yt + a.ny);
    uint8_t* s_rmap = s_wf + nw;
    for (uint32_t i = threadIdx.x; i < a.ny; i += 256) s_yt[i] = a.yt[i];
    if (threadIdx.x < 64) s_rmap[threadIdx.x] = a.rmap[threadIdx.x];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nw; i += 256) {
        s_new[i] = 0ull;
        s_wf[i] = a.wflags[s_yt[i >> 4].tile * 16u + (i & 15u)];
    }
    for (uint32_t i = threadIdx.x & 63u; i < 2u * nw; i += 64) s_accw[i] = 0ull;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t stride = a.stride;
    unsigned long long snap_local = 0ull;
    // traffic (wave-uniform): slot lines, peer ids, dense fallback rows, seen r/w, slot/row writes
    uint32_t t_sl = 0, t_col = 0, t_fb = 0, t_srd = 0, t_swr = 0, t_rw = 0, t_slw = 0;

    auto scatter = [&](unsigned long long* acc, uint32_t e) {
        if (e == kSlotTomb) return;
        const uint32_t pos = s_rmap[e >> 10];
        if (pos == 0xffu) return;
        const uint32_t b = e & 1023u;
        atomicOr(&acc[pos * 16u + (b >> 6)], 1ull << (b & 63u));
    };
    // slot first lines of the peers pb .. pb+8*kYoungQ-1 of a 64-peer id vector (8 lanes x 16 B
    // per peer)
    auto load_lines = [&](uint32_t cid, uint32_t pb, ulonglong2* q) {
#pragma unroll
        for (int k = 0; k < kYoungQ; k++) {
            const uint32_t p = pb + (uint32_t)k * 8u + (lane >> 3);
            const uint32_t u = (uint32_t)__shfl((int)cid, (int)(p & 63u), 64);
            q[k] = make_ulonglong2(0ull, 0ull);
            if (p < 64u && u != 0xffffffffu)
                q[k] = *reinterpret_cast<const ulonglong2*>(a.slot_cur + (uint64_t)u * kSlotU16 + (lane & 7u) * 8u);
        }
    };
    // scatter 8*kYoungQ peers' first lines; second lines and overflowed peers inline (rare)
    auto consume_lines = [&](unsigned long long* acc, uint32_t cid, uint32_t pb, const ulonglong2* q) {
        unsigned long long need2 = 0ull, ovf = 0ull;
#pragma unroll
        for (int k = 0; k < kYoungQ; k++) {
            const uint32_t p = pb + (uint32_t)k * 8u + (lane >> 3);
            const bool valid = p < 64u && (uint32_t)__shfl((int)cid, (int)(p & 63u), 64) != 0xffffffffu;
            const uint32_t hdr = (uint32_t)__shfl((int)(q[k].x & 0xffffull), (int)(lane & ~7u), 64);
            t_sl += wave_count(valid && (lane & 7u) == 0u);
            if (valid && hdr != kSlotOverflow) {
                const uint32_t lim = min(hdr, 63u);
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const uint32_t pos = (lane & 7u) * 8u + (uint32_t)j;
                    if (pos >= 1u && pos <= lim) scatter(acc, slot_entry(q[k], j));
                }
            }
            const bool lead = (lane & 7u) == 0u && valid;
            unsigned long long m2 = __ballot(lead && hdr != kSlotOverflow && hdr > 63u);
            unsigned long long mo = __ballot(lead && hdr == kSlotOverflow);
            while (m2) {
                const int L = __builtin_ctzll(m2);
                m2 &= m2 - 1ull;
                need2 |= 1ull << ((pb + (uint32_t)k * 8u + (uint32_t)L / 8u) & 63u);
            }
            while (mo) {
                const int L = __builtin_ctzll(mo);
                mo &= mo - 1ull;
                ovf |= 1ull << ((pb + (uint32_t)k * 8u + (uint32_t)L / 8u) & 63u);
            }
        }
        while (need2) {  // entries 64..127: one 8-lane group
            const int p = __builtin_ctzll(need2);
            need2 &= need2 - 1ull;
            const uint32_t u = (uint32_t)__shfl((int)cid, p, 64);
            t_sl++;
            if (lane < 8u) {
                const uint16_t* sl = a.slot_cur + (uint64_t)u * kSlotU16;
                const uint32_t hdr = sl[0];
                const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(sl + 64u + lane * 8u);
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (64u + lane * 8u + (uint32_t)j <= hdr) scatter(acc, slot_entry(x, j));
            }
        }
        while (ovf) {  // overflowed peers: their dense rows of every read-sparse tile
            const int p = __builtin_ctzll(ovf);
            ovf &= ovf - 1ull;
            const uint32_t u = (uint32_t)__shfl((int)cid, p, 64);
            for (uint32_t i = lane; i < nw; i += 64) {
                const YoungTile yt = s_yt[i >> 4];
                if (!(yt.flags & YT_READ)) continue;
                const uint64_t x = a.Fcur[(uint64_t)u * stride + yt.tile * 16u + (i & 15u)];
                if (x) acc[i] |= x;  // this lane owns word i
            }
            t_fb += (uint32_t)a.ny;
        }
    };

    for (uint64_t c0 = a.v0 + wave * 64u; c0 < a.n; c0 += nwaves * 64u) {
        const uint32_t cnt_nodes = (uint32_t)min<uint64_t>(64u, a.n - c0);
        const int64_t rp = a.rowptr[c0 + min(lane, cnt_nodes)];
        const int64_t rp_end = a.rowptr[c0 + cnt_nodes];
        auto nbeg = [&](uint32_t j) -> int32_t { return __shfl((int)rp, (int)(j & 63u), 64); };
        auto nend = [&](uint32_t j) -> int32_t {
            const int32_t nx = __shfl((int)rp, (int)((j + 1u) & 63u), 64);
            return j + 1u < 64u ? nx : (int32_t)rp_end;
        };
        auto load_cid = [&](uint32_t j) -> uint32_t {  // lane p: peer p of node j (first 64)
            if (j >= cnt_nodes) return 0xffffffffu;
            const int32_t b = nbeg(j), e = nend(j);
            return (int32_t)lane < e - b ? (uint32_t)a.col[b + (int32_t)lane] : 0xffffffffu;
        };
        uint32_t cidA = load_cid(0u), cidB = load_cid(1u);
        ulonglong2 qA[kYoungQ];
        load_lines(cidA, 0u, qA);
        uint64_t svP[kYoungWpl];  // own seen words of the node being finished
#pragma unroll
        for (int j = 0; j < kYoungWpl; j++) svP[j] = 0ull;
        for (uint32_t k = 0; k <= cnt_nodes; k++) {
            unsigned long long* accK = s_accw + (k & 1u) * nw;
            unsigned long long* accP = s_accw + ((k + 1u) & 1u) * nw;
            uint64_t svK[kYoungWpl];
#pragma unroll
            for (int j = 0; j < kYoungWpl; j++) svK[j] = 0ull;
            if (k < cnt_nodes) {
                const uint64_t v = c0 + k;
                ulonglong2 qB[kYoungQ];
                load_lines(cidB, 0u, qB);  // node k+1 (invalid ids past the chunk: no loads)
                const uint32_t cidC = load_cid(k + 2u);
                // ---- gather node k ----
                const int32_t b = nbeg(k), e = nend(k);
                t_col += (uint32_t)(e - b);
                consume_lines(accK, cidA, 0u, qA);
                constexpr int32_t kPB = 8 * kYoungQ;
                if (e - b > kPB) {  // the rest of the first 64 peers, then 64-peer chunks (dense graphs)
                    ulonglong2 q2[kYoungQ];
                    for (uint32_t pb = kPB; pb < 64u; pb += kPB) {
                        load_lines(cidA, pb, q2);
                        consume_lines(accK, cidA, pb, q2);
                    }
                    for (int32_t cb = b + 64; cb < e; cb += 64) {
                        const uint32_t cid = cb + (int32_t)lane < e ? (uint32_t)a.col[cb + (int32_t)lane] : 0xffffffffu;
                        for (uint32_t pb = 0; pb < 64u; pb += kPB) {
                            load_lines(cid, pb, q2);
                            consume_lines(accK, cid, pb, q2);
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                // ---- own seen words of node k that can take a bit (in flight until k+1) ----
#pragma unroll
                for (int j = 0; j < kYoungWpl; j++) {
                    const uint32_t i = lane + 64u * (uint32_t)j;
                    if (i < nw && accK[i] && !(s_wf[i] & WF_CLEAR))
                        svK[j] = a.seen[v * stride + s_yt[i >> 4].tile * 16u + (i & 15u)];
                }
                cidA = cidB;
                cidB = cidC;
#pragma unroll
                for (int q = 0; q < kYoungQ; q++) qA[q] = qB[q];
            }
            if (k > 0) {
                // ---- finish node k-1: dedup, seen, counters ----
                const uint64_t v = c0 + k - 1u;
                uint64_t nwv[kYoungWpl];
                uint32_t cnt = 0, cnt_sp = 0;
#pragma unroll
                for (int j = 0; j < kYoungWpl; j++) {
                    nwv[j] = 0ull;
                    const uint32_t i = lane + 64u * (uint32_t)j;
                    if (i >= nw) continue;
                    const YoungTile yt = s_yt[i >> 4];
                    const uint32_t w = yt.tile * 16u + (i & 15u);
                    const uint32_t f = s_wf[i];
                    const uint64_t inc = accP[i];
                    const bool clear = (f & WF_CLEAR) != 0u;
                    if (inc || clear) {
                        const uint64_t sv = clear ? 0ull : svP[j];
                        const uint64_t keep = (f & WF_KEEP) ? a.ctl[w].keep : ~0ull;
                        uint64_t x = inc & ~sv & keep;
                        if (f & WF_GROUP) x = group_fix(x, sv, a.ctl[w].gmask, a.ctl[w].gstart);
                        if (x || clear) a.seen[v * stride + w] = sv | x;
                        nwv[j] = x;
                        cnt += (uint32_t)__popcll(x);
                        if (a.snap && (f & WF_SNAP)) snap_local += (unsigned long long)__popcll(x & a.ctl[w].snap);
                        if (x) atomicOr(&s_new[i], (unsigned long long)x);
                        if (yt.flags & YT_WRITE) cnt_sp += (uint32_t)__popcll(x);
                    }
                    t_srd += wave_count(inc != 0ull && !clear);
                    t_swr += wave_count(nwv[j] != 0ull || clear);
                    accP[i] = 0ull;  // ready for node k+1
                }
                // ---- output: slot entries, or dense rows (overflowed / leaving the young set) ----
                const uint32_t total = (uint32_t)wave_sum((unsigned long long)cnt_sp);
                const bool overflow = total > a.cap;
                uint16_t* out = a.slot_next + v * kSlotU16;
                if (!overflow) {
                    uint32_t pos = 1u + wave_excl_scan(cnt_sp, lane);
#pragma unroll
                    for (int j = 0; j < kYoungWpl; j++) {
                        const uint32_t i = lane + 64u * (uint32_t)j;
                        if (i >= nw) continue;
                        const YoungTile yt = s_yt[i >> 4];
                        if (!(yt.flags & YT_WRITE)) continue;
                        uint64_t x = nwv[j];
                        while (x) {
                            const uint32_t bb = (uint32_t)__builtin_ctzll(x);
                            x &= x - 1ull;
                            out[pos++] = (uint16_t)(((uint32_t)yt.w_idx << 10) | ((i & 15u) << 6) | bb);
                        }
                    }
                }
                if (lane == 0) out[0] = (uint16_t)(overflow ? kSlotOverflow : total);
                t_slw += 1u + (total > 63u && !overflow ? 1u : 0u);
                unsigned long long nzw = 0ull;  // occupancy bits of leaving tiles
                uint32_t nz_tw = 0xffffffffu;
#pragma unroll
                for (int j = 0; j < kYoungWpl; j++) {
                    const uint32_t i = lane + 64u * (uint32_t)j;
                    const bool in = i < nw;
                    const YoungTile yt = in ? s_yt[i >> 4] : YoungTile{0u, 0, 0, 0, 0};
                    const bool dense_out = in && (!(yt.flags & YT_WRITE) || overflow);
                    // 16 consecutive lanes hold one tile: any bit in the tile?
                    const unsigned long long m = __ballot(in && nwv[j] != 0ull);
                    const bool tany = ((m >> (lane & ~15u)) & 0xffffull) != 0ull;
                    // overflowed nodes write every write-sparse row (readers check no occupancy)
                    const bool wr = dense_out && (tany || ((yt.flags & YT_WRITE) != 0u));
                    if (wr) a.Fnext[v * stride + yt.tile * 16u + (i & 15u)] = nwv[j];
                    t_rw += wave_count(wr && (i & 15u) == 0u);
                    if (in && !(yt.flags & YT_WRITE) && tany && (i & 15u) == 0u) {
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
                const uint32_t c = (uint32_t)wave_sum((unsigned long long)cnt);
                if (lane == 0 && c) {
                    a.recv[v] += c;
                    a.sent[v] += (uint64_t)c * a.deg[v];
                }
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < kYoungWpl; j++) svP[j] = svK[j];
        }
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.acct && lane == 0) {
        const uint32_t tv[7] = {t_sl, t_col, t_fb, t_srd, t_swr, t_rw, t_slw};
#pragma unroll
        for (int q = 0; q < 7; q++)
            if (tv[q]) atomicAdd(&a.acct[8 + q], (unsigned long long)tv[q]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nw; i += 256) {
        const unsigned long long x = s_new[i];
        if (x) atomicOr(&a.live[s_yt[i >> 4].tile * 16u + (i & 15u)], x);
    }
}
