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
constexpr uint32_t kYoungMax = 48;           // tiles per launch (LDS: 6 KiB per wave at 48)
constexpr uint32_t kYoungWriteMax = 40;      // write-sparse tiles per tick (w_idx < 40 <= 62)
constexpr int kYoungWpl = (int)(kYoungMax * 16 / 64);  // young words per lane (12)
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
    // s_lp, s_new, 4 wave accumulators (8 B per word each), tiles, word flags, rmap
    return (size_t)ny * 16u * 8u * 6u + (size_t)ny * sizeof(YoungTile) + (size_t)ny * 16u + 64u;
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

__global__ __launch_bounds__(256) void k_pull_young(YoungArgs a) {
    extern __shared__ unsigned long long smem[];
    const uint32_t nw = a.ny * 16u;
    unsigned long long* s_lp = smem;
    unsigned long long* s_new = smem + nw;
    unsigned long long* s_acc = smem + 2u * nw + (threadIdx.x >> 6) * nw;
    YoungTile* s_yt = reinterpret_cast<YoungTile*>(smem + 6u * nw);
    uint8_t* s_wf = reinterpret_cast<uint8_t*>(s_yt + a.ny);
    uint8_t* s_rmap = s_wf + nw;
    for (uint32_t i = threadIdx.x; i < a.ny; i += 256) s_yt[i] = a.yt[i];
    if (threadIdx.x < 64) s_rmap[threadIdx.x] = a.rmap[threadIdx.x];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nw; i += 256) {
        const uint32_t w = s_yt[i >> 4].tile * 16u + (i & 15u);
        s_lp[i] = a.live_prev ? a.live_prev[w] : ~0ull;
        s_new[i] = 0ull;
        s_wf[i] = a.wflags[w];
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * 4u;
    const uint64_t stride = a.stride;
    unsigned long long snap_local = 0ull;
    // traffic (wave-uniform): slot lines, peer ids, dense fallback rows, seen r/w, slot/row writes
    uint32_t t_sl = 0, t_col = 0, t_fb = 0, t_srd = 0, t_swr = 0, t_rw = 0, t_slw = 0;

    auto scatter = [&](uint32_t e) {
        if (e == kSlotTomb) return;
        const uint32_t pos = s_rmap[e >> 10];
        if (pos == 0xffu) return;
        const uint32_t b = e & 1023u;
        atomicOr(&s_acc[pos * 16u + (b >> 6)], 1ull << (b & 63u));
    };

    for (uint64_t v = a.v0 + wave; v < a.n; v += nwaves) {
        for (uint32_t i = lane; i < nw; i += 64) s_acc[i] = 0ull;
        __builtin_amdgcn_wave_barrier();
        const int64_t beg = a.rowptr[v], end = a.rowptr[v + 1];
        for (int64_t cb = beg; cb < end; cb += 64) {
            const int np = (int)min<int64_t>(64, end - cb);
            const uint32_t myu = (int)lane < np ? (uint32_t)a.col[cb + lane] : 0u;
            t_col += (uint32_t)np;
            unsigned long long need2 = 0ull, ovf = 0ull;  // peers (bit p), wave-uniform
            for (int pb = 0; pb < np; pb += 32) {
                ulonglong2 q[4];
                int pk[4];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    pk[k] = pb + k * 8 + (int)(lane >> 3);
                    const uint32_t u = (uint32_t)__shfl((int)myu, pk[k] & 63, 64);
                    q[k] = make_ulonglong2(0ull, 0ull);
                    if (pk[k] < np)
                        q[k] = *reinterpret_cast<const ulonglong2*>(a.slot_cur + (uint64_t)u * kSlotU16 + (lane & 7u) * 8u);
                }
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t hdr = (uint32_t)__shfl((int)(q[k].x & 0xffffull), (int)(lane & ~7u), 64);
                    const bool valid = pk[k] < np;
                    t_sl += wave_count(valid && (lane & 7u) == 0u);
                    if (valid && hdr != kSlotOverflow) {
                        const uint32_t lim = min(hdr, 63u);
#pragma unroll
                        for (int j = 0; j < 8; j++) {
                            const uint32_t pos = (lane & 7u) * 8u + (uint32_t)j;
                            const uint64_t word = j < 4 ? q[k].x : q[k].y;
                            const uint32_t e = (uint32_t)(word >> (16 * (j & 3))) & 0xffffu;
                            if (pos >= 1u && pos <= lim) scatter(e);
                        }
                    }
                    // per-peer flags from the peer's first lane
                    const bool lead = (lane & 7u) == 0u && valid;
                    unsigned long long m2 = __ballot(lead && hdr != kSlotOverflow && hdr > 63u);
                    unsigned long long mo = __ballot(lead && hdr == kSlotOverflow);
                    while (m2) {
                        const int L = __builtin_ctzll(m2);
                        m2 &= m2 - 1ull;
                        need2 |= 1ull << (pb + k * 8 + L / 8);
                    }
                    while (mo) {
                        const int L = __builtin_ctzll(mo);
                        mo &= mo - 1ull;
                        ovf |= 1ull << (pb + k * 8 + L / 8);
                    }
                }
            }
            // second slot lines (entries 64..127): one 8-lane group per peer
            while (need2) {
                const int p = __builtin_ctzll(need2);
                need2 &= need2 - 1ull;
                const uint32_t u = (uint32_t)__shfl((int)myu, p, 64);
                t_sl++;
                if (lane < 8u) {
                    const uint16_t* s = a.slot_cur + (uint64_t)u * kSlotU16;
                    const uint32_t hdr = s[0];
                    const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(s + 64u + lane * 8u);
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const uint32_t pos = 64u + lane * 8u + (uint32_t)j;
                        const uint64_t word = j < 4 ? x.x : x.y;
                        const uint32_t e = (uint32_t)(word >> (16 * (j & 3))) & 0xffffu;
                        if (pos <= hdr) scatter(e);
                    }
                }
            }
            // overflowed peers: their dense rows of every read-sparse tile
            while (ovf) {
                const int p = __builtin_ctzll(ovf);
                ovf &= ovf - 1ull;
                const uint32_t u = (uint32_t)__shfl((int)myu, p, 64);
                for (uint32_t i = lane; i < nw; i += 64) {
                    const YoungTile yt = s_yt[i >> 4];
                    if (!(yt.flags & YT_READ)) continue;
                    const uint64_t x = a.Fcur[(uint64_t)u * stride + yt.tile * 16u + (i & 15u)];
                    if (x) s_acc[i] |= x;  // this lane owns word i of the accumulator
                }
                t_fb += (uint32_t)a.ny;  // rows touched (at most one line per young tile)
            }
        }
        __builtin_amdgcn_wave_barrier();
        // ---- dedup, seen, counters ----
        uint64_t nwv[kYoungWpl];
        uint32_t cnt = 0, cnt_sp = 0;
#pragma unroll
        for (int k = 0; k < kYoungWpl; k++) {
            nwv[k] = 0ull;
            const uint32_t i = lane + 64u * (uint32_t)k;
            if (i >= nw) continue;
            const YoungTile yt = s_yt[i >> 4];
            const uint32_t w = yt.tile * 16u + (i & 15u);
            const uint32_t f = s_wf[i];
            const uint64_t inc = s_acc[i] & s_lp[i];
            const bool clear = (f & WF_CLEAR) != 0u;
            if (inc || clear) {
                uint64_t* sp = a.seen + v * stride + w;
                const uint64_t sv = clear ? 0ull : *sp;
                const uint64_t keep = (f & WF_KEEP) ? a.ctl[w].keep : ~0ull;
                uint64_t x = inc & ~sv & keep;
                if (f & WF_GROUP) x = group_fix(x, sv, a.ctl[w].gmask, a.ctl[w].gstart);
                if (x || clear) *sp = sv | x;
                nwv[k] = x;
                cnt += (uint32_t)__popcll(x);
                if (a.snap && (f & WF_SNAP)) snap_local += (unsigned long long)__popcll(x & a.ctl[w].snap);
                if (x) atomicOr(&s_new[i], (unsigned long long)x);
                if (yt.flags & YT_WRITE) cnt_sp += (uint32_t)__popcll(x);
            }
            t_srd += wave_count(inc != 0ull && !clear);
            t_swr += wave_count(nwv[k] != 0ull || clear);
        }
        // ---- output: slot entries, or dense rows when overflowed / leaving the young set ----
        const uint32_t total = (uint32_t)wave_sum((unsigned long long)cnt_sp);
        const bool overflow = total > a.cap;
        uint16_t* out = a.slot_next + v * kSlotU16;
        if (!overflow) {
            uint32_t pos = 1u + wave_excl_scan(cnt_sp, lane);
#pragma unroll
            for (int k = 0; k < kYoungWpl; k++) {
                const uint32_t i = lane + 64u * (uint32_t)k;
                if (i >= nw) continue;
                const YoungTile yt = s_yt[i >> 4];
                if (!(yt.flags & YT_WRITE)) continue;
                uint64_t x = nwv[k];
                while (x) {
                    const uint32_t b = (uint32_t)__builtin_ctzll(x);
                    x &= x - 1ull;
                    out[pos++] = (uint16_t)(((uint32_t)yt.w_idx << 10) | ((i & 15u) << 6) | b);
                }
            }
        }
        if (lane == 0) out[0] = (uint16_t)(overflow ? kSlotOverflow : total);
        t_slw += 1u + (total > 63u && !overflow ? 1u : 0u);
        unsigned long long nzw = 0ull;  // occupancy bits of leaving tiles, nz word 0 ..
        uint32_t nz_tw = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < kYoungWpl; k++) {
            const uint32_t i = lane + 64u * (uint32_t)k;
            const bool in = i < nw;
            const YoungTile yt = in ? s_yt[i >> 4] : YoungTile{0u, 0, 0, 0, 0};
            const bool dense_out = in && (!(yt.flags & YT_WRITE) || overflow);
            // 16 consecutive lanes hold one tile: any bit in the tile?
            const unsigned long long m = __ballot(in && nwv[k] != 0ull);
            const bool tany = ((m >> (lane & ~15u)) & 0xffffull) != 0ull;
            // overflowed nodes write every write-sparse row (readers do not check occupancy)
            const bool wr = dense_out && (tany || ((yt.flags & YT_WRITE) != 0u));
            if (wr) a.Fnext[v * stride + yt.tile * 16u + (i & 15u)] = nwv[k];
            t_rw += wave_count(wr && (i & 15u) == 0u);
            if (in && !(yt.flags & YT_WRITE) && tany && (i & 15u) == 0u) {
                const uint32_t tw = yt.tile >> 6;
                // nz words: the young list is sorted by tile, so one lane meets few tw values
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
