// dense_kernel.h -- the dense-graph pull as an int8 MFMA contraction over bit-packed operands
// (GOSSIP_MODE_DENSE), included by engine.hip after pull_kernel.h.
//
// For p ~ 0.3 the per-tick gather of GossipShareToPeers (p2pnode.cc:127-153) is an adjacency x
// frontier product:
//     Inc[v][c] = sum_u A[v][u] * F[u][c]        A[v][u] = [u in peers(v)],  F = frontier bits
// and only Inc > 0 is needed (the pull dedups against seen).  Both operands stay bit-packed in
// HBM -- the adjacency as n_pad x n_pad bits, the frontier transposed to one bit row per share
// column (k_transpose) -- and are expanded to int8 in registers right before
// v_mfma_i32_32x32x32_i8, so the GEMM streams 1/8 of the bytes an int8 adjacency would.
//
// Expansion.  The MFMA contracts over 32 k per instruction; lane half h supplies 16 of them.  A
// 32-bit word X holding the bits of k = 32kc .. 32kc+31 becomes the 4 dwords
//     X & (0x01010101 << (4h + e)),  e = 0..3
// i.e. byte b of dword e is nonzero iff bit 8b+4h+e of X is set.  A and B use the same map, so
// the contraction is over the same k on both sides, and every product is a power of two
// (2^(2d), or (-128)^2 for d = 7): Inc is a positive sum of at most 16384 per k, exact in int32
// for n_pad < 131072 x 8, and Inc > 0 iff some peer u of v carries share c.  One v_and per
// 4 bytes -- 4 VALU per fragment, 24 per 8 MFMAs -- hides under the 32-cycle MFMA issue gaps.
//
// Operand maps (pinned on gfx950 by tools/mfma_probe.hip with exact integer data): lane l holds
// 16 int8 of A row (l&31) and of B column (l&31); any k order shared by A and B gives the same
// product; C/D: lane l, register g -> row (g&3) + 8(g>>2) + 4(l>>5), column l&31.
//
// Tiling: block = 8 waves (2 x 4), output tile 256 rows x 256 columns (4 frontier words), wave
// tile 128 x 64 = 4 x 2 MFMA tiles (128 accumulator registers).  K advances kStageK = 1024 (128 B
// of bits per row) per stage through double-buffered LDS (2 x 72 KB, rows padded to 144 B: 9r mod
// 16 is a permutation, so 16 lanes' ds_read_b128 hit distinct 16-B slots; 512-k stages with 80-B
// rows measured 3 % lower MFMA utilisation, twice the barriers).  One barrier per stage: the
// stage's bit loads are issued a stage ahead.  A stage whose frontier bits are all zero for the
// block's 256 columns is skipped (__syncthreads_or), so sparse frontiers cost only the loads.
// Blocks are mapped XCD-major: the 4 column tiles of one row block run on one XCD together, so
// the adjacency is fetched from HBM once per tick and re-read from that XCD's L2.
#pragma once

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

struct BitsArgs {
    const uint32_t* Ab;  // n_pad rows x kw words: bit (u & 31) of word (u >> 5) = [u in peers(v)]
    const uint32_t* FT;  // ncols rows x kw words: bit u of row c = bit c of the frontier row u
    unsigned long long* inc;              // n x stride incoming words (OR of Inc > 0)
    const unsigned long long* live_prev;  // nullable: per-word liveness of the frontier
    unsigned long long* acct;             // [5] += MAC ops x2 executed, [6] += tiles skipped
    uint32_t n, n_pad, kw, stride;
    uint32_t mb, nt, ksplit, total;  // row blocks, column tiles, K splits, mb*nt*ksplit
    uint32_t mb0;                    // first row block (row partition)
};

#ifndef DENSE_STAGE_K
#define DENSE_STAGE_K 1024  // 512: 0.478 / 0.554 MFMA util on C2 / C5, 1024: 0.494 / 0.568 (half the barriers; profiles/r02/dense_stage_ab.txt)
#endif
constexpr uint32_t kDenseTile = 256;               // rows / columns per block tile
constexpr uint32_t kStageK = DENSE_STAGE_K;        // k per LDS stage
constexpr uint32_t kStageQ = kStageK / 128u;       // 16-B pieces of a row per stage
constexpr uint32_t kStageRow = kStageK / 8u + 16u; // padded LDS row: the stage's bits + 16 B
constexpr uint32_t kDensePad = kStageK;            // n_pad multiple (tile and stage)
static_assert(kStageK % 512u == 0u && ((kStageRow / 16u) & 1u), "stage: odd 16-B row pitch");

// Frontier bitmap (node rows of share words) -> one bit row per share column.  A wave takes
// 64 nodes x one word and transposes the 64 x 64 bit block with ballots.
__global__ __launch_bounds__(256) void k_transpose(const uint64_t* __restrict__ F, uint32_t stride,
                                                   uint32_t n, uint32_t kw, uint32_t nwords,
                                                   const unsigned long long* live_prev,
                                                   const unsigned long long* __restrict__ nz,
                                                   uint32_t ntw, uint32_t* __restrict__ FT) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t chunk = blockIdx.x * 4u + wave_in_block();  // 64-node chunk
    const uint32_t w = blockIdx.y;
    if (w >= nwords || chunk * 64u >= kw * 32u) return;
    if (live_prev) {  // a 4-word column tile with no live word is skipped by the GEMM
        const uint32_t g = w & ~3u;
        if ((live_prev[g] | live_prev[g + 1] | live_prev[g + 2] | live_prev[g + 3]) == 0ull) return;
    }
    const uint32_t u = chunk * 64u + lane;
    // a tile row whose occupancy bit is clear holds stale bits: read as empty
    const bool occ = u < n && ((nz[(uint64_t)u * ntw + (w >> 10)] >> ((w >> 4) & 63u)) & 1ull);
    const uint64_t x = occ ? F[(uint64_t)u * stride + w] : 0ull;
    uint64_t keep = 0ull;
#pragma unroll
    for (int b = 0; b < 64; b++) {
        const unsigned long long m = __ballot((x >> b) & 1ull);
        if (lane == (uint32_t)b) keep = m;
    }
    // row c = 64w + lane; this chunk's 64 node bits are words 2*chunk, 2*chunk+1 of the row
    uint64_t* row = reinterpret_cast<uint64_t*>(FT + (uint64_t)(w * 64u + lane) * kw);
    row[chunk] = keep;
}

__device__ __forceinline__ v4i_t dense_expand(uint32_t x, const uint32_t (&m)[4]) {
    return v4i_t{(int)(x & m[0]), (int)(x & m[1]), (int)(x & m[2]), (int)(x & m[3])};
}

__global__ __launch_bounds__(512, 1) void k_dense_bits(BitsArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t S[2][2][kDenseTile * kStageRow];
    // XCD-major tile order: hardware places block b on XCD b % 8; tile T = xcd * per + b / 8
    const uint32_t per = (a.total + 7u) / 8u;
    const uint32_t T = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (T >= a.total) return;
    const uint32_t z = T % a.ksplit;
    const uint32_t nt = (T / a.ksplit) % a.nt;
    const uint32_t mblk = a.mb0 + T / (a.ksplit * a.nt);
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
    const uint32_t wm = wid >> 2, wn = wid & 3u;
    const uint32_t w0 = nt * 4u;
    if (a.live_prev) {
        const unsigned long long lv = a.live_prev[w0] | a.live_prev[w0 + 1] | a.live_prev[w0 + 2] |
                                      a.live_prev[w0 + 3];
        if (lv == 0ull) {
            if (t == 0 && a.acct) acct_add(a.acct, 6, 1ull);
            return;
        }
    }
    const uint32_t nst = a.n_pad / kStageK;
    const uint32_t sper = (nst + a.ksplit - 1u) / a.ksplit;
    const uint32_t sb = z * sper, se = min(nst, sb + sper);
    if (sb >= se) return;

    // loader: threads 0-255 stage adjacency rows, 256-511 frontier columns; 64 B each per stage
    const uint32_t op = t >> 8, lrow = t & 255u;
    const uint32_t* src = op == 0 ? a.Ab + (uint64_t)(mblk * kDenseTile + lrow) * a.kw
                                  : a.FT + (uint64_t)(nt * kDenseTile + lrow) * a.kw;
    uint4 r[kStageQ];
#pragma unroll
    for (uint32_t q = 0; q < kStageQ; q++)
        r[q] = *reinterpret_cast<const uint4*>(src + (uint64_t)sb * (kStageK / 32u) + 4u * q);

    const uint32_t h = lane >> 5, rr = lane & 31u;
    uint32_t msk[4];
#pragma unroll
    for (int e = 0; e < 4; e++) msk[e] = 0x01010101u << (4u * h + (uint32_t)e);
    v16i_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = v16i_t{0};

    uint32_t computed = 0;
    for (uint32_t s = sb; s < se; s++) {
        const uint32_t p = (s - sb) & 1u;
        uint8_t* wr = &S[p][op][lrow * kStageRow];
#pragma unroll
        for (uint32_t q = 0; q < kStageQ; q++) *reinterpret_cast<uint4*>(wr + 16u * q) = r[q];
        int bnz = 0;
        if (op == 1) {
            uint32_t o = 0u;
#pragma unroll
            for (uint32_t q = 0; q < kStageQ; q++) o |= r[q].x | r[q].y | r[q].z | r[q].w;
            bnz = o != 0u;
        }
        if (s + 1u < se) {
#pragma unroll
            for (uint32_t q = 0; q < kStageQ; q++)
                r[q] = *reinterpret_cast<const uint4*>(src + (uint64_t)(s + 1u) * (kStageK / 32u) + 4u * q);
        }
        if (!__syncthreads_or(bnz)) continue;  // no frontier bit in this k range: nothing to add
        computed++;
        const uint8_t* As = &S[p][0][0];
        const uint8_t* Bs = &S[p][1][0];
#pragma unroll
        for (uint32_t kq = 0; kq < kStageQ; kq++) {  // 128 k = 16 B of each row
            uint4 xa[4], xb[2];
#pragma unroll
            for (int i = 0; i < 4; i++)
                xa[i] = *reinterpret_cast<const uint4*>(As + (wm * 128u + i * 32u + rr) * kStageRow + kq * 16u);
#pragma unroll
            for (int j = 0; j < 2; j++)
                xb[j] = *reinterpret_cast<const uint4*>(Bs + (wn * 64u + j * 32u + rr) * kStageRow + kq * 16u);
#pragma unroll
            for (int kc = 0; kc < 4; kc++) {
                v4i_t af[4], bf[2];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t x = kc == 0 ? xa[i].x : kc == 1 ? xa[i].y : kc == 2 ? xa[i].z : xa[i].w;
                    af[i] = dense_expand(x, msk);
                }
#pragma unroll
                for (int j = 0; j < 2; j++) {
                    const uint32_t x = kc == 0 ? xb[j].x : kc == 1 ? xb[j].y : kc == 2 ? xb[j].z : xb[j].w;
                    bf[j] = dense_expand(x, msk);
                }
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++)
                        acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    if (t == 0 && a.acct && computed)
        acct_add(a.acct, 5, 2ull * kDenseTile * kDenseTile * kStageK * computed);
    if (computed == 0) return;
    // ---- epilogue: Inc > 0 -> one 64-bit word per row (wave ballots), OR into inc ----
    // lane l collects rows l (lo) and l + 64 (hi) of the wave's 128
    uint64_t lo = 0ull, hi = 0ull;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int g = 0; g < 16; g++) {
            const unsigned long long q0 = __ballot(acc[i][0][g] > 0);
            const unsigned long long q1 = __ballot(acc[i][1][g] > 0);
            const uint64_t h0 = (q0 & 0xffffffffull) | (q1 << 32);               // lane half 0 row
            const uint64_t h1 = (q0 >> 32) | (q1 & 0xffffffff00000000ull);       // 4 rows below
            const uint32_t row = (uint32_t)(i & 1) * 32u + (g & 3) + 8u * (g >> 2);
            if (i < 2) {
                if (lane == row) lo = h0;
                if (lane == row + 4u) lo = h1;
            } else {
                if (lane == row) hi = h0;
                if (lane == row + 4u) hi = h1;
            }
        }
    const uint64_t v = (uint64_t)mblk * kDenseTile + wm * 128u + lane;
    unsigned long long* ip = a.inc + v * a.stride + w0 + wn;
    if (lo && v < a.n) atomicOr(ip, (unsigned long long)lo);
    if (hi && v + 64u < a.n) atomicOr(ip + 64ull * a.stride, (unsigned long long)hi);
}

// ------------------------------------------------------------------------------------------
// k_dense_dedup -- the rest of the DENSE-mode pull after the contraction: for every node and
// live word, new = inc & ~seen & keep (+ group_fix), seen |= new, F_next = new, recv/sent +=
// popcount(new) (p2pnode.cc:155-165, 189), tile occupancy and liveness -- the same per-pair
// semantics as k_pull's incoming-word path, but laid out for the chip rather than for a gather:
// one node per wave step (lane = a 16-B word pair of a 128-word pass), the grid's waves striding
// over the engine's rows.  k_pull serves 64 nodes per wave because its peer-id / occupancy
// pipeline is per 64-node chunk; with nothing to gather that layout left a 4,096-node graph
// 64 waves for the whole chip (C2: 307 us per dispatch).  HBM-bound: per live pair 16 B of
// incoming words read (+ zeroed when non-zero), 16 B of seen read and written, 16 B of F_next
// written.  Liveness: per block an LDS OR, then one global atomicOr per word only when the
// block adds bits the word does not already hold.  Blocks are 16 waves (1,024 threads) and
// the grid at most 2 blocks per CU: the per-word liveness atomics of a launch scale with the
// block count, and with 4-wave blocks (1,024 of them at C2) the same ~200 words took ~1,000
// atomics each (134 us per dispatch).
// ------------------------------------------------------------------------------------------
constexpr uint32_t kDedupWaves = 16;
__global__ __launch_bounds__(1024) void k_dense_dedup(PullArgs a) {
    extern __shared__ unsigned long long smem[];
    unsigned long long* s_lp = smem;
    unsigned long long* s_new = smem + a.wact;
    uint8_t* s_wf = reinterpret_cast<uint8_t*>(smem + 2u * a.wact);
    unsigned long long* s_keep = smem + 2u * a.wact + ((a.wact + 15u) & ~15u) / 8u;
    for (uint32_t i = threadIdx.x; i < a.wact; i += blockDim.x) {
        const uint8_t f = a.wflags[a.wbase + i];
        s_lp[i] = (a.live_prev && !a.noskip) ? a.live_prev[a.wbase + i] : ~0ull;
        s_new[i] = 0ull;
        s_wf[i] = f;
        if (a.keep_lds) s_keep[i] = (f & WF_KEEP) ? a.ctl[a.wbase + i].keep : ~0ull;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = a.stride;
    const uint64_t wave = (uint64_t)blockIdx.x * kDedupWaves + wave_in_block();
    const uint64_t nwaves = (uint64_t)gridDim.x * kDedupWaves;
    const uint32_t npass = (a.wact + 127u) / 128u;
    unsigned long long snap_local = 0ull;
    uint32_t t_srd = 0, t_swr = 0, t_fwr = 0;  // wave-uniform traffic accounting
    for (uint64_t v = a.v0 + wave; v < a.n; v += nwaves) {
        uint32_t cnt = 0;
        unsigned long long nzacc = 0ull;
        for (uint32_t pass = 0; pass < npass; pass++) {
            const uint32_t lw = pass * 128u + 2u * lane;
            const uint32_t w = a.wbase + lw;
            const bool act = lw < a.wact;
            uint32_t f0 = 0, f1 = 0;
            uint64_t lp0 = 0ull, lp1 = 0ull;
            if (act) {
                const uint16_t fl = *reinterpret_cast<const uint16_t*>(s_wf + lw);
                f0 = fl & 0xffu;
                f1 = fl >> 8;
                lp0 = s_lp[lw];
                lp1 = s_lp[lw + 1u];
            }
            const bool dead = (lp0 | lp1) == 0ull;
            ulonglong2 s2 = make_ulonglong2(0ull, 0ull), x = make_ulonglong2(0ull, 0ull);
            ulonglong2* ip = reinterpret_cast<ulonglong2*>(a.inc + v * stride + w);
            if (act && !dead) {  // the two loads of the pair, in flight together
                s2 = *reinterpret_cast<const ulonglong2*>(a.seen + v * stride + w);
                x = *ip;
            }
            if (f0 & WF_CLEAR) s2.x = 0ull;
            if (f1 & WF_CLEAR) s2.y = 0ull;
            uint64_t k0 = ~0ull, k1 = ~0ull;
            if (act && (f0 & WF_KEEP)) k0 = s_keep[lw];
            if (act && (f1 & WF_KEEP)) k1 = s_keep[lw + 1u];
            uint64_t n0 = 0ull, n1 = 0ull;
            if (act && !dead) {
                if ((x.x | x.y) != 0ull) *ip = make_ulonglong2(0ull, 0ull);  // consumed
                n0 = x.x & ~s2.x & k0;
                n1 = x.y & ~s2.y & k1;
                if (f0 & WF_GROUP) n0 = group_fix(n0, s2.x, a.ctl[w].gmask, a.ctl[w].gstart);
                if (f1 & WF_GROUP) n1 = group_fix(n1, s2.y, a.ctl[w + 1].gmask, a.ctl[w + 1].gstart);
            }
            // a 16-word tile row of F_next is written (and marked occupied) iff it got a bit
            int ta = (n0 | n1) != 0ull || (a.noskip && act);
            ta |= __shfl_xor(ta, 1, 64);
            ta |= __shfl_xor(ta, 2, 64);
            ta |= __shfl_xor(ta, 4, 64);
            const bool swr = act && (dead ? ((f0 | f1) & WF_CLEAR) != 0u
                                          : ((n0 | n1) != 0ull || ((f0 | f1) & WF_CLEAR) != 0u));
            t_fwr += wave_count(act && ta);
            t_srd += wave_count(act && !dead);
            t_swr += wave_count(swr);
            if (act) {
                uint64_t* sp = a.seen + v * stride + w;
                if (ta) *reinterpret_cast<ulonglong2*>(a.Fnext + v * stride + w) = make_ulonglong2(n0, n1);
                if (swr) {
                    if (dead && !((f0 & f1) & WF_CLEAR))
                        sp[(f0 & WF_CLEAR) ? 0 : 1] = 0ull;
                    else
                        *reinterpret_cast<ulonglong2*>(sp) = make_ulonglong2(s2.x | n0, s2.y | n1);
                }
                if (!dead) {
                    cnt += (uint32_t)(__popcll(n0) + __popcll(n1));
                    if (a.snap) {
                        if (f0 & WF_SNAP) snap_local += (unsigned long long)__popcll(n0 & a.ctl[w].snap);
                        if (f1 & WF_SNAP) snap_local += (unsigned long long)__popcll(n1 & a.ctl[w + 1].snap);
                    }
                    if (n0) atomicOr(&s_new[lw], (unsigned long long)n0);
                    if (n1) atomicOr(&s_new[lw + 1u], (unsigned long long)n1);
                }
            }
            // occupancy word of the node: 8 tile bits per pass, written whole once per word
            const uint32_t tw = (a.wbase + pass * 128u) >> 10;
            unsigned long long nb = (ta && act && (lane & 7u) == 0u) ? 1ull << ((w >> 4) & 63u) : 0ull;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nb |= __shfl_xor(nb, off, 64);
            nzacc |= nb;
            if (pass + 1u == npass || ((a.wbase + (pass + 1u) * 128u) >> 10) != tw) {
                if (lane == 0) a.nz_next[v * a.ntw + tw] = nzacc;
                nzacc = 0ull;
            }
        }
        const uint32_t c = (uint32_t)wave_sum((unsigned long long)cnt);
        if (lane == 0 && c) a.recv[v] += c;  // (sent: derived, engine.hip)
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.acct && lane == 0) {
        const uint32_t tv[3] = {t_srd, t_swr, t_fwr};
#pragma unroll
        for (int q = 0; q < 3; q++)
            if (tv[q]) acct_add(a.acct, 2 + q, (unsigned long long)tv[q]);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.wact; i += blockDim.x) {
        const unsigned long long x = s_new[i];
        if (!x) continue;
        const unsigned long long have = __hip_atomic_load(&a.live[a.wbase + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x & ~have) atomicOr(&a.live[a.wbase + i], x);
    }
}

// ------------------------------------------------------------------------------------------
// k_dense_fused -- the whole DENSE-mode pull of a tick in ONE persistent kernel (round 5): the
// contraction Inc = A x F, the dedup against seen (p2pnode.cc:155-165, 189), and the transposed
// frontier of the NEXT tick, so the tick needs neither k_transpose nor k_dense_dedup nor the
// incoming-word round trip through HBM.  Round 4 ran the three kernels in sequence: on C2 each
// dependent launch cost ~6 us of dispatch gap and k_dense_bits itself paid a prologue, a 3-barrier
// zero-stage test per stage and an epilogue per 256 x 256 tile with nothing to overlap them.
//
// Work: one block per CU walks its tiles (256 rows x 256 columns) in an XCD-major order (the
// column tiles of one row block run on one XCD together, the adjacency rows stay in its L2).
// Per tile only the K stages whose frontier bits are non-zero are computed: the producer of FT
// (this kernel's epilogue at t-1, plus k_births) sets a per-(column tile, stage) bit, so an empty
// stage is neither loaded nor multiplied.  Stages arrive by LDS-DMA (global_load_lds_dwordx4,
// 16 B per lane, no VGPR staging) into two 64-KB buffers; the next (tile, stage) is issued as soon
// as the current one has landed -- across tile boundaries, so the next tile's first stage loads
// while this tile's epilogue runs.  The LDS image is lane-linear per 1-KiB DMA piece (8 rows of
// 128 B); rows are XOR-swizzled on the SOURCE address -- position p of row r holds 16-B chunk
// p ^ ((r >> 1) & 7) -- so the 16 lanes of a ds_read_b128 (16 consecutive rows, one chunk) hit 16
// distinct 16-B bank groups.
//
// Epilogue per tile (every column tile of the window, dead ones included, so F_next and FT_next
// are written whole and need no occupancy test): Inc > 0 -> row words (wave ballots) -> LDS;
// per (row, word pair) new = inc & ~seen & keep, seen |= new, F_next = new, recv += popcount;
// then each wave transposes two 64 x 64 bit blocks of `new` (6 shuffle-and-mask steps) into the
// FT_next rows of its 64 columns, whose non-zero lanes give the word's liveness by ballot.
// Id groups (WF_GROUP), row partitions and the diagnostic no-skip pull take the three-kernel path
// (engine.hip decides per tick).
// ------------------------------------------------------------------------------------------
struct FusedArgs {
    const uint32_t* Ab;                    // n_pad rows x kw words of adjacency bits
    const uint32_t* FTc;                   // transposed F_cur: column rows x kw words
    uint32_t* FTn;                         // transposed F_next (written for every window column)
    const unsigned long long* snz_c;       // per column tile nstw words: bit s = stage s of FTc non-zero
    unsigned long long* snz_n;             // the same for FTn (zeroed by the last tick's launch)
    unsigned long long* snz_z;             // the buffer the next tick writes: zeroed here
    uint32_t snz_zwords;
    uint64_t* seen;
    uint64_t* Fnext;
    const WordCtl* ctl;
    const uint8_t* wflags;
    uint32_t* recv;
    unsigned long long* live;              // liveness of this tick
    const unsigned long long* live_prev;   // nullable: every word live
    unsigned long long* snap;              // nullable
    unsigned long long* acct;              // nullable
    unsigned long long* nz_next;
    uint32_t ntw;
    uint32_t n, n_pad, kw, stride;
    uint32_t nst, nstw;                    // K stages, stage-mask words per column tile
    uint32_t mb, nt, total;                // row blocks, column tiles, mb * nt
    uint32_t wact;                         // window words: occupancy bits of tiles < wact / 16
};

constexpr uint32_t kFStageBytes = 2u * kDenseTile * 128u;  // A + B rows of one 1024-k stage
constexpr uint32_t kFIncOff = 2u * kFStageBytes;           // 256 rows x 4 words of inc / new
constexpr uint32_t kFMiscOff = kFIncOff + kDenseTile * 4u * 8u;
constexpr uint32_t kFLdsBytes = kFMiscOff + 64u;
static_assert(kStageK == 1024u, "k_dense_fused stages 128-B rows");

typedef __attribute__((address_space(3))) uint8_t lds_u8_t;

// One LDS-DMA piece: 16 B per lane from gsrc to LDS byte address lds_dst + 16 x lane.  Inline asm,
// not __builtin_amdgcn_global_load_lds: for the builtin hipcc cannot tell which LDS bytes the DMA
// writes and waits vmcnt(0) before every later ds_read -- the next stage's DMA, issued to the other
// buffer, would then be waited for before the current stage is computed.  The kernel orders the
// DMA itself (vmcnt(0) + barrier before a buffer is read).  M0 is saved and restored around it.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

// stage s of tile (mblk, ct) into buffer `buf`: wave wid DMAs A rows and B rows [32 wid, 32 wid + 32)
__device__ __forceinline__ void fused_issue(const FusedArgs& a, uint8_t* S, uint32_t buf, uint32_t mblk, uint32_t ct,
                                            uint32_t s, uint32_t wid, uint32_t lane) {
    const uint32_t base = (uint32_t)(uintptr_t)(lds_u8_t*)S + buf * kFStageBytes;
    const uint32_t rs = lane >> 3, p = lane & 7u;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t row = wid * 32u + j * 8u + rs;
        const uint32_t q = p ^ ((row >> 1) & 7u);
        const uint32_t* ga = a.Ab + (uint64_t)(mblk * kDenseTile + row) * a.kw + s * 32u + q * 4u;
        const uint32_t* gb = a.FTc + (uint64_t)(ct * kDenseTile + row) * a.kw + s * 32u + q * 4u;
        glds16(ga, base + (wid * 32u + j * 8u) * 128u);
        glds16(gb, base + kDenseTile * 128u + (wid * 32u + j * 8u) * 128u);
    }
}

// the non-empty stages of column tile ct from stage `from` on (bit i of the result = stage from + i,
// up to 64 stages ahead); every stage when there are no masks (FT from k_transpose)
__device__ __forceinline__ uint64_t fused_stages(const FusedArgs& a, uint32_t ct, uint32_t from) {
    if (from >= a.nst) return 0ull;
    uint64_t m;
    if (!a.snz_c) {
        m = ~0ull;
    } else {
        const uint32_t wi = from >> 6, sh = from & 63u;
        m = a.snz_c[(uint64_t)ct * a.nstw + wi] >> sh;
        if (sh && wi + 1u < a.nstw) m |= a.snz_c[(uint64_t)ct * a.nstw + wi + 1u] << (64u - sh);
    }
    const uint32_t left = a.nst - from;
    return left >= 64u ? m : (m & ((1ull << left) - 1ull));
}

__device__ __forceinline__ bool fused_tile_live(const FusedArgs& a, uint32_t w0) {
    if (!a.live_prev) return true;
    return (a.live_prev[w0] | a.live_prev[w0 + 1] | a.live_prev[w0 + 2] | a.live_prev[w0 + 3]) != 0ull;
}

// 64 x 64 bit transpose across a wave: lane r holds row r (bit c = column c) on entry, column r
// (bit r' = row r') on exit
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x, uint32_t lane) {
#pragma unroll
    for (int j = 32; j >= 1; j >>= 1) {
        const uint64_t lo = j == 32 ? 0x00000000ffffffffull
                          : j == 16 ? 0x0000ffff0000ffffull
                          : j == 8 ? 0x00ff00ff00ff00ffull
                          : j == 4 ? 0x0f0f0f0f0f0f0f0full
                          : j == 2 ? 0x3333333333333333ull
                                   : 0x5555555555555555ull;
        const uint64_t y = __shfl_xor(x, j, 64);
        x = (lane & (uint32_t)j) ? ((x & ~lo) | ((y >> j) & lo)) : ((x & lo) | ((y & lo) << j));
    }
    return x;
}

__global__ __launch_bounds__(512, 1) void k_dense_fused(FusedArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t S[kFLdsBytes];
    unsigned long long* sInc = reinterpret_cast<unsigned long long*>(S + kFIncOff);
    unsigned long long* sMisc = reinterpret_cast<unsigned long long*>(S + kFMiscOff);  // [0..3] live, [4] any
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = wave_in_block();
    const uint32_t wm = wid >> 2, wn = wid & 3u;
    // XCD-major walk: block b runs on XCD b % 8 (speed only); XCD x owns tiles [x per, (x+1) per)
    const uint32_t nx = gridDim.x >= 8u ? 8u : 1u;
    const uint32_t xcd = blockIdx.x % nx, bpx = gridDim.x / nx, bi = blockIdx.x / nx;
    const uint32_t per = (a.total + nx - 1u) / nx;
    const uint32_t tlo = xcd * per, thi = min(a.total, tlo + per);
    for (uint32_t i = blockIdx.x * 512u + threadIdx.x; i < a.snz_zwords; i += gridDim.x * 512u) a.snz_z[i] = 0ull;
    if (bi >= bpx) return;  // (gridDim.x is a multiple of 8 when >= 8)

    const uint32_t h = lane >> 5, rr = lane & 31u, sw = (rr >> 1) & 7u;
    uint32_t msk[4];
#pragma unroll
    for (int e = 0; e < 4; e++) msk[e] = 0x01010101u << (4u * h + (uint32_t)e);

    // the (tile, stage) sequence of this block: tiles tlo + bi, + bpx, ... ; stages by mask
    auto tile_mb = [&](uint32_t T) { return T / a.nt; };
    auto tile_ct = [&](uint32_t T) { return T % a.nt; };
    // first stage >= from of tile T (a.nst if none; dead tiles have none)
    auto first_stage = [&](uint32_t T, uint32_t from) -> uint32_t {
        const uint32_t ct = tile_ct(T);
        if (!fused_tile_live(a, ct * 4u)) return a.nst;
        while (from < a.nst) {
            const uint64_t m = fused_stages(a, ct, from);
            if (m) return from + (uint32_t)__builtin_ctzll(m);
            from += 64u;
        }
        return a.nst;
    };
    // the next (tile, stage) to load after (T, s): T == thi when none
    uint32_t LT = tlo + bi, LS = a.nst;
    while (LT < thi && (LS = first_stage(LT, 0u)) >= a.nst) LT += bpx;
    uint32_t buf = 0;
    if (LT < thi) fused_issue(a, S, 0u, tile_mb(LT), tile_ct(LT), LS, wid, lane);

    unsigned long long macs = 0, skipped = 0;
    uint32_t t_srd = 0, t_swr = 0, t_fwr = 0;
    unsigned long long snap_local = 0;

    for (uint32_t T = tlo + bi; T < thi; T += bpx) {
        const uint32_t mblk = tile_mb(T), ct = tile_ct(T), w0 = ct * 4u;
        v16i_t acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[i][j] = v16i_t{0};
        uint32_t computed = 0;
        // the own seen pair of this thread's row (prefetched with the tile's last stage)
        const uint32_t er = t >> 1, ep = t & 1u;
        const uint64_t ev = (uint64_t)mblk * kDenseTile + er;
        const uint32_t wa = w0 + 2u * ep;
        const uint32_t fa = a.wflags[wa], fb = a.wflags[wa + 1];
        const uint64_t lpa = a.live_prev ? a.live_prev[wa] : ~0ull, lpb = a.live_prev ? a.live_prev[wa + 1] : ~0ull;
        const bool dead = (lpa | lpb) == 0ull;
        const bool need_seen = ev < a.n && (!dead || ((fa | fb) & WF_CLEAR));
        ulonglong2 s2 = make_ulonglong2(0ull, 0ull);
        bool seen_loaded = false;
        while (LT == T) {  // the tile's stages, each already issued into `buf`
            const uint32_t s = LS;
            // the next load: this tile's next stage, else the next tile with a stage
            uint32_t nT = T, nS = s + 1u < a.nst ? first_stage(T, s + 1u) : a.nst;
            if (nS >= a.nst) {
                nT = T + bpx;
                while (nT < thi && (nS = first_stage(nT, 0u)) >= a.nst) nT += bpx;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // stage s landed for every wave; buffer buf ^ 1 is free
            if (nT < thi) fused_issue(a, S, buf ^ 1u, tile_mb(nT), tile_ct(nT), nS, wid, lane);
            if (nT != T && need_seen) {  // last stage of the tile: the epilogue's seen pair
                s2 = *reinterpret_cast<const ulonglong2*>(a.seen + ev * a.stride + wa);
                seen_loaded = true;
            }
            const uint8_t* As = S + buf * kFStageBytes;
            const uint8_t* Bs = As + kDenseTile * 128u;
#pragma unroll
            for (uint32_t kq = 0; kq < kStageQ; kq++) {
                const uint32_t off = ((kq ^ sw) << 4);
                uint4 xa[4], xb[2];
#pragma unroll
                for (int i = 0; i < 4; i++)
                    xa[i] = *reinterpret_cast<const uint4*>(As + (wm * 128u + i * 32u + rr) * 128u + off);
#pragma unroll
                for (int j = 0; j < 2; j++)
                    xb[j] = *reinterpret_cast<const uint4*>(Bs + (wn * 64u + j * 32u + rr) * 128u + off);
#pragma unroll
                for (int kc = 0; kc < 4; kc++) {
                    v4i_t af[4], bf[2];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const uint32_t x = kc == 0 ? xa[i].x : kc == 1 ? xa[i].y : kc == 2 ? xa[i].z : xa[i].w;
                        af[i] = dense_expand(x, msk);
                    }
#pragma unroll
                    for (int j = 0; j < 2; j++) {
                        const uint32_t x = kc == 0 ? xb[j].x : kc == 1 ? xb[j].y : kc == 2 ? xb[j].z : xb[j].w;
                        bf[j] = dense_expand(x, msk);
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++)
#pragma unroll
                        for (int j = 0; j < 2; j++)
                            acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
                }
            }
            computed++;
            buf ^= 1u;
            LT = nT;
            LS = nS;
        }
        if (need_seen && !seen_loaded) s2 = *reinterpret_cast<const ulonglong2*>(a.seen + ev * a.stride + wa);
        macs += (unsigned long long)computed;
        skipped += computed == 0u;
        // ---- epilogue 1: Inc > 0 -> one 64-bit word per (row, word): wave ballots -> LDS ----
        if (t < 5u) sMisc[t] = 0ull;
        {
            uint64_t lo = 0ull, hi = 0ull;
            if (computed) {
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int g = 0; g < 16; g++) {
                        const unsigned long long q0 = __ballot(acc[i][0][g] > 0);
                        const unsigned long long q1 = __ballot(acc[i][1][g] > 0);
                        const uint64_t h0 = (q0 & 0xffffffffull) | (q1 << 32);
                        const uint64_t h1 = (q0 >> 32) | (q1 & 0xffffffff00000000ull);
                        const uint32_t row = (uint32_t)(i & 1) * 32u + (g & 3) + 8u * (g >> 2);
                        if (i < 2) {
                            if (lane == row) lo = h0;
                            if (lane == row + 4u) lo = h1;
                        } else {
                            if (lane == row) hi = h0;
                            if (lane == row + 4u) hi = h1;
                        }
                    }
            }
            sInc[(wm * 128u + lane) * 4u + wn] = lo;
            sInc[(wm * 128u + 64u + lane) * 4u + wn] = hi;
        }
        __syncthreads();
        // ---- epilogue 2: dedup of (row er, words wa, wa + 1) ----
        {
            uint64_t n0 = 0ull, n1 = 0ull;
            if (ev < a.n) {
                const uint64_t x0 = sInc[er * 4u + 2u * ep], x1 = sInc[er * 4u + 2u * ep + 1u];
                if (fa & WF_CLEAR) s2.x = 0ull;
                if (fb & WF_CLEAR) s2.y = 0ull;
                const uint64_t k0 = (fa & WF_KEEP) ? a.ctl[wa].keep : ~0ull;
                const uint64_t k1 = (fb & WF_KEEP) ? a.ctl[wa + 1].keep : ~0ull;
                n0 = x0 & ~s2.x & k0;
                n1 = x1 & ~s2.y & k1;
                const bool swr = (n0 | n1) != 0ull || ((fa | fb) & WF_CLEAR) != 0u;
                if (swr) *reinterpret_cast<ulonglong2*>(a.seen + ev * a.stride + wa) = make_ulonglong2(s2.x | n0, s2.y | n1);
                *reinterpret_cast<ulonglong2*>(a.Fnext + ev * a.stride + wa) = make_ulonglong2(n0, n1);
                t_srd += need_seen;
                t_swr += swr;
                t_fwr += 1u;
                if (a.snap) {
                    if (fa & WF_SNAP) snap_local += (unsigned long long)__popcll(n0 & a.ctl[wa].snap);
                    if (fb & WF_SNAP) snap_local += (unsigned long long)__popcll(n1 & a.ctl[wa + 1].snap);
                }
                // tile occupancy of F_next: every tile row of the window is written (zeros included)
                if (ct == 0u && ep == 0u) {
                    const uint32_t ntl = a.wact / 16u;
                    for (uint32_t j = 0; j < a.ntw; j++) {
                        const uint32_t lo_t = j * 64u;
                        const unsigned long long m = ntl <= lo_t ? 0ull : ntl - lo_t >= 64u ? ~0ull : ((1ull << (ntl - lo_t)) - 1ull);
                        a.nz_next[ev * a.ntw + j] = m;
                    }
                }
            }
            uint32_t cnt = (uint32_t)(__popcll(n0) + __popcll(n1));
            cnt += (uint32_t)__shfl_xor((int)cnt, 1, 64);
            if (ep == 0u && cnt) atomicAdd(&a.recv[ev], cnt);  // (sent: derived, engine.hip)
            sInc[er * 4u + 2u * ep] = n0;
            sInc[er * 4u + 2u * ep + 1u] = n1;
        }
        __syncthreads();
        // ---- epilogue 3: FT_next = new transposed; liveness; the next tick's stage bit ----
        {
            unsigned long long any = 0ull;
#pragma unroll
            for (uint32_t q = 0; q < 2; q++) {
                const uint32_t j = wid * 2u + q;         // 64 x 64 block j of the tile's 16
                const uint32_t wi = j & 3u, rg = j >> 2;  // word, 64-row group
                const uint64_t x = sInc[(rg * 64u + lane) * 4u + wi];
                const uint64_t col = wave_transpose64(x, lane);
                const uint64_t c = (uint64_t)(w0 + wi) * 64u + lane;
                *reinterpret_cast<uint64_t*>(a.FTn + c * a.kw + mblk * 8u + rg * 2u) = col;
                const unsigned long long lv = __ballot(col != 0ull);
                if (lane == 0 && lv) {
                    atomicOr(&sMisc[wi], lv);
                    any = 1ull;
                }
            }
            if (lane == 0 && any) atomicOr(&sMisc[4], 1ull);
        }
        __syncthreads();
        if (t < 4u) {
            const unsigned long long x = sMisc[t];
            if (x) {
                const unsigned long long have = __hip_atomic_load(&a.live[w0 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (x & ~have) atomicOr(&a.live[w0 + t], x);
            }
        } else if (t == 4u && sMisc[4]) {
            const uint32_t st = mblk >> 2;  // 4 row blocks of 256 per 1024-k stage
            atomicOr(&a.snz_n[(uint64_t)ct * a.nstw + (st >> 6)], 1ull << (st & 63u));
        }
        // (the next tile's first barrier orders sInc / sMisc reuse)
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.acct) {
        const uint32_t tv[3] = {(uint32_t)wave_sum(t_srd), (uint32_t)wave_sum(t_swr), (uint32_t)wave_sum(t_fwr)};
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 3; q++)
                if (tv[q]) acct_add(a.acct, 2 + q, (unsigned long long)tv[q]);
        }
        if (t == 0 && macs) acct_add(a.acct, 5, 2ull * kDenseTile * kDenseTile * kStageK * macs);
        if (t == 0 && skipped) acct_add(a.acct, 6, skipped);
    }
}
