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
// 64 nodes x one word and transposes the 64 x 64 bit block with ballots.  snz (nullable): the
// fused kernel's stage masks, bit (chunk / 16) of column tile w / 4 set where the block is non-zero.
__global__ __launch_bounds__(256) void k_transpose(const uint64_t* __restrict__ F, uint32_t stride,
                                                   uint32_t n, uint32_t kw, uint32_t nwords,
                                                   const unsigned long long* live_prev,
                                                   const unsigned long long* __restrict__ nz,
                                                   uint32_t ntw, uint32_t* __restrict__ FT,
                                                   unsigned long long* snz, uint32_t nstw) {
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
    if (snz && __ballot(keep != 0ull) && lane == 0) {
        const uint32_t st = chunk / 16u;  // 1,024-node K stage
        atomicOr(&snz[(uint64_t)(w >> 2) * nstw + (st >> 6)], 1ull << (st & 63u));
    }
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
// Work: tiles of 256 rows x 256 columns; per tile only the K stages whose frontier bits are
// non-zero are computed: the producer of FT (this kernel's epilogue at t-1, plus k_births, or
// k_transpose) sets a per-(column tile, stage) bit, so an empty stage is neither loaded nor
// multiplied.  A (tile, non-empty stage) pair is a UNIT.  Schedule: one block per CU (XCD-major
// block order); the live tiles, in GROUPED order (groups of GM row blocks, column tile major
// within a group, so the blocks of one XCD share a few adjacency row blocks and FT tiles in its
// L2), go out in at most `rmax` data-parallel ROUNDS, block b taking tile r G + b in round r.  The
// remaining tiles are the tail: their units, in the same order, fill each block's DEFICIT below
// the mean load ceil(U / G) (column tiles differ in non-empty stages, so the rounds leave blocks
// unevenly loaded), so no CU waits for a whole tile while others idle.  A tile split between
// blocks is reduced by OR: Inc > 0 iff some partial sum is > 0 (all products are >= 0), so each
// block ORs its partial row words into `inc` (atomics), counts its units into the tile's ticket,
// and the block that completes the ticket takes the words back (atomic exchange with 0) and runs
// the epilogue.  (Pure stream-K over all units -- one equal contiguous range per block --
// measured slower on C5: a block's range spans row blocks no other block of its XCD is reading;
// DESIGN.md §3.)  Stages arrive by LDS-DMA (global_load_lds_dwordx4,
// 16 B per lane, no VGPR staging) into two 64-KB buffers; the next (tile, stage) is issued as soon
// as the current one has landed -- across tile boundaries, so the next tile's first stage loads
// while this tile's epilogue runs.  The LDS image is lane-linear per 1-KiB DMA piece (8 rows of
// 128 B); rows are XOR-swizzled on the SOURCE address -- position p of row r holds 16-B chunk
// p ^ ((r >> 1) & 7) -- so the 16 lanes of a ds_read_b128 (16 consecutive rows, one chunk) hit 16
// distinct 16-B bank groups.
//
// Active tiles.  A 16-word tile of the window is ACTIVE this tick if some word of it was live last
// tick, is (re)allocated (WF_CLEAR) or takes a generation (WF_BIRTH).  The 4 column tiles of an
// active tile run the epilogue below even when they compute nothing, so F_next and FT_next are
// written whole there (zeros included) and need no occupancy test; occupancy bit = active.  An
// inactive tile is skipped: its F_next rows keep stale words behind a clear occupancy bit (k_births
// writes a fresh row whole), and its stale FT rows are never read (no word of it can be live next
// tick: nothing arrives in it and no generation lands in it).
// Epilogue per tile: Inc > 0 -> row words (wave ballots) -> LDS;
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
    unsigned long long* inc;               // n x stride words: partial Inc > 0 of split tiles (zero between uses)
    uint32_t* tix;                         // per tile: units reduced so far (zero between uses)
    uint32_t rmax;                         // most data-parallel rounds (A/B: GOSSIP_DENSE_ROUNDS)
    uint32_t gm;                           // row blocks per tile group (tile order, header comment)
    unsigned long long* pts;               // nullable: [4] block 0's start, [5] max block end (phase timer)
    // Row partition (round 6, engine.hip fused_rows): the launch covers the rows of row blocks
    // [mb0, mb0 + mb) -- the host offsets every per-row pointer (Ab, seen, Fnext, recv, inc,
    // nz_next) and FTn by the first row and sets n to the rank's row count; only the stage bit of a
    // tile's F_next (a 1,024-node stage of the WHOLE node range) needs the absolute row block.
    uint32_t mb0;
};

constexpr uint32_t kFStageBytes = 2u * kDenseTile * 128u;  // A + B rows of one 1024-k stage
constexpr uint32_t kFIncOff = 2u * kFStageBytes;           // 256 rows x 4 words of inc / new
constexpr uint32_t kFMiscOff = kFIncOff + kDenseTile * 4u * 8u;
constexpr uint32_t kFActWords = 4;                          // active-tile bits: windows <= 4,096 words
constexpr uint32_t kFActOff = kFMiscOff + 64u;
constexpr uint32_t kFMaxCt = kFActWords * 64u * 4u;         // column tiles of the widest window
static_assert(kFMaxCt <= 4096u, "the prefix scan packs a live-tile count of 12 bits");
constexpr uint32_t kFCtOff = kFActOff + kFActWords * 8u;    // per column tile: units, prefix (u32)
constexpr uint32_t kFLctOff = kFCtOff + 2u * kFMaxCt * 4u;  // the column tiles with units, in order (u16)
constexpr uint32_t kFFlgOff = kFLctOff + kFMaxCt * 2u;      // per column tile: its 4 word-flag bytes
constexpr uint32_t kFS2Off = (kFFlgOff + kFMaxCt * 4u + 15u) & ~15u;  // the epilogue's seen pairs (LDS-DMA)
constexpr uint32_t kFLdsBytes = kFS2Off + 512u * 16u;
static_assert(kFLdsBytes <= 163840u, "k_dense_fused LDS");
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

// x of lane (lane ^ J), every lane active: DPP quad permutes (J = 1, 2), row shifts both ways
// (J = 4, 8) and gfx950's permlane swaps (J = 16, 32) -- VALU only, no ds_bpermute round trip
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x, uint32_t lane) {
    if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
    if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);
    if constexpr (J == 4 || J == 8) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + J, 0xF, 0xF, false);  // row_shl: lane + J
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x110 + J, 0xF, 0xF, false);  // row_shr: lane - J
        return (lane & (uint32_t)J) ? dn : up;
    }
    if constexpr (J == 16) {  // swaps the odd 16-lane rows of the first operand with the even rows of the second
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16u) ? (uint32_t)r[0] : (uint32_t)r[1];
    }
    if constexpr (J == 32) {  // swaps the upper 32 lanes of the first operand with the lower 32 of the second
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32u) ? (uint32_t)r[0] : (uint32_t)r[1];
    }
    return x;
}

template <int J>
__device__ __forceinline__ uint64_t transpose_step(uint64_t x, uint32_t lane, uint64_t lo) {
    const uint64_t y = ((uint64_t)lane_xor<J>((uint32_t)(x >> 32), lane) << 32) | lane_xor<J>((uint32_t)x, lane);
    return (lane & (uint32_t)J) ? ((x & ~lo) | ((y >> J) & lo)) : ((x & lo) | ((y & lo) << J));
}

// 64 x 64 bit transpose across a wave: lane r holds row r (bit c = column c) on entry, column r
// (bit r' = row r') on exit (block swaps of 32, 16, ..., 1)
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x, uint32_t lane) {
    x = transpose_step<32>(x, lane, 0x00000000ffffffffull);
    x = transpose_step<16>(x, lane, 0x0000ffff0000ffffull);
    x = transpose_step<8>(x, lane, 0x00ff00ff00ff00ffull);
    x = transpose_step<4>(x, lane, 0x0f0f0f0f0f0f0f0full);
    x = transpose_step<2>(x, lane, 0x3333333333333333ull);
    x = transpose_step<1>(x, lane, 0x5555555555555555ull);
    return x;
}

// Lanes L and L + 4 of the pair (x0, x1) := (a0, a1) and (b0, b1) (wave-uniform SGPR values):
// v_writelane (one VALU each, EXEC ignored).  The row words of the fused epilogue's ballots are
// placed this way: the select form (lane == row ? h : x) cost a compare, SGPR->VGPR moves and
// lane-mask reloads per row (hipcc has no writelane builtin).  The s_nop keeps the writelanes 5
// wait states behind the compares that wrote their SGPRs (without it, bits were lost).
template <int L>
__device__ __forceinline__ void write_lanes(uint32_t& x0, uint32_t& x1, uint32_t a0, uint32_t a1, uint32_t b0,
                                            uint32_t b1) {
    asm volatile(
        "s_nop 4\n\t"
        "v_writelane_b32 %0, %2, %6\n\t"
        "v_writelane_b32 %1, %3, %6\n\t"
        "v_writelane_b32 %0, %4, %7\n\t"
        "v_writelane_b32 %1, %5, %7"
        : "+v"(x0), "+v"(x1)
        : "s"(a0), "s"(a1), "s"(b0), "s"(b1), "n"(L), "n"(L + 4));
}
// Inc > 0 -> row words: ballot of MFMA register g of tiles (i, 0) and (i, 1) = row (g & 3) + 8 (g >> 2)
// (+ 32 for odd i) in its low half, the row 4 below in its high half; w[0..1] = lo (rows 0..63 of
// the wave), w[2..3] = hi (rows 64..127), low / high 32 columns
template <int K>
__device__ __forceinline__ void fused_row_words(const v16i_t (&acc)[4][2], uint32_t (&w)[4]) {
    if constexpr (K < 64) {
        constexpr int i = K / 16, g = K % 16;
        constexpr int row = (i & 1) * 32 + (g & 3) + 8 * (g >> 2);
        constexpr int d = i < 2 ? 0 : 2;
        const unsigned long long q0 = __ballot(acc[i][0][g] > 0);
        const unsigned long long q1 = __ballot(acc[i][1][g] > 0);
        write_lanes<row>(w[d], w[d + 1], (uint32_t)q0, (uint32_t)q1, (uint32_t)(q0 >> 32), (uint32_t)(q1 >> 32));
        fused_row_words<K + 1>(acc, w);
    }
}

// Diagnostic build DENSE_STAMPS: shader cycles per phase of k_dense_fused (s_memtime), summed over
// waves into acct[22..29] (engine.hip prints them); no output depends on them.  0 prologue and
// epilogue-only tiles, 1 stage barrier (waves waiting for each other), 2 stage issue + MFMA,
// 3 ballots, 4 split-tile reduction, 5 epilogue dedup, 6 epilogue transpose + liveness, 7 the
// wave's own stage wait (vmcnt: its DMA pieces, and stores of a deferred epilogue); acct[30]
// block time (s_memrealtime, 100 MHz) and acct[31] its shader cycles, per block
#ifdef DENSE_STAMPS
#define DSTAMP(k)                                              \
    do {                                                       \
        const uint64_t ds_t = __builtin_amdgcn_s_memtime();    \
        dcyc[k] += ds_t - dlast;                               \
        dlast = ds_t;                                          \
    } while (0)
#else
#define DSTAMP(k) \
    do {          \
    } while (0)
#endif

__global__ __launch_bounds__(512, 1) void k_dense_fused(FusedArgs a) {
#ifdef DENSE_STAMPS
    uint64_t dcyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t dlast = __builtin_amdgcn_s_memtime();
    const uint64_t drt0 = __builtin_amdgcn_s_memrealtime(), dmt0 = dlast;  // (block time, 100 MHz; clock calibration)
#endif
    __shared__ __attribute__((aligned(16))) uint8_t S[kFLdsBytes];
    unsigned long long* sInc = reinterpret_cast<unsigned long long*>(S + kFIncOff);
    unsigned long long* sMisc = reinterpret_cast<unsigned long long*>(S + kFMiscOff);  // [0..3] live, [4] any, [5] flag, [6] wave sums
    unsigned long long* sAct = reinterpret_cast<unsigned long long*>(S + kFActOff);
    uint32_t* sCtU = reinterpret_cast<uint32_t*>(S + kFCtOff);  // units of column tile ct (any row block)
    uint32_t* sCtP = sCtU + kFMaxCt;                             // exclusive prefix of sCtU
    uint16_t* sLct = reinterpret_cast<uint16_t*>(S + kFLctOff);  // column tiles with units, in order
    uint32_t* sCtF = reinterpret_cast<uint32_t*>(S + kFFlgOff);  // the column tile's word flags
    const ulonglong2* sS2 = reinterpret_cast<const ulonglong2*>(S + kFS2Off);  // thread t's seen pair
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = wave_in_block();
    const uint32_t wm = wid >> 2, wn = wid & 3u;
    if (a.pts && blockIdx.x == 0 && t == 0) a.pts[4] = __builtin_amdgcn_s_memrealtime();  // (dispatched first)
    for (uint32_t i = blockIdx.x * 512u + t; i < a.snz_zwords; i += gridDim.x * 512u) a.snz_z[i] = 0ull;
    // Per column tile ct (thread t, +512): its 4 flag bytes, its 4 live_prev words and its stage
    // masks, all loaded before any is used (one round trip).  Active 16-word tiles (header comment:
    // 4 column tiles, lanes 4k..4k+3) -> LDS bitmap, then F_next's occupancy words; units per column
    // tile: its non-empty stages if its tile is active and the column tile was live last tick.
    if (t < kFActWords) sAct[t] = 0ull;
    __syncthreads();
    for (uint32_t ct0 = 0; ct0 < a.nt; ct0 += 512u) {  // (uniform trip count: the quad shuffles see every lane)
        const uint32_t ct = ct0 + t;
        const bool in = ct < a.nt;
        uint32_t f = 0u, u = 0u;
        uint64_t lp = 0ull;
        if (in) {
            f = *reinterpret_cast<const uint32_t*>(a.wflags + ct * 4u);
            if (a.live_prev) {
                const ulonglong2* p = reinterpret_cast<const ulonglong2*>(a.live_prev + ct * 4u);
                const ulonglong2 x = p[0], y = p[1];
                lp = x.x | x.y | y.x | y.y;
            } else {
                lp = ~0ull;
            }
            for (uint32_t s0 = 0; s0 < a.nst; s0 += 64u) u += (uint32_t)__popcll(fused_stages(a, ct, s0));
        }
        uint32_t c = (in && (lp != 0ull || (f & (0x01010101u * (WF_CLEAR | WF_BIRTH))) != 0u)) ? 1u : 0u;
        c |= lane_xor<1>(c, lane);
        c |= lane_xor<2>(c, lane);
        if (in) {
            if ((ct & 3u) == 0u && c) atomicOr(&sAct[ct >> 8], 1ull << ((ct >> 2) & 63u));
            sCtU[ct] = (c && lp != 0ull) ? u : 0u;
            sCtF[ct] = f;
        }
    }
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * 512u + t; i < (uint64_t)a.n * a.ntw; i += (uint64_t)gridDim.x * 512u)
        a.nz_next[i] = sAct[i % a.ntw];
    auto active = [&](uint32_t ct) -> bool { return (sAct[ct >> 8] >> ((ct >> 2) & 63u)) & 1ull; };
    // exclusive prefix over the column tiles of (units << 12 | live), so the same scan places the
    // live column tiles: each thread sums a run of them, the block scans the runs (units < 2^20:
    // the host's gate ntw <= kFActWords keeps nt <= kFMaxCt = 1,024 column tiles -- the LDS
    // tables' size, and what keeps the packed 12-bit live count exact -- x <= 512 stages)
    const uint32_t run = (a.nt + 511u) / 512u, c0 = t * run;
    uint32_t mine = 0;
    for (uint32_t c = c0; c < min(a.nt, c0 + run); c++) mine += (sCtU[c] << 12) | (sCtU[c] ? 1u : 0u);
    uint32_t incl = mine;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, off, 64);
        if (lane >= (uint32_t)off) incl += y;
    }
    uint32_t* sWave = reinterpret_cast<uint32_t*>(sInc);  // 8 wave totals (sInc is free until the first tile)
    if (lane == 63u) sWave[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, rowU = 0;
    for (uint32_t q = 0; q < 8u; q++) {
        const uint32_t x = sWave[q];
        if (q < wid) wbase += x;
        rowU += x;
    }
    {
        uint32_t p = wbase + incl - mine;
        for (uint32_t c = c0; c < min(a.nt, c0 + run); c++) {
            sCtP[c] = p >> 12;
            if (sCtU[c]) sLct[p & 4095u] = (uint16_t)c;
            p += (sCtU[c] << 12) | (sCtU[c] ? 1u : 0u);
        }
    }
    __syncthreads();
    const uint32_t nlc = rowU & 4095u;  // (packed: units in the high bits, live column tiles in the low 12)
    rowU >>= 12;
    // blocks in XCD-major order (block b runs on XCD b % 8: adjacent ords share an XCD)
    const uint32_t G = gridDim.x;
    const uint32_t nx = G >= 8u ? 8u : 1u;
    const uint32_t ord = (blockIdx.x % nx) * (G / nx) + blockIdx.x / nx;
    // Tile order: groups of GM row blocks; within a group, column tile major, then row block; each
    // tile's units (its non-empty stages) contiguous.  32 consecutive tiles -- the blocks of one XCD
    // in a round -- then span GM row blocks x 32 / GM column tiles: per stage they read GM
    // adjacency tiles and 32 / GM FT tiles through that XCD's L2, not 1 + 32 (row-major order)
    const uint32_t GM = a.gm;
    const uint64_t GU = (uint64_t)GM * rowU;   // units of a full group
    const uint64_t U = (uint64_t)a.mb * rowU;  // units of the tick
    const uint32_t L = a.mb * nlc;             // live tiles
    auto grows = [&](uint32_t g) -> uint32_t { return min(GM, a.mb - g * GM); };
    // the i-th live tile in tile order -> (row block, column tile), and its first unit
    auto tile_at = [&](uint32_t i, uint32_t& mblk, uint32_t& ct) -> uint64_t {
        const uint32_t g = i / (GM * nlc), j = i - g * (GM * nlc), rows = grows(g);
        ct = sLct[j / rows];
        const uint32_t r = j % rows;
        mblk = g * GM + r;
        return g * GU + (uint64_t)rows * sCtP[ct] + (uint64_t)r * sCtU[ct];
    };
    const uint32_t R = min(L / G, a.rmax);    // whole data-parallel rounds
    // the tail: live tiles [R G, L), whose units fill the blocks' deficits below the mean load
    // ceil(U / G) in ord order (column tiles differ in non-empty stages, so the rounds leave the
    // blocks unequal; an even split of the tail would keep that difference)
    uint64_t tail0 = U;
    if (R * G < L) {
        uint32_t m_, c_;
        tail0 = tile_at(R * G, m_, c_);
    }
    uint64_t tu0, tu1;
    {
        const uint64_t Tm = (U + G - 1u) / G, Ut = U - tail0;
        uint32_t* sTw = reinterpret_cast<uint32_t*>(sInc) + 32;  // wave totals, then the deficits'
        uint32_t* sD = sTw + 8;                                  // prefix sD[0..G] (sInc is free here)
        uint32_t d = 0;
        if (t < G) {
            uint64_t w = 0;
            for (uint32_t k = 0; k < R; k++) {
                uint32_t m_, c_;
                tile_at(k * G + t, m_, c_);
                w += sCtU[c_];
            }
            d = w < Tm ? (uint32_t)(Tm - w) : 0u;  // (sum of deficits <= G Tm < 2^31)
        }
        uint32_t di = d;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)di, off, 64);
            if (lane >= (uint32_t)off) di += y;
        }
        if (lane == 63u) sTw[wid] = di;
        __syncthreads();
        uint32_t db = 0;
        for (uint32_t q = 0; q < wid; q++) db += sTw[q];
        if (t < G) sD[t + 1u] = db + di;
        if (t == 0) sD[0] = 0u;
        __syncthreads();
        tu0 = tail0 + min<uint64_t>(sD[ord], Ut);
        tu1 = tail0 + min<uint64_t>(sD[ord + 1u], Ut);
    }
    // this block's range k: round k's tile (k < R), then (k == R) its share of the tail
    auto range_of = [&](uint32_t k, uint64_t& b, uint64_t& e) -> bool {
        if (k < R) {
            uint32_t m_, ct;
            b = tile_at(k * G + ord, m_, ct);
            e = b + sCtU[ct];
            return true;
        }
        b = tu0;
        e = tu1;
        return k == R && tu0 < tu1;
    };

    const uint32_t h = lane >> 5, rr = lane & 31u, sw = (rr >> 1) & 7u;
    uint32_t msk[4];
#pragma unroll
    for (int e = 0; e < 4; e++) msk[e] = 0x01010101u << (4u * h + (uint32_t)e);
    unsigned long long macs = 0;
    uint32_t t_srd = 0, t_swr = 0, t_fwr = 0;
    unsigned long long snap_local = 0;
    const uint32_t er = t >> 1, ep = t & 1u;  // epilogue: row er, word pair ep of the tile

    // the s-th non-empty stage of column tile ct, from stage `from` on (the first one: n = 0)
    auto stage_from = [&](uint32_t ct, uint32_t from) -> uint32_t {
        while (from < a.nst) {
            const uint64_t m = fused_stages(a, ct, from);
            if (m) return from + (uint32_t)__builtin_ctzll(m);
            from += 64u;
        }
        return a.nst;
    };
    // one-word stage masks (nst <= 64 stages): the current tile's mask stays in a register, so the
    // next unit of the same tile needs no load (a load there waited at every unit: vmcnt(0))
    const bool one_word = a.nstw == 1u;
    auto stage_in = [&](uint64_t m, uint32_t from) -> uint32_t {
        if (from >= a.nst) return a.nst;
        m >>= from;
        return m ? from + (uint32_t)__builtin_ctzll(m) : a.nst;
    };
    // unit u -> (row block, column tile, stage); also the tile's first unit
    auto locate = [&](uint64_t u, uint32_t& mblk, uint32_t& ct, uint32_t& st, uint64_t& tfirst) {
        const uint32_t g = (uint32_t)(u / GU), rows = grows(g);
        const uint32_t rem = (uint32_t)(u - g * GU);  // (< GM rowU < 2^26)
        uint32_t lo = 0, hi = a.nt;  // last ct with rows sCtP[ct] <= rem and sCtU[ct] > 0
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) / 2u;
            if (rows * sCtP[mid] <= rem) lo = mid; else hi = mid;
        }
        while (lo + 1u < a.nt && (sCtU[lo] == 0u || rows * (sCtP[lo] + sCtU[lo]) <= rem)) lo++;  // (never taken)
        ct = lo;
        const uint32_t rem2 = rem - rows * sCtP[ct], r = rem2 / sCtU[ct];
        uint32_t k = rem2 - r * sCtU[ct];
        mblk = g * GM + r;
        tfirst = u - k;
        st = stage_from(ct, 0u);
        while (k--) st = stage_from(ct, st + 1u);
    };

    // ---- the epilogue's per-thread inputs (row er, words wa, wa + 1 of tile (mblk, ct)), loaded
    //      with no dependence between them -- one round trip, issued with the tile's last stage ----
    //      (the own seen pairs go to LDS by DMA, so no register holds them across the MFMA loop and
    //      no wait for them lands before it: loaded into registers, the compiler spilled them and
    //      waited vmcnt(0) -- for the next stage's DMA too -- at every tile's last stage; the flags
    //      come from the prologue's copy in LDS.  Landed at the next vmcnt(0) + barrier.)
    const uint32_t s2_lds = (uint32_t)(uintptr_t)(lds_u8_t*)S + kFS2Off + wid * 1024u;
    auto epi_issue = [&](uint32_t mblk, uint32_t ct) {
        const uint64_t ev = min<uint64_t>((uint64_t)mblk * kDenseTile + er, (uint64_t)a.n - 1u);  // (rows >= n: unused)
        glds16(a.seen + ev * a.stride + ct * 4u + 2u * ep, s2_lds);
    };
    // ---- the epilogue of tile (mblk, ct): sInc holds its Inc > 0 words ----
    auto epilogue = [&](uint32_t mblk, uint32_t ct) {
        const uint32_t w0 = ct * 4u;
        const uint64_t ev = (uint64_t)mblk * kDenseTile + er;
        const uint32_t wa = w0 + 2u * ep;
        const uint32_t f4 = sCtF[ct];
        const uint32_t fa = (f4 >> (16u * ep)) & 0xffu, fb = (f4 >> (16u * ep + 8u)) & 0xffu;
        ulonglong2 s2 = sS2[t];
        DSTAMP(3);
        uint64_t n0 = 0ull, n1 = 0ull;
        if (ev < a.n) {
            const uint64_t x0 = sInc[er * 4u + 2u * ep], x1 = sInc[er * 4u + 2u * ep + 1u];
            if (fa & WF_CLEAR) s2.x = 0ull;
            if (fb & WF_CLEAR) s2.y = 0ull;
            const uint64_t k0 = (fa & WF_KEEP) ? a.ctl[wa].keep : ~0ull;  // (cut words only: rare)
            const uint64_t k1 = (fb & WF_KEEP) ? a.ctl[wa + 1].keep : ~0ull;
            n0 = x0 & ~s2.x & k0;
            n1 = x1 & ~s2.y & k1;
            const bool swr = (n0 | n1) != 0ull || ((fa | fb) & WF_CLEAR) != 0u;
            if (swr) *reinterpret_cast<ulonglong2*>(a.seen + ev * a.stride + wa) = make_ulonglong2(s2.x | n0, s2.y | n1);
            *reinterpret_cast<ulonglong2*>(a.Fnext + ev * a.stride + wa) = make_ulonglong2(n0, n1);
            t_srd += 1u;  // (the seen pair is loaded for every row)
            t_swr += swr;
            t_fwr += 1u;
            if (a.snap) {
                if (fa & WF_SNAP) snap_local += (unsigned long long)__popcll(n0 & a.ctl[wa].snap);
                if (fb & WF_SNAP) snap_local += (unsigned long long)__popcll(n1 & a.ctl[wa + 1].snap);
            }
        }
        uint32_t cnt = (uint32_t)(__popcll(n0) + __popcll(n1));
        cnt += (uint32_t)__shfl_xor((int)cnt, 1, 64);
        if (ep == 0u && cnt) atomicAdd(&a.recv[ev], cnt);  // (sent: derived, engine.hip)
        if (t < 5u) sMisc[t] = 0ull;
        sInc[er * 4u + 2u * ep] = n0;
        sInc[er * 4u + 2u * ep + 1u] = n1;
        __syncthreads();
        DSTAMP(5);
        // FT_next = new transposed (two 64 x 64 blocks per wave); liveness; the next tick's stage bit
        unsigned long long any = 0ull;
#pragma unroll
        for (uint32_t q = 0; q < 2; q++) {
            const uint32_t j = wid * 2u + q;
            const uint32_t wi = j & 3u, rg = j >> 2;
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
        __syncthreads();
        if (t < 4u) {
            const unsigned long long x = sMisc[t];
            if (x) atomicOr(&a.live[w0 + t], x);  // (no return: nothing waits for it)
        } else if (t == 4u && sMisc[4]) {
            const uint32_t stg = (a.mb0 + mblk) >> 2;  // 4 row blocks of 256 per 1024-k stage
            atomicOr(&a.snz_n[(uint64_t)ct * a.nstw + (stg >> 6)], 1ull << (stg & 63u));
        }
        __syncthreads();  // (sInc / sMisc reuse by the next tile)
        DSTAMP(6);
    };

    // the first unit's stage goes out first, then the epilogue-only tiles -- active, no unit
    // (nothing computed; F_next / FT_next zeroed, seen words of re-allocated words cleared),
    // dealt round-robin -- run while it loads
    uint32_t buf = 0;
    uint32_t LM = 0, LC = 0, LS = 0;
    uint64_t LF = 0, LK = 0;  // LK: the current tile's stage mask (one_word)
    uint32_t rk = 0;
    uint64_t rb = 0, re = 0;
    bool have = range_of(0u, rb, re);
    if (have) {
        locate(rb, LM, LC, LS, LF);
        if (one_word) LK = fused_stages(a, LC, 0u);
        fused_issue(a, S, 0u, LM, LC, LS, wid, lane);
    }
    DSTAMP(0);
    for (uint32_t T = ord; T < a.total; T += G) {
        const uint32_t ct = T % a.nt, mblk = T / a.nt;
        if (!active(ct) || sCtU[ct] != 0u) continue;
        epi_issue(mblk, ct);
        sInc[er * 4u + 2u * ep] = 0ull;
        sInc[er * 4u + 2u * ep + 1u] = 0ull;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        epilogue(mblk, ct);
    }
    DSTAMP(0);  // (epilogue-only tiles: with the prologue)
    // ---- this block's ranges, each a run of units [rb, re); the unit loads chain across them ----
    uint64_t u = rb;
    // A whole tile's epilogue is deferred to just after the next unit's barrier and before that
    // unit's stage issue: its stores then have a whole unit of MFMA to complete before the next
    // stage wait (vmcnt counts stores and atomics too: an epilogue right before a wait would hold
    // every tile boundary for their acks)
    bool pend = false;
    uint32_t pM = 0, pC = 0;
    while (have) {
        // one tile segment: units [u, end) of tile (mblk, ct) -- the whole tile or a part of it
        const uint32_t mblk = LM, ct = LC;
        const uint64_t tfirst = LF, tlast = tfirst + sCtU[ct];
        const uint64_t end = min<uint64_t>(re, tlast);
        const uint64_t seg_b = max<uint64_t>(rb, tfirst);  // this block's first unit of the tile
        const bool whole = seg_b == tfirst && end == tlast;
        const uint32_t w0 = ct * 4u;
        const uint64_t ev = (uint64_t)mblk * kDenseTile + er;
        const uint32_t wa = w0 + 2u * ep;
        v16i_t acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[i][j] = v16i_t{0};
        // after the segment: the next range when this one ends with it
        bool next_have = true;
        uint32_t next_k = rk;
        uint64_t next_b = rb, next_e = re;
        for (; u < end; u++) {
            const uint32_t s = LS;
            // the next unit: the tile's next stage, else the range's next column tile with units,
            // else the first unit of the block's next range
            uint32_t nM = LM, nC = LC, nS = a.nst;
            uint64_t nF = LF, nK = LK;
            bool more = true;
            if (u + 1u < re) {
                if (u + 1u < tlast) {
                    nS = one_word ? stage_in(LK, s + 1u) : stage_from(LC, s + 1u);
                } else {  // the next tile in tile order (one exists: u + 1 < re <= U)
                    const uint32_t g = LM / GM;
                    if (LM - g * GM + 1u < grows(g)) {
                        nM = LM + 1u;
                    } else {
                        nM = g * GM;
                        nC = LC + 1u;
                        while (true) {
                            if (nC >= a.nt) { nC = 0; nM += GM; }  // (the next group)
                            if (sCtU[nC]) break;
                            nC++;
                        }
                    }
                    nF = tlast;
                    if (!one_word) {
                        nS = stage_from(nC, 0u);
                    } else {
                        if (nC != LC) nK = fused_stages(a, nC, 0u);  // (masks are per column tile)
                        nS = stage_in(nK, 0u);
                    }
                }
            } else {
                more = false;
                for (uint32_t k = rk + 1u; k <= R; k++) {
                    uint64_t b, e;
                    if (range_of(k, b, e)) {
                        more = true;
                        next_k = k;
                        next_b = b;
                        next_e = e;
                        locate(b, nM, nC, nS, nF);
                        if (one_word) nK = fused_stages(a, nC, 0u);
                        break;
                    }
                }
                next_have = more;
            }
            DSTAMP(2);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            DSTAMP(7);  // (this wave's stage wait)
            __syncthreads();  // stage s landed for every wave; buffer buf ^ 1 is free
            DSTAMP(1);
            if (pend) {  // (no stage in flight: the epilogue's barriers drain nothing)
                epilogue(pM, pC);
                pend = false;
            }
            if (more) fused_issue(a, S, buf ^ 1u, nM, nC, nS, wid, lane);
            if (u + 1u == end && whole) epi_issue(mblk, ct);  // the epilogue's seen pairs, early
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
            macs++;
            DSTAMP(2);
            buf ^= 1u;
            LM = nM; LC = nC; LS = nS; LF = nF; LK = nK;
        }
        // ---- Inc > 0 -> one 64-bit word per (row, word): wave ballots; lane l collects rows l (lo)
        //      and l + 64 (hi) of the wave's 128 (a ballot of register g of MFMA tile (i, j) holds
        //      columns 32j..32j+31 of row (g & 3) + 8 (g >> 2) in its low half, of the row 4 below in
        //      its high half) ----
        uint32_t rw[4] = {0u, 0u, 0u, 0u};
        fused_row_words<0>(acc, rw);
        const uint64_t lo = (uint64_t)rw[0] | ((uint64_t)rw[1] << 32), hi = (uint64_t)rw[2] | ((uint64_t)rw[3] << 32);
        DSTAMP(3);
        const uint64_t vlo = (uint64_t)mblk * kDenseTile + wm * 128u + lane;
        if (whole) {
            sInc[(wm * 128u + lane) * 4u + wn] = lo;
            sInc[(wm * 128u + 64u + lane) * 4u + wn] = hi;
            pend = true;  // (the next unit's barrier orders these writes before the epilogue)
            pM = mblk;
            pC = ct;
        } else {
            // a split tile: OR the partial words into inc, count the units into the tile's ticket;
            // the block completing it takes the words back and runs the epilogue
            unsigned long long* ip = a.inc + vlo * a.stride + w0 + wn;
            if (lo && vlo < a.n) atomicOr(ip, (unsigned long long)lo);
            if (hi && vlo + 64u < a.n) atomicOr(ip + 64ull * a.stride, (unsigned long long)hi);
            // every wave waits for its atomics' acknowledgements before the barrier (a
            // barrier alone need not: the compiler may drop the wait), so all of this block's ORs
            // are performed before its ticket.  No fence beyond that: the ORs, the ticket and the
            // completing block's exchanges are device-scope atomics, performed in order at the
            // address's coherence point, and the exchange is issued after the ticket that counted
            // this block returned -- a release fence here wrote back the XCD's L2 (buffer_wbl2) in
            // every split tile: C2's phase 0.0995 -> 0.108 ms (profiles/r06/dense_*)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                const uint32_t mineu = (uint32_t)(end - seg_b);  // units this block reduced into the tile
                const uint32_t T = mblk * a.nt + ct;
                const uint32_t old = __hip_atomic_fetch_add(&a.tix[T], mineu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const bool last = old + mineu == sCtU[ct];
                if (last) __hip_atomic_store(&a.tix[T], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sMisc[5] = last ? 1ull : 0ull;
            }
            __syncthreads();
            DSTAMP(4);
            if (sMisc[5]) {
                // (atomic exchange: the other blocks' atomics are read where they were performed)
                if (ev < a.n) {
                    unsigned long long* rp = a.inc + ev * a.stride + wa;
                    sInc[er * 4u + 2u * ep] = atomicExch(rp, 0ull);
                    sInc[er * 4u + 2u * ep + 1u] = atomicExch(rp + 1, 0ull);
                } else {
                    sInc[er * 4u + 2u * ep] = 0ull;
                    sInc[er * 4u + 2u * ep + 1u] = 0ull;
                }
                epi_issue(mblk, ct);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                epilogue(mblk, ct);
            }
        }
        if (u == re) {  // the range is done: on to the next one (its first unit is already loading)
            have = next_have;
            rk = next_k;
            rb = next_b;
            re = next_e;
            u = rb;
        }
    }
    if (pend) {  // the last tile's epilogue
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        epilogue(pM, pC);
    }
    if (a.snap) {
        snap_local = wave_sum(snap_local);
        if (lane == 0 && snap_local) atomicAdd(a.snap, snap_local);
    }
    if (a.pts) {  // (every wave's last store issued; the end stamp of the block's last wave)
        __syncthreads();
        if (t == 0) atomicMax(&a.pts[5], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
#ifdef DENSE_STAMPS
    if (a.acct && lane == 0)
        for (int k = 0; k < 8; k++) acct_add(a.acct, 22u + (uint32_t)k, (unsigned long long)dcyc[k]);
    if (a.acct && t == 0) {  // block 0..G-1 durations: realtime ticks, shader cycles (wave 0)
        acct_add(a.acct, 30u, (unsigned long long)(__builtin_amdgcn_s_memrealtime() - drt0));
        acct_add(a.acct, 31u, (unsigned long long)(__builtin_amdgcn_s_memtime() - dmt0));
    }
#endif
    if (a.acct) {
        const uint32_t tv[3] = {(uint32_t)wave_sum(t_srd), (uint32_t)wave_sum(t_swr), (uint32_t)wave_sum(t_fwr)};
        if (lane == 0) {
#pragma unroll
            for (int q = 0; q < 3; q++)
                if (tv[q]) acct_add(a.acct, 2 + q, (unsigned long long)tv[q]);
        }
        if (t == 0 && macs) acct_add(a.acct, 5, 2ull * kDenseTile * kDenseTile * kStageK * macs);
        if (t == 0 && ord == 0) {  // tiles computing nothing (no live word or no non-empty stage)
            uint32_t z = 0;
            for (uint32_t c = 0; c < a.nt; c++) z += sCtU[c] == 0u;
            if (z) acct_add(a.acct, 6, (unsigned long long)z * a.mb);
        }
    }
}

// ---- FT slice exchange (row partition with the fused tick, engine.hip exchange_ft) -----------
// A rank's message, u32 words: [W x S] its nodes' bits of every window column of FT_next (column c:
// words [c S, c S + S), the rank's rows lo .. hi as words lo / 32 .. of FT's column row; S = the
// largest rank's word count, zero-padded), then [2 nsnz] its F_next stage masks, [2 wact] its partial
// liveness.  Every rank all-gathers the messages and unpacks the others' (k_ft_unpack).
__global__ __launch_bounds__(256) void k_ft_pack(const uint32_t* __restrict__ FT, uint32_t kw, uint32_t lo_w,
                                                 uint32_t S, uint32_t Sown, uint32_t W,
                                                 const unsigned long long* __restrict__ snz, uint32_t nsnz,
                                                 const unsigned long long* __restrict__ live, uint32_t wact,
                                                 uint32_t* __restrict__ msg) {
    const uint64_t nft = (uint64_t)W * S, tot = nft + 2ull * nsnz + 2ull * wact;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < tot; i += (uint64_t)gridDim.x * 256u) {
        uint32_t x;
        if (i < nft) {
            const uint32_t c = (uint32_t)(i / S), j = (uint32_t)(i - (uint64_t)c * S);
            x = j < Sown ? FT[(uint64_t)c * kw + lo_w + j] : 0u;
        } else if (i < nft + 2ull * nsnz) {
            const uint64_t k = i - nft;
            x = (uint32_t)(snz[k >> 1] >> (32u * (k & 1u)));
        } else {
            const uint64_t k = i - nft - 2ull * nsnz;
            x = (uint32_t)(live[k >> 1] >> (32u * (k & 1u)));
        }
        msg[i] = x;
    }
}
// Rank r's message into this rank's FT_next (its rows' words of every column), stage masks and
// liveness (OR: every rank's stage bits and live words are partial)
__global__ __launch_bounds__(256) void k_ft_unpack(uint32_t* __restrict__ FT, uint32_t kw, uint32_t lo_w, uint32_t S,
                                                   uint32_t Sr, uint32_t W, const uint32_t* __restrict__ msg,
                                                   unsigned long long* __restrict__ snz, uint32_t nsnz,
                                                   unsigned long long* __restrict__ live, uint32_t wact) {
    const uint64_t nft = (uint64_t)W * S, tot = nft + nsnz + wact;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < tot; i += (uint64_t)gridDim.x * 256u) {
        if (i < nft) {
            const uint32_t c = (uint32_t)(i / S), j = (uint32_t)(i - (uint64_t)c * S);
            if (j < Sr) FT[(uint64_t)c * kw + lo_w + j] = msg[i];
        } else {
            const uint64_t k = i - nft;
            const uint32_t* p = msg + nft + 2ull * k;
            const unsigned long long x = (unsigned long long)p[0] | ((unsigned long long)p[1] << 32);
            if (x) {
                if (k < nsnz) snz[k] |= x;
                else live[k - nsnz] |= x;
            }
        }
    }
}
