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
    const uint32_t chunk = blockIdx.x * 4u + (threadIdx.x >> 6);  // 64-node chunk
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
            if (t == 0 && a.acct) atomicAdd(&a.acct[6], 1ull);
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
        atomicAdd(&a.acct[5], 2ull * kDenseTile * kDenseTile * kStageK * computed);
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
