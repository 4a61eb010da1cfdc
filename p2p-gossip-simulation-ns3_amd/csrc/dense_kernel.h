// dense_kernel.h -- the dense-graph pull as an int8 MFMA contraction (GOSSIP_MODE_DENSE),
// included by engine.hip after pull_kernel.h.
//
// For p ~ 0.3 the per-tick gather of GossipShareToPeers (p2pnode.cc:127-153) is what it really
// is, an adjacency x frontier product:
//     Inc[v][c] = sum_u A[v][u] * F[u][c]        A = multiplicity of u in peers(v) in {0,1,2}
// run on v_mfma_i32_32x32x32_i8 with int32 accumulation, so Inc is the exact number of copies
// of share c that reach v this tick (duplicates included).  The epilogue turns Inc > 0 into a
// frontier word with a wave ballot and applies the same dedup / counter / liveness logic as
// k_pull.
//
// Operand maps (pinned on gfx950 by tools/mfma_probe.hip with exact integer data): lane l holds
// 16 int8 of A row (l&31) and of B column (l&31); the two lane halves (l>>5) hold the two
// 16-wide k halves (any k order shared by A and B gives the same product); C/D: lane l,
// register g -> row (g&3) + 8(g>>2) + 4(l>>5), column l&31.
//
// Tiling: block = 4 waves, output tile 128 rows x 128 columns (= 2 frontier words); each wave
// owns 64 x 64 (2 x 2 MFMA tiles).  K advances 64 per step through LDS tiles whose rows are
// padded to 80 B (conflict-free ds_read_b128: 16 lanes of a group hit 16 distinct 16-B slots).
#pragma once

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

struct DenseArgs {
    const int8_t* A8;      // n_pad x n_pad, row-major, multiplicities
    const int8_t* F8T;     // ncols x n_pad, column-major frontier (F8T[c * n_pad + u])
    const uint32_t* deg;
    uint64_t* Fnext;
    uint64_t* seen;
    const WordCtl* ctl;
    const uint8_t* wflags;
    uint32_t* recv;
    uint64_t* sent;
    unsigned long long* live;
    const unsigned long long* live_prev;
    const unsigned long long* live_pp;
    unsigned long long* snap;
    unsigned long long* acct;  // [5] = tiles computed, [6] = tiles skipped
    uint32_t n, n_pad, stride, wact;
};

// F (bitmap rows) -> F8T (int8, column-major).  Thread = (column c, 16 consecutive u).
__global__ __launch_bounds__(256) void k_expand(const uint64_t* __restrict__ F, uint32_t stride,
                                                uint32_t n, uint32_t n_pad, uint32_t ncols,
                                                int8_t* __restrict__ F8T) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    const uint32_t u0 = blockIdx.y * 16u;
    if (c >= ncols) return;
    const uint32_t w = c >> 6, b = c & 63u;
    uint32_t out[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t u = u0 + i;
        const uint32_t bit = (u < n) ? (uint32_t)((F[(uint64_t)u * stride + w] >> b) & 1ull) : 0u;
        out[i >> 2] |= bit << (8 * (i & 3));
    }
    *reinterpret_cast<uint4*>(F8T + (uint64_t)c * n_pad + u0) = make_uint4(out[0], out[1], out[2], out[3]);
}

constexpr int kDRow = 80;  // padded LDS row (bytes) for a 64-byte k slice

__global__ __launch_bounds__(256) void k_dense_pull(DenseArgs a) {
    __shared__ __attribute__((aligned(16))) int8_t As[128 * kDRow];
    __shared__ __attribute__((aligned(16))) int8_t Bs[128 * kDRow];
    const uint32_t m0 = blockIdx.x * 128u;
    const uint32_t w0 = blockIdx.y * 2u;  // the two frontier words of this column tile
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
    const uint32_t wm = wid >> 1, wn = wid & 1u;
    const uint64_t stride = a.stride;
    const unsigned long long lp0 = a.live_prev ? a.live_prev[w0] : ~0ull;
    const unsigned long long lp1 = a.live_prev ? a.live_prev[w0 + 1] : ~0ull;
    const bool pp_dirty = a.live_pp ? ((a.live_pp[w0] | a.live_pp[w0 + 1]) != 0ull) : true;
    const uint16_t fl = *reinterpret_cast<const uint16_t*>(a.wflags + w0);

    if ((lp0 | lp1) == 0ull) {
        // nothing can arrive in these two words: only seen resets / stale F_next words
        if (t < 128u) {
            const uint64_t v = m0 + t;
            if (v < a.n) {
                uint64_t* sp = a.seen + v * stride + w0;
                uint64_t* fp = a.Fnext + v * stride + w0;
                if (fl & WF_CLEAR) sp[0] = 0ull;
                if ((fl >> 8) & WF_CLEAR) sp[1] = 0ull;
                if (pp_dirty) *reinterpret_cast<ulonglong2*>(fp) = make_ulonglong2(0ull, 0ull);
            }
        }
        if (t == 0 && a.acct) atomicAdd(&a.acct[6], 1ull);
        return;
    }

    v16i_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = v16i_t{0};
    const uint32_t r = lane & 31u, h = lane >> 5;
    const uint32_t lrow = t >> 1, lhalf = t & 1u;  // tile loader: row/col and 32-byte half
    const int8_t* Ag = a.A8 + (uint64_t)(m0 + lrow) * a.n_pad + lhalf * 32u;
    const int8_t* Bg = a.F8T + (uint64_t)(w0 * 64u + lrow) * a.n_pad + lhalf * 32u;
    for (uint32_t k0 = 0; k0 < a.n_pad; k0 += 64u) {
        const uint4 a0 = *reinterpret_cast<const uint4*>(Ag + k0);
        const uint4 a1 = *reinterpret_cast<const uint4*>(Ag + k0 + 16);
        const uint4 b0 = *reinterpret_cast<const uint4*>(Bg + k0);
        const uint4 b1 = *reinterpret_cast<const uint4*>(Bg + k0 + 16);
        __syncthreads();  // previous step's fragment reads are done
        *reinterpret_cast<uint4*>(As + lrow * kDRow + lhalf * 32u) = a0;
        *reinterpret_cast<uint4*>(As + lrow * kDRow + lhalf * 32u + 16) = a1;
        *reinterpret_cast<uint4*>(Bs + lrow * kDRow + lhalf * 32u) = b0;
        *reinterpret_cast<uint4*>(Bs + lrow * kDRow + lhalf * 32u + 16) = b1;
        __syncthreads();
#pragma unroll
        for (uint32_t kc = 0; kc < 2; kc++) {
            v4i_t af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; i++) {
                af[i] = *reinterpret_cast<const v4i_t*>(As + (wm * 64u + i * 32u + r) * kDRow + kc * 32u + 16u * h);
                bf[i] = *reinterpret_cast<const v4i_t*>(Bs + (wn * 64u + i * 32u + r) * kDRow + kc * 32u + 16u * h);
            }
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
    }

    // ---- epilogue: Inc > 0 -> one 64-bit frontier word per row (ballots across the wave) ----
    uint64_t inc = 0ull;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int g = 0; g < 16; g++) {
            const unsigned long long q0 = __ballot(acc[i][0][g] > 0);
            const unsigned long long q1 = __ballot(acc[i][1][g] > 0);
            const uint32_t rowA = (uint32_t)i * 32u + (g & 3) + 8u * (g >> 2);  // lane half 0
            const uint64_t wa = (q0 & 0xffffffffull) | (q1 << 32);
            const uint64_t wb = (q0 >> 32) | (q1 & 0xffffffff00000000ull);   // row rowA + 4
            if (lane == rowA) inc = wa;
            if (lane == rowA + 4u) inc = wb;
        }
    const uint64_t v = m0 + wm * 64u + lane;
    const uint32_t w = w0 + wn;
    const uint32_t f = wn ? (fl >> 8) : (fl & 0xffu);
    const unsigned long long lp = wn ? lp1 : lp0;
    if (t == 0 && a.acct) atomicAdd(&a.acct[5], 1ull);
    if (v >= a.n) return;
    uint64_t* sp = a.seen + v * stride + w;
    uint64_t* fp = a.Fnext + v * stride + w;
    if (lp == 0ull) {  // this word of the pair is dead
        if (f & WF_CLEAR) *sp = 0ull;
        if (pp_dirty) *fp = 0ull;
        return;
    }
    uint64_t s = (f & WF_CLEAR) ? 0ull : *sp;
    const uint64_t keep = (f & WF_KEEP) ? a.ctl[w].keep : ~0ull;
    uint64_t nw = inc & ~s & keep;
    if (f & WF_GROUP) nw = group_fix(nw, s, a.ctl[w].gmask, a.ctl[w].gstart);
    if (nw || (f & WF_CLEAR)) *sp = s | nw;
    if (nw || pp_dirty) *fp = nw;
    if (nw) {
        const uint32_t c = (uint32_t)__popcll(nw);
        atomicAdd(&a.recv[v], c);
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.sent[v]), (unsigned long long)c * a.deg[v]);
        atomicOr(&a.live[w], (unsigned long long)nw);
        if (a.snap && (f & WF_SNAP)) atomicAdd(a.snap, (unsigned long long)__popcll(nw & a.ctl[w].snap));
    }
}
