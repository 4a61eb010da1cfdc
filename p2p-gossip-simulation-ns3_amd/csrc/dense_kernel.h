// dense_kernel.h -- the dense-graph pull as an int8 MFMA contraction (GOSSIP_MODE_DENSE),
// included by engine.hip after pull_kernel.h.
//
// For p ~ 0.3 the per-tick gather of GossipShareToPeers (p2pnode.cc:127-153) is what it really
// is, an adjacency x frontier product:
//     Inc[v][c] = sum_u A[v][u] * F[u][c]        A = multiplicity of u in peers(v) in {0,1,2}
// run on v_mfma_i32_32x32x32_i8 with int32 accumulation, so Inc is the exact number of copies
// of share c reaching v this tick (duplicates included).  Each adjacency byte is reused across
// the 256 share columns of a block tile, which is why this beats streaming a frontier row per
// edge on dense graphs.
//
// Pipeline per tick: k_expand (frontier bitmap -> int8, column-major) -> k_dense_gemm (partial
// Inc over a K range; Inc > 0 ballots OR-ed into an incoming bitmap) -> k_pull in "incoming"
// mode (dedup, seen, counters, liveness; the same code as the sparse path).  Split-K is exact
// because partial sums are non-negative: Inc > 0 iff some partial is > 0.
//
// Operand maps (pinned on gfx950 by tools/mfma_probe.hip with exact integer data): lane l holds
// 16 int8 of A row (l&31) and of B column (l&31); the two lane halves (l>>5) hold the two
// 16-wide k halves (any k order shared by A and B gives the same product); C/D: lane l,
// register g -> row (g&3) + 8(g>>2) + 4(l>>5), column l&31.
//
// Tiling: block = 4 waves (2 x 2), output tile 128 rows x 256 columns (4 frontier words), wave
// tile 64 x 128 = 2 x 4 MFMA tiles (128 accumulator registers).  K advances 128 bytes per step
// through LDS rows padded to 144 B (16 lanes of a ds_read_b128 group hit 16 distinct 16-B slots:
// 9r mod 16 is a permutation).  The next step's global loads are issued before the current
// step's MFMAs (register prefetch) so HBM/L2 latency hides under 32 MFMAs per wave.
#pragma once

typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v16i_t __attribute__((ext_vector_type(16)));

struct GemmArgs {
    const int8_t* A8;   // n_pad x n_pad, row-major, multiplicities
    const int8_t* F8T;  // ncols x n_pad, column-major frontier (F8T[c * n_pad + u])
    unsigned long long* inc;  // n x stride incoming words (OR of Inc > 0)
    const unsigned long long* live_prev;  // nullable
    unsigned long long* acct;             // [5] += MAC ops x2, [6] += tiles skipped
    uint32_t n, n_pad, stride, ksplit;
};

// F (bitmap rows) -> F8T (int8, column-major).  Thread = (column c, 16 consecutive u).
__global__ __launch_bounds__(256) void k_expand(const uint64_t* __restrict__ F, uint32_t stride,
                                                uint32_t n, uint32_t n_pad, uint32_t ncols,
                                                const unsigned long long* live_prev,
                                                int8_t* __restrict__ F8T) {
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;
    const uint32_t u0 = blockIdx.y * 16u;
    if (c >= ncols) return;
    const uint32_t w = c >> 6, b = c & 63u;
    if (live_prev) {  // a 4-word GEMM column tile with no live word is skipped by the GEMM
        const uint32_t g = w & ~3u;
        if ((live_prev[g] | live_prev[g + 1] | live_prev[g + 2] | live_prev[g + 3]) == 0ull) return;
    }
    uint32_t out[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t u = u0 + i;
        const uint32_t bit = (u < n) ? (uint32_t)((F[(uint64_t)u * stride + w] >> b) & 1ull) : 0u;
        out[i >> 2] |= bit << (8 * (i & 3));
    }
    *reinterpret_cast<uint4*>(F8T + (uint64_t)c * n_pad + u0) = make_uint4(out[0], out[1], out[2], out[3]);
}

constexpr int kGRow = 144;  // padded LDS row (bytes) for a 128-byte k slice

__global__ __launch_bounds__(256, 2) void k_dense_gemm(GemmArgs a) {
    __shared__ __attribute__((aligned(16))) int8_t As[128 * kGRow];
    __shared__ __attribute__((aligned(16))) int8_t Bs[256 * kGRow];
    const uint32_t m0 = blockIdx.x * 128u;
    const uint32_t w0 = blockIdx.y * 4u;  // four frontier words = 256 columns
    const uint32_t t = threadIdx.x, lane = t & 63u, wid = t >> 6;
    const uint32_t wm = wid >> 1, wn = wid & 1u;
    if (a.live_prev) {
        const unsigned long long lv = a.live_prev[w0] | a.live_prev[w0 + 1] | a.live_prev[w0 + 2] |
                                      a.live_prev[w0 + 3];
        if (lv == 0ull) {
            if (t == 0 && a.acct) atomicAdd(&a.acct[6], 1ull);
            return;
        }
    }
    const uint32_t ksteps = a.n_pad / 128u;
    const uint32_t per = (ksteps + a.ksplit - 1u) / a.ksplit;
    const uint32_t kb = blockIdx.z * per, ke = min(ksteps, kb + per);
    if (kb >= ke) return;

    v16i_t acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = v16i_t{0};
    const uint32_t r = lane & 31u, h = lane >> 5;
    // tile loaders: A -- row t>>1, 64-byte half t&1 (4 x 16 B); B -- column t (8 x 16 B)
    const int8_t* Ag = a.A8 + (uint64_t)(m0 + (t >> 1)) * a.n_pad + (t & 1u) * 64u;
    const int8_t* Bg = a.F8T + (uint64_t)(w0 * 64u + t) * a.n_pad;
    int8_t* Aw = As + (t >> 1) * kGRow + (t & 1u) * 64u;
    int8_t* Bw = Bs + t * kGRow;
    uint4 ra[4], rb[8];
    {
        const uint64_t k0 = (uint64_t)kb * 128u;
#pragma unroll
        for (int q = 0; q < 4; q++) ra[q] = *reinterpret_cast<const uint4*>(Ag + k0 + 16 * q);
#pragma unroll
        for (int q = 0; q < 8; q++) rb[q] = *reinterpret_cast<const uint4*>(Bg + k0 + 16 * q);
    }
    for (uint32_t ks = kb; ks < ke; ks++) {
        __syncthreads();  // everyone finished reading the previous step's tiles
#pragma unroll
        for (int q = 0; q < 4; q++) *reinterpret_cast<uint4*>(Aw + 16 * q) = ra[q];
#pragma unroll
        for (int q = 0; q < 8; q++) *reinterpret_cast<uint4*>(Bw + 16 * q) = rb[q];
        __syncthreads();
        if (ks + 1u < ke) {  // prefetch the next step while this one computes
            const uint64_t k0 = (uint64_t)(ks + 1u) * 128u;
#pragma unroll
            for (int q = 0; q < 4; q++) ra[q] = *reinterpret_cast<const uint4*>(Ag + k0 + 16 * q);
#pragma unroll
            for (int q = 0; q < 8; q++) rb[q] = *reinterpret_cast<const uint4*>(Bg + k0 + 16 * q);
        }
#pragma unroll
        for (uint32_t kc = 0; kc < 4; kc++) {
            v4i_t af[2], bf[4];
#pragma unroll
            for (int i = 0; i < 2; i++)
                af[i] = *reinterpret_cast<const v4i_t*>(As + (wm * 64u + i * 32u + r) * kGRow + kc * 32u + 16u * h);
#pragma unroll
            for (int j = 0; j < 4; j++)
                bf[j] = *reinterpret_cast<const v4i_t*>(Bs + (wn * 128u + j * 32u + r) * kGRow + kc * 32u + 16u * h);
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
    }
    // ---- epilogue: Inc > 0 -> two 64-bit words per row (wave ballots), OR into inc ----
    uint64_t inc0 = 0ull, inc1 = 0ull;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int g = 0; g < 16; g++) {
            const unsigned long long q0 = __ballot(acc[i][0][g] > 0);
            const unsigned long long q1 = __ballot(acc[i][1][g] > 0);
            const unsigned long long q2 = __ballot(acc[i][2][g] > 0);
            const unsigned long long q3 = __ballot(acc[i][3][g] > 0);
            const uint32_t rowA = (uint32_t)i * 32u + (g & 3) + 8u * (g >> 2);  // lane half 0
            if (lane == rowA) {
                inc0 = (q0 & 0xffffffffull) | (q1 << 32);
                inc1 = (q2 & 0xffffffffull) | (q3 << 32);
            }
            if (lane == rowA + 4u) {  // lane half 1 rows sit 4 below
                inc0 = (q0 >> 32) | (q1 & 0xffffffff00000000ull);
                inc1 = (q2 >> 32) | (q3 & 0xffffffff00000000ull);
            }
        }
    if (t == 0 && a.acct) atomicAdd(&a.acct[5], 2ull * 128ull * 256ull * 128ull * (ke - kb));
    const uint64_t v = m0 + wm * 64u + lane;
    if (v >= a.n) return;
    unsigned long long* ip = a.inc + v * a.stride + w0 + wn * 2u;
    if (inc0) atomicOr(ip, (unsigned long long)inc0);
    if (inc1) atomicOr(ip + 1, (unsigned long long)inc1);
}
