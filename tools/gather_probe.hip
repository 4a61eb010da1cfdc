// gather_probe.hip -- achievable HBM rate for random row gathers of R bytes (R = 64 .. 2048),
// the access shape of k_pull's peer-row reads (R = 128: one 16-word tile row).
// Each wave-instruction reads 1 KiB: 1024/R rows of R bytes at hashed random row indices of a
// 4 GiB table; 8 instructions in flight per lane.  Prints GB/s per R.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int R>
__global__ __launch_bounds__(256) void gather(const uint4* __restrict__ tab, uint64_t nrows,
                                              uint32_t iters, uint4* __restrict__ out) {
    constexpr int LPR = R / 16;  // lanes per row
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (uint32_t it = 0; it < iters; it += 8) {
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t rid = hash32((uint32_t)(wave * 977u + (it + k) * 64u + lane / LPR)) % (uint32_t)nrows;
            q[k] = tab[(uint64_t)rid * LPR + (lane % LPR)];
        }
#pragma unroll
        for (int k = 0; k < 8; k++) { acc.x ^= q[k].x; acc.y ^= q[k].y; acc.z ^= q[k].z; acc.w ^= q[k].w; }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

template <int R>
void run(const uint4* tab, uint64_t bytes, uint4* out) {
    const uint64_t nrows = bytes / R;
    const uint32_t grid = 2048, iters = 512;
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    gather<R><<<grid, 256>>>(tab, nrows, iters, out);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) gather<R><<<grid, 256>>>(tab, nrows, iters, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    const double moved = 5.0 * grid * 4.0 * iters * 1024.0;
    printf("{\"table_gib\": %llu, \"row_bytes\": %d, \"GBps\": %.1f}\n", (unsigned long long)(nrows * R >> 30), R, moved / (ms * 1e6));
}

int main(int argc, char** argv) {
    // table size in GiB (default 4): random rows over ~100 GB behave like k_pull's frontier rows
    const uint64_t bytes = (uint64_t)(argc > 1 ? atoi(argv[1]) : 4) << 30;
    uint4* tab = nullptr;
    uint4* out = nullptr;
    if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(tab, 1, bytes);
    run<64>(tab, bytes, out);
    run<128>(tab, bytes, out);
    run<256>(tab, bytes, out);
    run<512>(tab, bytes, out);
    run<1024>(tab, bytes, out);
    hipFree(tab);
    hipFree(out);
    return 0;
}
