// mfma_probe.hip -- pin the operand/result lane maps of v_mfma_i32_32x32x32_i8 on gfx950 with
// exact integer data (the guide documents bf16 maps only).  Prints which hypothesis matches.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_probe.hip -o /tmp/mfma_probe && /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// Hypothesis k-map for the 16 bytes lane l holds: k = kmap(h, j), h = l >> 5, j = 0..15.
__host__ __device__ inline int kmap(int hyp, int h, int j) {
    if (hyp == 0) return 16 * h + j;                                  // contiguous halves
    if (hyp == 1) return (j < 8) ? (8 * h + j) : (16 + 8 * h + (j - 8));  // interleaved by 8
    return 2 * j + h;                                                  // interleaved by 1
}

__global__ void probe(const signed char* A, const signed char* B, int* C, int hyp) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    signed char a[16], b[16];
    for (int j = 0; j < 16; j++) {
        const int k = kmap(hyp, h, j);
        a[j] = A[r * 32 + k];   // A[row r][k]
        b[j] = B[k * 32 + r];   // B[k][col r]
    }
    v4i av, bv;
    memcpy(&av, a, 16);
    memcpy(&bv, b, 16);
    v16i acc = {0};
    acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
    for (int g = 0; g < 16; g++) {
        const int row = (g & 3) + 8 * (g >> 2) + 4 * h;  // dtype-independent C/D map
        C[row * 32 + r] = acc[g];
    }
}

int main() {
    signed char hA[1024], hB[1024];
    srand(7);
    for (int i = 0; i < 1024; i++) {
        hA[i] = (signed char)(rand() % 3);
        hB[i] = (signed char)(rand() % 2);
    }
    int ref[1024];
    for (int i = 0; i < 32; i++)
        for (int j = 0; j < 32; j++) {
            int s = 0;
            for (int k = 0; k < 32; k++) s += hA[i * 32 + k] * hB[k * 32 + j];
            ref[i * 32 + j] = s;
        }
    signed char *dA, *dB;
    int* dC;
    if (hipMalloc(&dA, 1024) || hipMalloc(&dB, 1024) || hipMalloc(&dC, 4096)) return 1;
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    for (int hyp = 0; hyp < 3; hyp++) {
        hipMemset(dC, 0, 4096);
        probe<<<1, 64>>>(dA, dB, dC, hyp);
        int hC[1024];
        hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 1024; i++) bad += hC[i] != ref[i];
        printf("hypothesis %d: %d/1024 mismatches\n", hyp, bad);
    }
    return 0;
}
