// mfma_i8_probe.hip -- check the A/B operand lane maps of v_mfma_i32_32x32x32_i8 on gfx950 with exact
// integer data (cdna_hip_programming.md: "other dtypes: check the map with exact integer data").
// Prints mismatch counts for candidate maps; the W-CRT MFMA GEMM uses the one that gives 0.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// k index of element j (0..15) of lane half h under map `m`
__host__ __device__ inline int kmap(int m, int h, int j) {
    switch (m) {
        case 0: return 16 * h + j;                                   // contiguous 16 per half
        case 1: return (j < 8) ? 8 * h + j : 16 + 8 * h + (j - 8);   // two 8-runs
        case 2: return 4 * h + (j & 3) + 8 * (j >> 2);               // 4-runs interleaved
        default: return 2 * j + h;                                   // interleaved
    }
}

__global__ void probe(const signed char* A, const signed char* B, int* C, int m) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    signed char a[16], b[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[r * 32 + kmap(m, h, j)];   // A[row][k]
        b[j] = B[kmap(m, h, j) * 32 + r];   // B[k][col]
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v16i c = {0};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
    for (int reg = 0; reg < 16; ++reg) {
        const int col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
        C[row * 32 + col] = c[reg];
    }
}

int main() {
    signed char hA[1024], hB[1024];
    srand(7);
    for (int i = 0; i < 1024; ++i) {
        hA[i] = (signed char)(rand() % 256 - 128);
        hB[i] = (signed char)(rand() % 256 - 128);
    }
    int ref[1024];
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            int s = 0;
            for (int k = 0; k < 32; ++k) s += hA[i * 32 + k] * hB[k * 32 + j];
            ref[i * 32 + j] = s;
        }
    signed char *dA, *dB;
    int* dC;
    if (hipMalloc(&dA, 1024) || hipMalloc(&dB, 1024) || hipMalloc(&dC, 4096)) return 1;
    (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    for (int m = 0; m < 4; ++m) {
        probe<<<1, 64>>>(dA, dB, dC, m);
        int hC[1024];
        (void)hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
        std::printf("k-map %d: %d / 1024 mismatches\n", m, bad);
    }
    return 0;
}
