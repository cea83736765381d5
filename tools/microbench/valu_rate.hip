// Microbenchmark: issue rate of single VALU instruction kinds on gfx950 (cycles per wave64 instruction per SIMD).
// Each thread runs 8 independent accumulator chains of one instruction through inline asm (so the compiler neither
// folds nor reorders them); 8 waves per SIMD hide the latency.  Cycles = wall time x the shader clock (s_memrealtime
// is the fixed 100 MHz counter, so the clock is taken from the measured ns and a nominal 2.4 GHz: the printed
// "cycles/inst" is an upper bound at 2.4 GHz and its ratios between kinds are what matter).
// Used for DESIGN.md §3.1 (U64: are the 32-bit integer multiplies quarter rate?).
// build: hipcc -O3 --offload-arch=gfx950 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);     \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

constexpr int ITERS = 2048;

enum Kind { ADD_U32, MUL_LO_U32, MUL_HI_U32, MAD_U64_U32, FMA_F64, ADD_F64, LSHL_ADD_U64, MUL_U32_U24, BFI_B32 };

template <int K>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b = seed ^ threadIdx.x;
    uint64_t a64[8];
    double d[8];
    const double dm = 1.0000001;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = seed + i * 7919u + threadIdx.x;
        a64[i] = ((uint64_t)a[i] << 20) ^ i;
        d[i] = (double)a[i];
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (K == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (K == MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (K == MUL_HI_U32) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (K == MAD_U64_U32) {
                uint64_t c;
                asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a64[i]), "=s"(c) : "v"(a[i]), "v"(b));
            }
            if constexpr (K == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[i]) : "v"(dm));
            if constexpr (K == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[i]) : "v"(dm));
            if constexpr (K == LSHL_ADD_U64) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a64[i]) : "v"(a64[(i + 1) & 7]));
            if constexpr (K == MUL_U32_U24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            if constexpr (K == BFI_B32) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(a[i]) : "v"(b));
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= a[i] ^ (uint32_t)a64[i] ^ (uint32_t)(a64[i] >> 32) ^ (uint32_t)(int64_t)d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int K>
static int run(const char* name, uint32_t* out, int cus) {
    const int blocks = cus * 8;   // 8 workgroups x 4 waves per CU = 8 waves per SIMD
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double wave_insts_per_simd = (double)reps * 8 /* waves per SIMD */ * ITERS * 8;
    const double cyc = ms * 1e-3 * 2.4e9 / wave_insts_per_simd;
    printf("{\"inst\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_inst_at_2.4GHz\": %.2f}\n", name, ms, cyc);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    CHECK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    printf("# %s, %d CUs, clockRate %d kHz\n", p.gcnArchName, cus, p.clockRate);
    run<ADD_U32>("v_add_u32", out, cus);
    run<MUL_LO_U32>("v_mul_lo_u32", out, cus);
    run<MUL_HI_U32>("v_mul_hi_u32", out, cus);
    run<MAD_U64_U32>("v_mad_u64_u32", out, cus);
    run<MUL_U32_U24>("v_mul_u32_u24", out, cus);
    run<BFI_B32>("v_bfi_b32", out, cus);
    run<LSHL_ADD_U64>("v_lshl_add_u64", out, cus);
    run<FMA_F64>("v_fma_f64", out, cus);
    run<ADD_F64>("v_add_f64", out, cus);
    CHECK(hipFree(out));
    return 0;
}
