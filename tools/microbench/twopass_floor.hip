// twopass_floor: the memory schedule of the C3 forward NTT (N = 2^16, L = 8, batch 1024 = 4 GiB in place, two
// passes per 228 MiB chunk) with the butterflies removed -- what any two-pass plan on this chip can reach at
// best, next to the one-pass floor (every byte read once and written once: the 16N the roofline counts).
//
//   A  two passes per chunk with the NTT's own access patterns: a column pass (16-column x 256-row tiles, one
//      column per lane group, plain loads / plain stores: the intermediate stays in the Infinity Cache) then a
//      block pass (16 contiguous 256-element rows per workgroup, plain loads / sc1 nt stores), each lane moving
//      16 words, persistent grids with the XCD-contiguous tile order the NTT uses (no LDS, no DMA)
//   B  two passes per chunk as contiguous 16-B in-place read-modify-write sweeps (the same bytes, the
//      friendliest order)
//   C  one contiguous in-place read-modify-write sweep over the whole 4 GiB (the single-pass floor)
//
// Each line: ms per 4 GiB "transform", the equivalent forward-NTT/s at C3 (8192 NTTs per call) and the
// roofline fraction the bench line would report for it (16N bytes per NTT / 8 TB/s).  Data values are
// perturbed so no pass can be skipped; nothing is checked.  Build: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) {                                                                    \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);          \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

constexpr int LOGN = 16, NPOLY = 8192, NCHUNK = 18;
constexpr uint64_t N = 1ull << LOGN;

// blockIdx -> tile, XCD-aware as the NTT's xcd_remap: workgroups are dispatched round-robin over the 8 XCDs, so
// logical tile l runs on XCD l % 8; give each XCD a contiguous run of tiles (nb % 8 == 0 here)
__device__ __forceinline__ uint32_t xcd_tile(uint32_t l, uint32_t nb) { return (l & 7) * (nb >> 3) + (l >> 3); }

// column pass: tile = 16 columns x 256 rows of one polynomial (256 x 256 view), 256 threads: lane group gl =
// t % 16 (column), tau = t / 16 owns rows tau * 16 + k -- the NTT's round-1 store layout; persistent grid
__global__ __launch_bounds__(256) void col_pass(uint64_t* d, uint32_t ntiles) {
    const uint32_t gl = threadIdx.x & 15, tau = threadIdx.x >> 4;
    for (uint32_t l = blockIdx.x; l < ntiles; l += gridDim.x) {
        const uint32_t tile = xcd_tile(l, ntiles);
        const uint32_t poly = tile >> 4, ct = tile & 15;
        uint64_t* base = d + ((uint64_t)poly << LOGN) + ct * 16 + gl;
        uint64_t x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = base[(uint64_t)(tau * 16 + k) << 8];
#pragma unroll
        for (int k = 0; k < 16; ++k) base[(uint64_t)(tau * 16 + k) << 8] = x[k] + 1;
    }
}

// block pass: 16 contiguous 256-element rows per 256-thread workgroup (4 per wave), element k * 16 + tau of row
// gl, outputs stored sc1 nt as the NTT's final stores; persistent grid
__global__ __launch_bounds__(256) void blk_pass(uint64_t* d, uint32_t ntiles) {
    const uint32_t gl = threadIdx.x >> 4, tau = threadIdx.x & 15;
    for (uint32_t l = blockIdx.x; l < ntiles; l += gridDim.x) {
        const uint32_t tile = xcd_tile(l, ntiles);
        uint64_t* row = d + ((uint64_t)tile * 16 + gl) * 256 + tau;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row, 0, 0x7FFFFFFF, 0x00020000);
        uint64_t x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = row[k * 16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, x[k] ^ 3), rs, k * 16 * 8, 0, 18);
    }
}

// contiguous in-place read-modify-write, 16 B per lane, grid-stride
__global__ __launch_bounds__(256) void rmw(ulonglong2* o, size_t n16, int nt) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t st = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += st) {
        ulonglong2 v = o[i];
        v.x += 1;
        v.y ^= 3;
        if (nt) {   // non-temporal, as the NTT's final stores (which are sc1 nt)
            __builtin_nontemporal_store(v.x, &o[i].x);
            __builtin_nontemporal_store(v.y, &o[i].y);
        } else {
            o[i] = v;
        }
    }
}

int main() {
    const size_t bytes = (size_t)NPOLY * N * 8;
    uint64_t* d;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(d, 1, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const uint32_t cb = (NPOLY + NCHUNK - 1) / NCHUNK;   // 456 polys = 228 MiB, the NTT's equal chunks
    auto variant_a = [&]() {
        for (uint32_t p0 = 0; p0 < NPOLY; p0 += cb) {
            const uint32_t np = p0 + cb <= NPOLY ? cb : NPOLY - p0;
            hipLaunchKernelGGL(col_pass, dim3(512), dim3(256), 0, 0, d + (uint64_t)p0 * N, np * 16);
            hipLaunchKernelGGL(blk_pass, dim3(2048), dim3(256), 0, 0, d + (uint64_t)p0 * N, np * 16);
        }
    };
    auto variant_b = [&]() {
        for (uint32_t p0 = 0; p0 < NPOLY; p0 += cb) {
            const uint32_t np = p0 + cb <= NPOLY ? cb : NPOLY - p0;
            const size_t n16 = (size_t)np * N / 2;
            hipLaunchKernelGGL(rmw, dim3(2048), dim3(256), 0, 0, (ulonglong2*)(d + (uint64_t)p0 * N), n16, 0);
            hipLaunchKernelGGL(rmw, dim3(2048), dim3(256), 0, 0, (ulonglong2*)(d + (uint64_t)p0 * N), n16, 1);
        }
    };
    auto variant_c = [&]() { hipLaunchKernelGGL(rmw, dim3(2048), dim3(256), 0, 0, (ulonglong2*)d, bytes / 16, 1); };
    for (int rep = 0; rep < 2; ++rep) {
        for (int vi = 0; vi < 3; ++vi) {
            const char* name = vi == 0 ? "A two-pass, NTT access patterns (column 16x256 tiles, 4-row block tiles)"
                               : vi == 1 ? "B two-pass, contiguous in-place sweeps"
                                         : "C one-pass, contiguous in-place sweep (the 16N floor)";
            auto run = [&]() {
                if (vi == 0) variant_a();
                else if (vi == 1) variant_b();
                else variant_c();
            };
            for (int w = 0; w < 5; ++w) run();
            CHECK(hipDeviceSynchronize());
            const int iters = 20;
            CHECK(hipEventRecord(e0));
            for (int it = 0; it < iters; ++it) run();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= iters;
            const double ntt_s = NPOLY / (ms * 1e-3);   // 8192 NTTs (1024 polys x 8 limbs) per 4 GiB
            const double alg = 16.0 * N * ntt_s / 1e9;  // GB/s algorithmic (8N read + 8N write per NTT)
            printf("{\"rep\": %d, \"variant\": \"%s\", \"ms_per_4GiB\": %.4f, \"equiv_fwd_NTT_per_s\": %.0f, "
                   "\"equiv_frac\": %.4f, \"fabric_GBps\": %.1f}\n",
                   rep, name, ms, ntt_s, alg / 8000.0, (vi == 2 ? 2.0 : 4.0) * bytes / (ms * 1e-3) / 1e9);
        }
    }
    CHECK(hipFree(d));
    return 0;
}
