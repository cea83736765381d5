// cache_bench: does the MI355X Infinity Cache (256 MiB) serve data written by a previous kernel?
// Decides the N = 2^16 NTT design (DESIGN.md §N=2^16): two passes with the intermediate re-read from
// cache vs from HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

__global__ void k_read(const ulonglong2* __restrict__ in, uint64_t* out, size_t n2) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (; i < n2; i += st) { ulonglong2 v = in[i]; acc ^= v.x ^ v.y; }
    if (acc == 0x12345) out[0] = acc;
}
__global__ void k_write(ulonglong2* __restrict__ o, size_t n2, uint64_t salt) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (; i < n2; i += st) o[i] = make_ulonglong2(i ^ salt, i + salt);
}
__global__ void k_rmw(ulonglong2* __restrict__ o, size_t n2) {   // read-modify-write in place
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
    for (; i < n2; i += st) { ulonglong2 v = o[i]; v.x += 1; v.y ^= 3; o[i] = v; }
}
// Same-CU write-then-read: each block owns a contiguous `per_block` byte slab; it writes it, barriers,
// and reads it back (possibly several times) -- the fused one-workgroup-per-polynomial pattern.
__global__ void k_slab(ulonglong2* __restrict__ buf, size_t per_block16, int rounds, uint64_t* out) {
    ulonglong2* s = buf + blockIdx.x * per_block16;
    uint64_t acc = 0;
    for (size_t i = threadIdx.x; i < per_block16; i += blockDim.x) { ulonglong2 v = s[i]; acc += v.x; s[i] = make_ulonglong2(v.x + 1, v.y); }
    for (int r = 0; r < rounds; ++r) {
        __syncthreads();
        for (size_t i = threadIdx.x; i < per_block16; i += blockDim.x) { ulonglong2 v = s[i]; acc += v.y; s[i] = make_ulonglong2(v.x, v.y + acc); }
    }
    if (acc == 0x12345) out[0] = acc;
}

int main() {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    const size_t big = 4ULL << 30;
    void *buf, *flush;
    uint64_t* dout;
    CHECK(hipMalloc(&buf, big)); CHECK(hipMalloc(&flush, big)); CHECK(hipMalloc(&dout, 64));
    CHECK(hipMemset(buf, 1, big)); CHECK(hipMemset(flush, 2, big));
    const int G = 2048, T = 256;
    float ms;
    auto doflush = [&]() { k_read<<<G, T>>>((const ulonglong2*)flush, dout, (1ULL << 30) / 16); };
    for (size_t mib : {16, 32, 64, 96, 128, 192, 256, 384, 1024, 4096}) {
        const size_t S = mib << 20, n2 = S / 16;
        // read after read
        doflush();
        k_read<<<G, T>>>((const ulonglong2*)buf, dout, n2);
        CHECK(hipEventRecord(a));
        k_read<<<G, T>>>((const ulonglong2*)buf, dout, n2);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); CHECK(hipEventElapsedTime(&ms, a, b));
        double rr = S / (ms * 1e-3) / 1e9;
        // read after write
        doflush();
        k_write<<<G, T>>>((ulonglong2*)buf, n2, mib);
        CHECK(hipEventRecord(a));
        k_read<<<G, T>>>((const ulonglong2*)buf, dout, n2);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); CHECK(hipEventElapsedTime(&ms, a, b));
        double rw = S / (ms * 1e-3) / 1e9;
        // rmw after rmw (two-pass NTT pattern); report 2nd pass R+W bandwidth
        doflush();
        CHECK(hipEventRecord(a));
        k_rmw<<<G, T>>>((ulonglong2*)buf, n2);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); CHECK(hipEventElapsedTime(&ms, a, b));
        double r1 = 2.0 * S / (ms * 1e-3) / 1e9;
        CHECK(hipEventRecord(a));
        k_rmw<<<G, T>>>((ulonglong2*)buf, n2);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); CHECK(hipEventElapsedTime(&ms, a, b));
        double r2 = 2.0 * S / (ms * 1e-3) / 1e9;
        printf("%5zu MiB: read-after-read %7.0f GB/s | read-after-write %7.0f GB/s | rmw#1 %7.0f rmw#2 %7.0f GB/s (R+W)\n",
               mib, rr, rw, r1, r2);
    }
    // fused slab pattern: 4 GiB total in slabs of 512 KiB per block, 1..2 rounds of re-read
    for (size_t slab_kib : {128, 256, 512}) {
        for (int blocks_per_launch : {256, 512, 1024}) {
            const size_t per16 = (slab_kib << 10) / 16;
            const size_t nslab = big / (slab_kib << 10);
            CHECK(hipEventRecord(a));
            for (size_t s0 = 0; s0 < nslab; s0 += blocks_per_launch)
                k_slab<<<blocks_per_launch, 1024>>>((ulonglong2*)buf + s0 * per16, per16, 1, dout);
            CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); CHECK(hipEventElapsedTime(&ms, a, b));
            printf("slab %zu KiB x %d blocks/launch: 2 R+W passes over 4 GiB in %.3f ms = %.0f GB/s algorithmic(1R+1W)\n",
                   slab_kib, blocks_per_launch, ms, 2.0 * big / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
