// Microbenchmark: throughput of the candidate 64-bit modular-multiply
// formulations on gfx950, plus an HBM streaming copy for the roofline.
// Used once to choose the NTT butterfly arithmetic.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int VPT = 8;     // independent values per thread
constexpr int ITERS = 256;

// Harvey/Shoup lazy butterfly: u,v in [0,2q) -> X,Y in [0,4q) then fold.
__global__ void k_int_shoup(uint64_t* out, uint64_t q, uint64_t w, uint64_t ws) {
    uint64_t v[VPT], u[VPT];
    uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < VPT; ++i) { v[i] = (tid * 7919u + i * 104729u) % q; u[i] = (tid + i) % q; }
    const uint64_t two_q = 2 * q;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            uint64_t hi = __umul64hi(v[i], ws);
            uint64_t t = v[i] * w - hi * q;          // [0,2q)
            uint64_t ur = u[i] >= two_q ? u[i] - two_q : u[i];
            uint64_t x = ur + t;
            uint64_t y = ur - t + two_q;
            u[i] = x; v[i] = y >= two_q ? y - two_q : y;
        }
    }
    uint64_t acc = 0;
    for (int i = 0; i < VPT; ++i) acc ^= u[i] ^ v[i];
    out[tid] = acc;
}

// FP64 butterfly on signed residues held exactly in doubles (q < 2^50).
__global__ void k_fp64(double* out, double q, double w, double wq) {
    double v[VPT], u[VPT];
    uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < VPT; ++i) { v[i] = (double)((tid * 7919u + i * 104729u) % (uint64_t)q); u[i] = (double)((tid + i) % (uint64_t)q); }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            double hi = v[i] * w;
            double lo = fma(v[i], w, -hi);
            double k = rint(v[i] * wq);
            double t = fma(-k, q, hi) + lo;       // ~(-q/2, q/2) + eps
            double x = u[i] + t;
            double y = u[i] - t;
            // keep bounded: fold x,y back to (-q/2.., ..) with one select each
            x = (x > 0.5 * q) ? x - q : x;
            y = (y < -0.5 * q) ? y + q : y;
            u[i] = x; v[i] = y;
        }
    }
    double acc = 0;
    for (int i = 0; i < VPT; ++i) acc += u[i] + v[i];
    out[tid] = acc;
}

// FP64 butterfly with magic-constant rounding instead of v_rndne_f64
__global__ void k_fp64_magic(double* out, double q, double w, double wq) {
    double v[VPT], u[VPT];
    uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < VPT; ++i) { v[i] = (double)((tid * 7919u + i * 104729u) % (uint64_t)q); u[i] = (double)((tid + i) % (uint64_t)q); }
    const double M = 6755399441055744.0;  // 1.5 * 2^52
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            double hi = v[i] * w;
            double lo = fma(v[i], w, -hi);
            double k = fma(v[i], wq, M) - M;
            double t = fma(-k, q, hi) + lo;
            double x = u[i] + t;
            double y = u[i] - t;
            x = (x > 0.5 * q) ? x - q : x;
            y = (y < -0.5 * q) ? y + q : y;
            u[i] = x; v[i] = y;
        }
    }
    double acc = 0;
    for (int i = 0; i < VPT; ++i) acc += u[i] + v[i];
    out[tid] = acc;
}

// plain FP64 CT butterfly without range folding (what the NTT kernel does between reductions)
__global__ void k_fp64_plain(double* out, double q, double w, double wq) {
    double v[VPT], u[VPT];
    uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < VPT; ++i) { v[i] = (double)((tid * 7919u + i * 104729u) % (uint64_t)q); u[i] = (double)((tid + i) % (uint64_t)q); }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            double hi = v[i] * w;
            double lo = fma(v[i], w, -hi);
            double k = rint(v[i] * wq);
            double t = fma(-k, q, hi) + lo;
            double x = u[i] + t;
            double y = u[i] - t;
            u[i] = y * 0.5; v[i] = x * 0.5;   // keep bounded, 1 op each
        }
    }
    double acc = 0;
    for (int i = 0; i < VPT; ++i) acc += u[i] + v[i];
    out[tid] = acc;
}

// 64-bit Montgomery butterfly (R = 2^64), lazy.
__global__ void k_int_mont(uint64_t* out, uint64_t q, uint64_t wm, uint64_t qinv_neg) {
    uint64_t v[VPT], u[VPT];
    uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < VPT; ++i) { v[i] = (tid * 7919u + i * 104729u) % q; u[i] = (tid + i) % q; }
    const uint64_t two_q = 2 * q;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int i = 0; i < VPT; ++i) {
            uint64_t lo = v[i] * wm;
            uint64_t hi = __umul64hi(v[i], wm);
            uint64_t m = lo * qinv_neg;
            uint64_t t = hi + __umul64hi(m, q) + (lo != 0);  // in [0,2q)
            uint64_t ur = u[i] >= two_q ? u[i] - two_q : u[i];
            uint64_t x = ur + t;
            uint64_t y = ur - t + two_q;
            u[i] = x; v[i] = y >= two_q ? y - two_q : y;
        }
    }
    uint64_t acc = 0;
    for (int i = 0; i < VPT; ++i) acc ^= u[i] ^ v[i];
    out[tid] = acc;
}

__global__ void k_copy(const ulonglong2* __restrict__ in, ulonglong2* __restrict__ out, size_t n2) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n2; i += stride) out[i] = in[i];
}

__global__ void k_read(const ulonglong2* __restrict__ in, uint64_t* out, size_t n2) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (; i < n2; i += stride) { ulonglong2 v = in[i]; acc ^= v.x ^ v.y; }
    if (acc == 0x12345) out[0] = acc;
}

int main() {
    const int threads = 256, blocks = 256 * 16;
    const size_t nthr = (size_t)threads * blocks;
    uint64_t* d_out; CHECK(hipMalloc(&d_out, nthr * 8));
    hipEvent_t a, b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    const uint64_t q = (1ULL << 49) + 123457;   // not prime; throughput only
    const uint64_t w = 0x1234567890ULL % q;
    const uint64_t ws = (uint64_t)(((unsigned __int128)w << 64) / q);
    const double bfl = (double)nthr * VPT * ITERS;
    float ms;
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(hipEventRecord(a));
        k_int_shoup<<<blocks, threads>>>(d_out, q, w, ws);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("int_shoup  butterflies/s = %.3e  (%.3f ms)\n", bfl / (ms * 1e-3), ms);
        CHECK(hipEventRecord(a));
        k_fp64<<<blocks, threads>>>((double*)d_out, (double)q, (double)w, (double)w / (double)q);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("fp64       butterflies/s = %.3e  (%.3f ms)\n", bfl / (ms * 1e-3), ms);
        CHECK(hipEventRecord(a));
        k_fp64_magic<<<blocks, threads>>>((double*)d_out, (double)q, (double)w, (double)w / (double)q);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("fp64_magic butterflies/s = %.3e  (%.3f ms)\n", bfl / (ms * 1e-3), ms);
        CHECK(hipEventRecord(a));
        k_fp64_plain<<<blocks, threads>>>((double*)d_out, (double)q, (double)w, (double)w / (double)q);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("fp64_plain butterflies/s = %.3e  (%.3f ms)\n", bfl / (ms * 1e-3), ms);
        CHECK(hipEventRecord(a));
        k_int_mont<<<blocks, threads>>>(d_out, q | 1, w, 0x9E3779B97F4A7C15ULL);
        CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("int_mont   butterflies/s = %.3e  (%.3f ms)\n", bfl / (ms * 1e-3), ms);
    }
    const size_t bytes = 4ULL << 30;
    void *d_in, *d_o2;
    CHECK(hipMalloc(&d_in, bytes)); CHECK(hipMalloc(&d_o2, bytes));
    CHECK(hipMemset(d_in, 1, bytes));
    for (int gb : {1024, 2048, 4096, 8192}) {
        for (int rep = 0; rep < 2; ++rep) {
            CHECK(hipEventRecord(a));
            k_copy<<<gb, 256>>>((const ulonglong2*)d_in, (ulonglong2*)d_o2, bytes / 16);
            CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
            CHECK(hipEventElapsedTime(&ms, a, b));
            printf("copy grid=%d 4GiB: %.1f GB/s (R+W)\n", gb, 2.0 * bytes / (ms * 1e-3) / 1e9);
            CHECK(hipEventRecord(a));
            k_read<<<gb, 256>>>((const ulonglong2*)d_in, d_out, bytes / 16);
            CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b));
            CHECK(hipEventElapsedTime(&ms, a, b));
            printf("read grid=%d 4GiB: %.1f GB/s\n", gb, 1.0 * bytes / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
