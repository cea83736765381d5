// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the NTT
// kernels use (8 B per lane, coalesced) against known byte counts (MI355X_MICROARCH.md: only 16 B/lane
// streaming is calibrated there).  Each kernel streams BYTES in and out of a 2 GiB buffer pair.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t BYTES = 2ull << 30;

__global__ void copy8(const unsigned long long* __restrict__ a, unsigned long long* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i] + 1;
}
__global__ void copy16(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        ulonglong2 v = a[i];
        v.x += 1;
        b[i] = v;
    }
}

int main() {
    void *a, *b;
    if (hipMalloc(&a, BYTES) || hipMalloc(&b, BYTES)) return 1;
    (void)hipMemset(a, 1, BYTES);
    (void)hipMemset(b, 0, BYTES);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        float ms8, ms16;
        (void)hipEventRecord(e0);
        copy8<<<8192, 256>>>((const unsigned long long*)a, (unsigned long long*)b, BYTES / 8);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms8, e0, e1);
        (void)hipEventRecord(e0);
        copy16<<<8192, 256>>>((const ulonglong2*)a, (ulonglong2*)b, BYTES / 16);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms16, e0, e1);
        std::printf("rep %d: copy8 %.3f ms (%.0f GB/s r+w), copy16 %.3f ms (%.0f GB/s)\n", rep, ms8,
                    2.0 * BYTES / ms8 / 1e6, ms16, 2.0 * BYTES / ms16 / 1e6);
    }
    std::printf("known bytes per dispatch: read %zu, write %zu\n", BYTES, BYTES);
    return 0;
}
