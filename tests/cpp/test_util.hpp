// Small helpers shared by the C++ API programs (host-side checks only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(2);                                                                           \
        }                                                                                           \
    } while (0)

static int g_failures = 0;
#define EXPECT(cond, ...)                                    \
    do {                                                     \
        if (!(cond)) {                                       \
            std::printf("  [FAIL] %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                        \
            std::printf("\n");                               \
            ++g_failures;                                    \
        }                                                    \
    } while (0)

template <class T>
T* dev_alloc(size_t n) {
    T* p = nullptr;
    HIP_OK(hipMalloc(&p, n * sizeof(T)));
    return p;
}
template <class T>
std::vector<T> d2h(const T* d, size_t n) {
    std::vector<T> h(n);
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost));
    return h;
}
template <class T>
T* h2d(const std::vector<T>& h) {
    T* d = dev_alloc<T>(h.size());
    HIP_OK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}
static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((unsigned __int128)a * b % q); }
static inline uint64_t powmod(uint64_t a, uint64_t e, uint64_t q) {
    uint64_t r = 1;
    a %= q;
    for (; e; e >>= 1, a = mulmod(a, a, q))
        if (e & 1) r = mulmod(r, a, q);
    return r;
}
static inline uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
