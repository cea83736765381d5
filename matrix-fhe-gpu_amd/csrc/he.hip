// he.hip -- W-axis transforms, XY encoder transforms, layouts, samplers and the
// encode / keygen / encrypt / decrypt / decode pipelines at reference geometry.
//
// Reference: src/core/HE.cu (W-CRT 437-470, 716-781, 1029-1114, 1245-1270; samplers 564-627,
// 690-713; ring ops 509-560; layouts 1330-1368; pipelines 1272-1307, 1370-1708),
// src/core/batched_encoder.cu:161-228, src/core/encoder.cu:425-501.
//
// Differences by design (results identical): one batched launch instead of per-lane launch loops
// (batched_encoder.cu:192-196, HE.cu:1653-1668, 1676-1679); no per-call malloc/free (a context
// workspace instead); the W-CRT output is written straight into the layout the caller needs;
// CRT compose and f64/delta are fused.
#include <hip/hip_runtime.h>

#include <cmath>

#include "gemm.hpp"
#include "mfhe_ctx.hpp"
#include "ring_row.hpp"

extern "C" int mfhe_ntt_fwd(mfhe_ctx*, uint64_t*, size_t, int, int, mfhe_stream_t);
extern "C" int mfhe_ntt_inv(mfhe_ctx*, uint64_t*, size_t, int, int, mfhe_stream_t);
extern "C" int mfhe_crt_compose(mfhe_ctx*, const uint64_t*, size_t, size_t, uint64_t*, uint8_t*, mfhe_stream_t);
extern "C" int mfhe_crt_compose_f64(mfhe_ctx*, const uint64_t*, size_t, size_t, double*, size_t, mfhe_stream_t);
namespace mfhe {
int crt_compose_f64_pair(mfhe_ctx*, const uint64_t*, const uint64_t*, size_t, size_t, double*, double*, size_t, hipStream_t);
}
extern "C" int mfhe_rns_decompose(mfhe_ctx*, const double*, size_t, size_t, size_t, uint64_t*, mfhe_stream_t);

namespace mfhe {

static inline dim3 g1(uint64_t total, uint32_t th = 256) { return dim3((uint32_t)((total + th - 1) / th)); }

// ---------------- layouts: HE.cu:1330-1368 ----------------
template <bool TO_POLY>
__global__ void layout_kernel(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, int log_n, int L,
                              uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;   // matrix-major index
    if (i >= total) return;
    const uint64_t n = 1ull << log_n, n2 = n * n;
    const uint64_t x = i & (n - 1), y = (i >> log_n) & (n - 1);
    const uint32_t wl = (uint32_t)(i >> (2 * log_n)), w = wl / (uint32_t)L, l = wl - w * (uint32_t)L;   // wl < 2^32
    const uint64_t p = (((uint64_t)w * n + y) * L + l) * n + x;
    (void)n2;
    if (TO_POLY) out[p] = in[i];
    else out[i] = in[p];
}

// ---------------- samplers (deterministic in the element index) ----------------
// ternary_secret_kernel HE.cu:690-713, [phi][L][n]
__global__ void ternary_kernel(uint64_t* s, const uint64_t* qmu, int L, int log_n, uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint64_t n = 1ull << log_n, single = (uint64_t)L * n;
    const uint64_t off = idx % single;
    const int limb = (int)(off >> log_n);
    const uint64_t coeff = off & (n - 1), poly = idx / single;
    const uint64_t t = poly * 1315423911ULL + coeff * 2654435761ULL;
    const int r = (int)((t * 11400714819323198485ULL) % 3ULL);
    const uint64_t q = qmu[2 * limb];
    s[idx] = (r == 0) ? 0 : (r == 1) ? 1 : q - 1;
}

// uniform_random_kernel HE.cu:564-578, matrix-major [phi][L][n*n].  The seed is the element's index in the
// WHOLE parameter set ([phi][Ltot][n*n], this context's limb l being global limb lbase + l), so a residue
// shard (mfhe_ctx_set_limb_shard) draws exactly its limbs of the unsharded a.
__global__ void uniform_kernel(uint64_t* a, const uint64_t* qmu, int L, int log_n, uint64_t total, int lbase, int Ltot) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint64_t n2 = 1ull << (2 * log_n), pos = idx & (n2 - 1);
    const uint32_t wl = (uint32_t)(idx >> (2 * log_n)), w = wl / (uint32_t)L;   // wl < 2^32: 32-bit division
    const int limb = (int)(wl - w * (uint32_t)L);
    uint64_t seed = 123456789ULL + (((uint64_t)w * (uint64_t)Ltot + (uint64_t)(lbase + limb)) << (2 * log_n)) + pos;
    seed = seed * 6364136223846793005ULL + 1442695040888963407ULL;
    // seed % q by Barrett (mu = floor(2^64 / q)): the quotient estimate is at most 2 low, so r < 3q
    const uint64_t q = qmu[2 * limb], mu = qmu[2 * limb + 1];
    uint64_t r = seed - __umul64hi(seed, mu) * q;
    r = r >= q ? r - q : r;
    a[idx] = r >= q ? r - q : r;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// gaussian_noise_kernel HE.cu:581-627: one centred sample per [w][y][x], same integer in every limb.
// One thread per sample (the reference draws it once per limb), written to all L limbs.
__global__ void gaussian_kernel(uint64_t* e, const uint64_t* qmu, int L, int log_n, uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint64_t n2 = 1ull << (2 * log_n);
    const uint64_t w = idx >> (2 * log_n), pos = idx & (n2 - 1);
    const uint64_t r1 = splitmix64(0xD6E8FEB86659FD93ULL ^ (w * n2 + pos));
    const uint64_t r2 = splitmix64(r1);
    const double inv53 = 1.0 / 9007199254740992.0;
    const double u1 = ((double)(r1 >> 11) + 1.0) * inv53;
    const double u2 = ((double)(r2 >> 11) + 1.0) * inv53;
    const double mag = 3.2 * sqrt(-2.0 * log(u1));
    const double z = mag * cos(6.283185307179586 * u2);
    const long long nz = llround(z);
    uint64_t* out = e + w * L * n2 + pos;
    for (int limb = 0; limb < L; ++limb) {
        const uint64_t q = qmu[2 * limb];
        out[(uint64_t)limb * n2] = (nz >= 0) ? (uint64_t)nz : q - (uint64_t)(-nz);
    }
}

// The same draw as gaussian_kernel, once per [w][y][x] as a centred integer in a double: the factored W-CRT's
// digitize reads it for every limb (gemm.hip FoldSrc, qsrc 3), so the L-limb residue array never reaches HBM.
__global__ void gaussian_compact_kernel(double* e, int log_n, uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint64_t n2 = 1ull << (2 * log_n);
    const uint64_t w = idx >> (2 * log_n), pos = idx & (n2 - 1);
    const uint64_t r1 = splitmix64(0xD6E8FEB86659FD93ULL ^ (w * n2 + pos));
    const uint64_t r2 = splitmix64(r1);
    const double inv53 = 1.0 / 9007199254740992.0;
    const double u1 = ((double)(r1 >> 11) + 1.0) * inv53;
    const double u2 = ((double)(r2 >> 11) + 1.0) * inv53;
    const double mag = 3.2 * sqrt(-2.0 * log(u1));
    const double z = mag * cos(6.283185307179586 * u2);
    e[idx] = (double)llround(z);
}

// The same draw once more, written as the one signed digit of e in the dense W-CRT GEMM's B layout (k-panel-major
// [512 / 32][P][32] bytes, k = w, p = pos; gemm.hip mod_gemm_mfma_smallb_kernel), shared by every limb: |e| <= 27
// (u1 >= 2^-53), so the int8 holds e exactly.  One thread per 4 consecutive k of one position (a 4-byte store), the
// 8 threads of a position's 32-k panel row adjacent: every wave writes 2 KiB contiguous.
__global__ void gaussian_i8_kernel(int8_t* __restrict__ b8, int log_n, uint32_t P) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;   // (panel, pos, k group of 4)
    if (idx >= 128ull * P) return;
    const uint64_t row = idx >> 3;                                          // panel * P + pos
    const uint32_t pos = (uint32_t)(row % P), k0 = (uint32_t)(row / P) * 32 + (uint32_t)(idx & 7) * 4;
    const uint64_t n2 = 1ull << (2 * log_n);
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t w = k0 + j;
        const uint64_t r1 = splitmix64(0xD6E8FEB86659FD93ULL ^ (w * n2 + pos));
        const uint64_t r2 = splitmix64(r1);
        const double inv53 = 1.0 / 9007199254740992.0;
        const double u1 = ((double)(r1 >> 11) + 1.0) * inv53;
        const double u2 = ((double)(r2 >> 11) + 1.0) * inv53;
        const double mag = 3.2 * sqrt(-2.0 * log(u1));
        const double z = mag * cos(6.283185307179586 * u2);
        word |= (uint32_t)(uint8_t)(int8_t)llround(z) << (8 * j);
    }
    *(uint32_t*)(b8 + row * 32 + (k0 & 31)) = word;
}

// ---------------- ring ops (poly-major [phi*n][L][n]) ----------------
// pointwise_mul_s_kernel HE.cu:509-531: t = a * s[w][l][x], w = poly / n.  The reference reduces with
// an __int128 % per element (a software division here too); this uses the exact FP64 modmul of the NTT
// (ntt_arith.hpp) when every q < 2^50, else a u128 fold with 2^64 mod q and one Barrett step.
__global__ __launch_bounds__(256) void mul_s_kernel(const uint64_t* __restrict__ a, const uint64_t* __restrict__ s,
                                                    uint64_t* __restrict__ t, const uint64_t* __restrict__ qmu,
                                                    const uint64_t* __restrict__ r64, const LimbConst* __restrict__ lf,
                                                    int L, int log_n, uint32_t total) {
    const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint32_t n = 1u << log_n, single = (uint32_t)L << log_n;
    const uint32_t poly = idx / single, off = idx - poly * single;
    const int l = (int)(off >> log_n);
    const uint32_t coeff = off & (n - 1), w = poly >> log_n;
    const uint64_t av = a[idx], sv = s[((uint64_t)w * L + l) * n + coeff];
    if (lf) {
        const ArithF64 ar(lf[l]);
        t[idx] = ar.canon(ar.mulmod(ArithF64::from_u64(av), ArithF64::from_u64(sv)));
        return;
    }
    const uint64_t q = qmu[2 * l], mu = qmu[2 * l + 1], rr = r64[l];
    uint64_t hi = __umul64hi(av, sv), lo = av * sv;
    while (hi) {
        const unsigned __int128 f = (unsigned __int128)hi * rr + lo;
        hi = (uint64_t)(f >> 64);
        lo = (uint64_t)f;
    }
    uint64_t r = lo - __umul64hi(lo, mu) * q;
    t[idx] = r >= q ? r - q : r;
}

// encrypt epilogue, fused: for matrix-major index i (x, y, l, w) and its poly-major index p,
//   ct_k.b[i] = m_k[i] - t[p] + e[p] mod q   (combine_b_kernel HE.cu:535-547, then poly_to_matrix)
//   ct_k.a[i] = a_eval[p]                   (the shared a, poly_to_matrix)
// for k = re (and im when given) in one pass: 3 + 2 reads and 2 + 2 writes instead of the 20 array
// passes of layout -> combine -> layout -> layout per component.
__global__ __launch_bounds__(256) void enc_combine_kernel(const uint64_t* __restrict__ m_re,
                                                          const uint64_t* __restrict__ m_im,
                                                          const uint64_t* __restrict__ t, const uint64_t* __restrict__ e,
                                                          const uint64_t* __restrict__ aev, uint64_t* __restrict__ ct_re,
                                                          uint64_t* __restrict__ ct_im, const uint64_t* __restrict__ qmu,
                                                          int log_n, int L, uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;   // matrix-major index
    if (i >= total) return;
    const uint64_t n = 1ull << log_n;
    const uint64_t x = i & (n - 1), y = (i >> log_n) & (n - 1);
    const uint32_t wl = (uint32_t)(i >> (2 * log_n)), w = wl / (uint32_t)L, l = wl - w * (uint32_t)L;   // wl < 2^32
    const uint64_t p = (((uint64_t)w * n + y) * L + l) * n + x;
    const uint64_t q = qmu[2 * l];
    const uint64_t tv = t[p], ev = e[p], av = aev[p];
    auto bval = [&](uint64_t m) {
        uint64_t d = m >= tv ? m - tv : m + q - tv;
        d += ev;
        return d >= q ? d - q : d;
    };
    ct_re[i] = bval(m_re[i]);
    ct_re[total + i] = av;
    if (m_im) {
        ct_im[i] = bval(m_im[i]);
        ct_im[total + i] = av;
    }
}

struct RingArgs {
    const LimbConst* lf;     // [L]
    const double* tw;        // ph_f tables [L][n]
    const double* itw;
    const double* ninv;      // [L]
    const uint64_t* sk;      // [w][L][n], NTT form
    int L;
    uint64_t rows;           // 512 n L
};

#ifndef MFHE_ENC_NT
#define MFHE_ENC_NT 1   // enc_ring_kernel's row streams as nontemporal accesses (read / written once; 0 for A/B)
#endif
// encrypt, fused: t = a * s over X (ring_mul_row), then encrypt_pair's combine (HE.cu:1530-1552):
// ct_k.b = m_k - t + e, ct_k.a = a, written matrix-major; a, e poly-major.  One thread: 4 coefficients
// of matrix row R = (w L + l) n + y.
template <int LOGN>
// a_mm: a is already in both ciphertexts (the W-CRT GEMM wrote it there, matrix-major): read it from aev + i0 and
// write only the b halves -- 6 of the 8 row streams
__global__ __launch_bounds__(256) void enc_ring_kernel(RingArgs ra, const uint64_t* __restrict__ aev,
                                                       const uint64_t* __restrict__ e, const uint64_t* __restrict__ m_re,
                                                       const uint64_t* __restrict__ m_im, uint64_t* __restrict__ ct_re,
                                                       uint64_t* __restrict__ ct_im, int a_mm) {
    constexpr int N = 1 << LOGN, T = N / 4;
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const int j = (int)(g % T);
    const uint64_t R = g / T;
    const bool live = R < ra.rows;                     // dead lanes still take part in the shuffles
    const uint64_t Rc = live ? R : 0;
    const uint64_t y = Rc % N;
    const uint32_t wl = (uint32_t)(Rc / N), w = wl / (uint32_t)ra.L, l = wl - w * (uint32_t)ra.L;   // wl < 2^32
    constexpr bool LDS = LOGN == 6 && MFHE_RING_LDS;   // ring_mul_row64_lds: reg s holds coefficient j + 16 s
    const uint64_t i0 = Rc * N, p0 = (((uint64_t)w * N + y) * ra.L + l) * N;   // row starts: matrix- / poly-major
    const LimbConst lc = ra.lf[l];
    const ArithF64 ar(lc);
    uint64_t av[4], sk[4];
    constexpr bool NT = MFHE_ENC_NT && LDS;
    ld_row<LDS, NT>(aev + (a_mm ? i0 : p0), j, av);
    ld4(ra.sk + ((uint64_t)w * ra.L + l) * N + 4 * j, sk);
    // the combine's operands are loaded before the ring product (clamped rows for dead lanes), so their latency
    // overlaps the butterflies instead of following them
    uint64_t ev[4], mv[4], mi[4], b[4];
    ld_row<LDS, NT>(e + p0, j, ev);
    ld_row<LDS, NT>(m_re + i0, j, mv);
    if (m_im) ld_row<LDS, NT>(m_im + i0, j, mi);
    double x[4], sv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        x[s] = ArithF64::from_u64(av[s]);
        sv[s] = centred_f(sk[s], lc.qf);
    }
    if constexpr (LDS) {
        __shared__ double rscr[16 * 68];
        ring_mul_row64_lds(x, sv, j, ar, ra.tw + l * N, ra.itw + l * N, ra.ninv[l], rscr + (threadIdx.x >> 4) * 68);
    } else {
        ring_mul_row<LOGN>(x, sv, j, ar, ra.tw + l * N, ra.itw + l * N, ra.ninv[l]);
    }
    if (!live) return;
    const uint64_t q = lc.q, total = ra.rows * N;
    auto bval = [&](uint64_t m, int s) {
        const uint64_t tv = ar.canon(x[s]);
        uint64_t d = m >= tv ? m - tv : m + q - tv;
        d += ev[s];
        return d >= q ? d - q : d;
    };
#pragma unroll
    for (int s = 0; s < 4; ++s) b[s] = bval(mv[s], s);
    st_row<LDS, NT>(ct_re + i0, j, b);
    if (!a_mm) st_row<LDS, NT>(ct_re + total + i0, j, av);
    if (m_im) {
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = bval(mi[s], s);
        st_row<LDS, NT>(ct_im + i0, j, b);
        if (!a_mm) st_row<LDS, NT>(ct_im + total + i0, j, av);
    }
}

// decrypt, fused: out = ct.b + INTT(NTT(ct.a) * s), ct matrix-major in, out poly-major (HE.cu:1553-1601:
// matrix_to_poly, X-NTT, pointwise_mul_s, X-INTT, add_poly).
template <int LOGN>
__global__ __launch_bounds__(256) void dec_ring_kernel(RingArgs ra, const uint64_t* __restrict__ ct,
                                                       uint64_t* __restrict__ out) {
    constexpr int N = 1 << LOGN, T = N / 4;
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const int j = (int)(g % T);
    const uint64_t R = g / T;
    const bool live = R < ra.rows;
    const uint64_t Rc = live ? R : 0;
    const uint64_t y = Rc % N;
    const uint32_t wl = (uint32_t)(Rc / N), w = wl / (uint32_t)ra.L, l = wl - w * (uint32_t)ra.L;   // wl < 2^32
    constexpr bool LDS = LOGN == 6 && MFHE_RING_LDS;   // as enc_ring_kernel
    const uint64_t i0 = Rc * N, total = ra.rows * N;
    const uint64_t p0 = (((uint64_t)w * N + y) * ra.L + l) * N;
    const LimbConst lc = ra.lf[l];
    const ArithF64 ar(lc);
    uint64_t av[4], sk[4], bv[4];
    ld_row<LDS>(ct + total + i0, j, av);
    ld4(ra.sk + ((uint64_t)w * ra.L + l) * N + 4 * j, sk);
    ld_row<LDS>(ct + i0, j, bv);   // before the ring product, so its latency overlaps the butterflies (clamped row if dead)
    double x[4], sv[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        x[s] = ArithF64::from_u64(av[s]);
        sv[s] = centred_f(sk[s], lc.qf);
    }
    if constexpr (LDS) {
        __shared__ double rscr[16 * 68];
        ring_mul_row64_lds(x, sv, j, ar, ra.tw + l * N, ra.itw + l * N, ra.ninv[l], rscr + (threadIdx.x >> 4) * 68);
    } else {
        ring_mul_row<LOGN>(x, sv, j, ar, ra.tw + l * N, ra.itw + l * N, ra.ninv[l]);
    }
    if (!live) return;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint64_t sum = bv[s] + ar.canon(x[s]);
        bv[s] = sum >= lc.q ? sum - lc.q : sum;
    }
    st_row<LDS>(out + p0, j, bv);
}

static bool ring_fused_ok(const mfhe_ctx* c, int logn) {
    return c->he_fused && c->f64_ok && c->ph_f.tw && logn >= 2 && logn <= 6;
}

static RingArgs ring_args(const mfhe_ctx* c, const uint64_t* sk, int L, uint64_t rows) {
    RingArgs ra;
    ra.lf = c->d_limbs;
    ra.tw = c->ph_f.tw;
    ra.itw = c->ph_f.itw;
    ra.ninv = c->ph_f.ninv;
    ra.sk = sk;
    ra.L = L;
    ra.rows = rows;
    return ra;
}

// decrypt_and_decode: the decrypt fused into the factored inverse W-CRT's digitize (n = 64, the same conditions
// as the factored inverse in use_mfma plus ring_fused_ok)
static bool dec_fused_ok(const mfhe_ctx* c, int logn) {
    return ring_fused_ok(c, logn) && logn == 6 && c->wcrt_mfma == 1 && c->wD && c->d_wZidig && c->d_wepi &&
           c->d_wifold && c->d_wiz && c->d_wphi;
}

#define MFHE_RING_DISPATCH(KERNEL, logn, grid, s, ...)                                       \
    switch (logn) {                                                                           \
        case 2: hipLaunchKernelGGL(KERNEL<2>, grid, dim3(256), 0, s, __VA_ARGS__); break;     \
        case 3: hipLaunchKernelGGL(KERNEL<3>, grid, dim3(256), 0, s, __VA_ARGS__); break;     \
        case 4: hipLaunchKernelGGL(KERNEL<4>, grid, dim3(256), 0, s, __VA_ARGS__); break;     \
        case 5: hipLaunchKernelGGL(KERNEL<5>, grid, dim3(256), 0, s, __VA_ARGS__); break;     \
        default: hipLaunchKernelGGL(KERNEL<6>, grid, dim3(256), 0, s, __VA_ARGS__); break;    \
    }

// decrypt epilogue, fused: out[p] = ct.b[i] + t[p] mod q (matrix_to_poly of b, then add_poly_kernel
// HE.cu:549-560), over the poly-major index p.
__global__ __launch_bounds__(256) void dec_combine_kernel(const uint64_t* __restrict__ ctb, const uint64_t* __restrict__ t,
                                                          uint64_t* __restrict__ out, const uint64_t* __restrict__ qmu,
                                                          int log_n, int L, uint64_t total) {
    const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;   // poly-major index [w n + y][l][x]
    if (p >= total) return;
    const uint64_t n = 1ull << log_n;
    const uint64_t x = p & (n - 1), rest = p >> log_n, l = rest % L, wy = rest / L;
    const uint64_t y = wy & (n - 1), w = wy >> log_n;
    const uint64_t i = (((w * L + l) << log_n) + y) * n + x;            // matrix-major [w][l][y][x]
    const uint64_t q = qmu[2 * l];
    const uint64_t sum = ctb[i] + t[p];
    out[p] = sum >= q ? sum - q : sum;
}

// centred int64 -> RNS matrix-major (centered_int_to_rns_matrix_kernel HE.cu:815-835)
__global__ void centered_to_rns_kernel(const int64_t* in, uint64_t* out, const uint64_t* qmu, int L, uint64_t n2,
                                       uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint64_t pos = idx % n2, t = idx / n2;
    const int l = (int)(t % L);
    const uint64_t w = t / L;
    const int64_t v = in[w * n2 + pos];
    const int64_t q = (int64_t)qmu[2 * l];
    int64_t r = v % q;
    if (r < 0) r += q;
    out[idx] = (uint64_t)r;
}

// he_big_to_i64_checked HE.cu:904-915 over compose output
__global__ void big_to_i64_kernel(const uint64_t* mag, const uint8_t* neg, int W, int64_t* out, uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    bool over = mag[i * W] > (uint64_t)INT64_MAX;
    for (int k = 1; k < W; ++k) over |= mag[i * W + k] != 0;
    const bool ng = neg[i] != 0;
    out[i] = over ? (ng ? INT64_MIN : INT64_MAX) : (ng ? -(int64_t)mag[i * W] : (int64_t)mag[i * W]);
}

// limb-0 centring after the inverse (HE.cu:1112-1113)
__global__ void center_limb0_kernel(const uint64_t* in, int64_t* out, uint64_t q, uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const uint64_t a = in[i];
    out[i] = (a > (q >> 1)) ? (int64_t)a - (int64_t)q : (int64_t)a;
}

// (hi:lo) mod q: fold hi with r64 = 2^64 mod q, then one Barrett step (mu = floor(2^64 / q))
__device__ __forceinline__ uint64_t mod128(unsigned __int128 v, uint64_t q, uint64_t mu, uint64_t r64) {
    uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
    while (hi) {
        const unsigned __int128 t = (unsigned __int128)hi * r64 + lo;
        hi = (uint64_t)(t >> 64);
        lo = (uint64_t)t;
    }
    uint64_t r = lo - __umul64hi(lo, mu) * q;
    return r >= q ? r - q : r;
}

// add_ct_kernel HE.cu:631-645 / mul_tensor_kernel HE.cu:648-669 over matrix-major [phi][L][n2]
// (limb = (idx / n2) % L).  `half` = words of one ciphertext component.
__global__ void ct_add_kernel(const uint64_t* x, const uint64_t* y, uint64_t* r,
                              const uint64_t* qmu, int L, int log_n2, uint64_t half) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= 2 * half) return;
    const int l = (int)(((idx % half) >> log_n2) % (uint64_t)L);
    const uint64_t q = qmu[2 * l];
    const uint64_t s = x[idx] + y[idx];
    r[idx] = s >= q ? s - q : s;
}
__global__ void ct_mul_kernel(const uint64_t* __restrict__ c1, const uint64_t* __restrict__ c2, uint64_t* d0,
                              uint64_t* d1, uint64_t* d2, const uint64_t* qmu, const uint64_t* r64, int L, int log_n2,
                              uint64_t half) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= half) return;
    const int l = (int)((idx >> log_n2) % (uint64_t)L);
    const uint64_t q = qmu[2 * l], mu = qmu[2 * l + 1], rr = r64[l];
    const uint64_t b1 = c1[idx], a1 = c1[half + idx], b2 = c2[idx], a2 = c2[half + idx];
    using u128 = unsigned __int128;
    d0[idx] = mod128((u128)b1 * b2, q, mu, rr);
    const uint64_t t1 = mod128((u128)b1 * a2, q, mu, rr), t2 = mod128((u128)a1 * b2, q, mu, rr);
    const uint64_t t = t1 + t2;
    d1[idx] = t >= q ? t - q : t;
    d2[idx] = mod128((u128)a1 * a2, q, mu, rr);
}

// planar <-> interleaved complex for the split re/im W-DFT entry points (HE.cu:472-502)
__global__ void pack_i64_pair_kernel(const int64_t* re, const int64_t* im, double2* out, uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < total) out[i] = make_double2((double)re[i], (double)im[i]);
}
__global__ void pack_f64_pair_kernel(const double* re, const double* im, double2* out, uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < total) out[i] = make_double2(re[i], im[i]);
}
__global__ void unpack_pair_kernel(const double2* in, double* re, double* im, uint64_t total) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < total) {
        const double2 v = in[i];
        re[i] = v.x;
        im[i] = v.y;
    }
}

// ---------------- helpers ----------------
static int need_wcrt(const mfhe_ctx* c) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (!(c->conv & MFHE_CONV_WCRT)) return set_error(MFHE_ENOTREADY, "context was created without MFHE_CONV_WCRT");
    return MFHE_OK;
}

struct Geo2 {
    int L, logn;
    uint64_t n, n2, words, cnt;   // words = phi*L*n2 ; cnt = phi*n2
};
static Geo2 geo(const mfhe_ctx* c) {
    Geo2 g;
    g.L = c->L;
    g.logn = c->logN;
    g.n = c->N;
    g.n2 = g.n * g.n;
    g.words = (uint64_t)mfhe_ctx::PHI * g.L * g.n2;
    g.cnt = (uint64_t)mfhe_ctx::PHI * g.n2;
    return g;
}

static size_t ws_need(const mfhe_ctx* c) {
    const Geo2 g = geo(c);
    return 10 * g.words * 8 + g.cnt * (size_t)c->W * 8 + 4 * g.cnt * 16 + 2 * g.cnt + (64 << 10);
}

static int ensure_ws(mfhe_ctx* c) {
    const size_t need = ws_need(c);
    if (c->ws_bytes >= need) return MFHE_OK;
    if (c->ws) MFHE_HIP(hipFree(c->ws));
    c->ws = nullptr;
    c->ws_bytes = 0;
    MFHE_HIP(hipMalloc(&c->ws, need));
    c->ws_bytes = need;
    return MFHE_OK;
}

struct Bump {
    char* p;
    template <class T>
    T* get(size_t n) {
        T* r = (T*)p;
        p += ((n * sizeof(T) + 255) / 256) * 256;
        return r;
    }
};

// W-CRT forward: B matrix-major [r][L][pos] (or vector [r][L][x]); C in the requested layout
enum class WOut { Poly, Matrix, Vector };
#define RC(x) do { int _r = (x); if (_r) return _r; } while (0)

// i8 MFMA operands for A = V or V^-1 (gemm.hip); leaves a on the VALU kernel when unavailable.  slot 1: the side
// stream's digit planes (HeFork)
static int use_mfma(mfhe_ctx* c, ModGemmArgs& a, const uint64_t* A, int L, int slot = 0) {
    if (!c->wcrt_mfma || !c->wD || (A != c->d_wV && A != c->d_wVinv)) return MFHE_OK;
    const size_t need = mod_gemm_mfma_ws(a.P, L, c->wD);
    void*& ws = slot ? c->gemm_ws2 : c->gemm_ws;
    size_t& wsb = slot ? c->gemm_ws2_bytes : c->gemm_ws_bytes;
    if (wsb < need) {
        if (ws) MFHE_HIP(hipFree(ws));
        ws = nullptr;
        wsb = 0;
        MFHE_HIP(hipMalloc(&ws, need));
        wsb = need;
    }
    a.Adig = A == c->d_wV ? c->d_wVdig : c->d_wVidig;
    a.adL = a.aL ? (uint64_t)c->wD * 512 * 512 : 0;
    a.D = c->wD;
    a.rtab = c->d_wrtab;
    a.Bdig = (int8_t*)ws;
    // a.aL == 0: one A shared by every limb (vector transforms) -> every limb uses the full digit count
    a.limbD = (a.aL && (int)c->wDl.size() == L) ? c->wDl.data() : nullptr;
    a.epi = c->d_wepi;
    a.lds_stage = c->wcrt_mfma != 2;
    a.pipe = c->wcrt_pipe;
    // mode 1: the forward transform of a per-limb V runs factored (half the MACs, gemm.hip)
    if (c->wcrt_mfma == 1 && A == c->d_wV && a.aL && c->d_wZdig && a.epi) {
        a.Adig = c->d_wZdig;
        a.adL = (uint64_t)c->wD * 256 * 256;
        a.fold = c->d_wfold;
    }
    // ... and the inverse of a per-limb V^-1 (interpolation through 771 = 3 x 257, reduced mod Phi_771)
    if (c->wcrt_mfma == 1 && A == c->d_wVinv && a.aL && c->d_wZidig && a.epi) {
        a.Adig = c->d_wZidig;
        a.adL = (uint64_t)c->wD * 256 * 256;
        a.ifold = c->d_wifold;
        a.iz = c->d_wiz;
        a.phi = c->d_wphi;
    }
    return MFHE_OK;
}

// qf (encode): B replaced by the W-IDFT's doubles, quantized and reduced inside the factored forward's digitize
// kernel (gemm.hip mfma_digitize_fold_kernel<D, SRC>, and the encrypt samplers with it); only when quant_fused_ok(c)
static bool quant_fused_ok(const mfhe_ctx* c) {
    return c->wcrt_mfma == 1 && c->wD && c->d_wZdig && c->d_wepi && c->d_wfold;
}
// the GEMM arguments of one W-CRT transform (wcrt_gemm launches them; encode / decode may launch two of them as
// pairs, gemm.hip launch_mod_gemm_pair)
static int wcrt_args(mfhe_ctx* c, ModGemmArgs& a, const uint64_t* A, const uint64_t* B, bool b_poly, uint64_t* C,
                     WOut out, bool vector, int qsrc = 0, const double* qf = nullptr, uint64_t qf_step = 1,
                     const RingArgs* dec = nullptr, int slot = 0, uint64_t* C2 = nullptr) {
    const Geo2 g = geo(c);
    a.A = A;
    a.aL = 512ull * 512;
    a.M = 512;
    a.K = 512;
    a.qmu = c->d_rns_mu;
    a.r64 = c->d_r64;
    a.B = B;
    a.C = C;
    a.C2 = C2;
    a.log_n = g.logn;
    if (vector) {
        a.P = (uint32_t)g.n;
        a.bL = g.n; a.sbK = (uint64_t)g.L * g.n; a.sbY = 0;
        a.cL = g.n; a.scM = (uint64_t)g.L * g.n; a.scY = 0;
    } else {
        a.P = (uint32_t)g.n2;
        if (b_poly) { a.bL = g.n; a.sbK = g.n * g.L * g.n; a.sbY = (uint64_t)g.L * g.n; }
        else { a.bL = g.n2; a.sbK = (uint64_t)g.L * g.n2; a.sbY = g.n; }
        if (out == WOut::Poly) { a.cL = g.n; a.scM = g.n * g.L * g.n; a.scY = (uint64_t)g.L * g.n; }
        else { a.cL = g.n2; a.scM = (uint64_t)g.L * g.n2; a.scY = g.n; }
    }
    RC(use_mfma(c, a, A, g.L, slot));
    if (C2 && !a.fold) return set_error(MFHE_EINVAL, "W-CRT: a second output needs the factored forward");
    if (dec) {
        // B is the ciphertext: the factored inverse's digitize decrypts it row by row (gemm.hip
        // mfma_digitize_ifold_dec_kernel); only where dec_fused_ok(c)
        if (!a.ifold) return set_error(MFHE_EINVAL, "W-CRT: a decrypt-fused source needs the factored inverse");
        a.dct = B;
        a.dtotal = g.words;
        a.dsk = dec->sk;
        a.dlf = dec->lf;
        a.dtw = dec->tw;
        a.ditw = dec->itw;
        a.dninv = dec->ninv;
    }
    if (qsrc) {
        if (!a.fold) return set_error(MFHE_EINVAL, "W-CRT: a fused digitize source needs the factored forward");
        a.qsrc = qsrc;
        a.qf = qf;
        a.qf_row = g.n2 * qf_step;
        a.qf_step = qf_step;
        a.delta = c->delta;
        a.lbase = c->limb_base;
        a.Ltot = c->limbs_total ? c->limbs_total : g.L;
    }
    return MFHE_OK;
}
static int wcrt_gemm(mfhe_ctx* c, const uint64_t* A, const uint64_t* B, bool b_poly, uint64_t* C, WOut out,
                     bool vector, hipStream_t s, int qsrc = 0, const double* qf = nullptr, uint64_t qf_step = 1,
                     const RingArgs* dec = nullptr, int slot = 0, uint64_t* C2 = nullptr) {
    ModGemmArgs a;
    RC(wcrt_args(c, a, A, B, b_poly, C, out, vector, qsrc, qf, qf_step, dec, slot, C2));
    return launch_mod_gemm(a, c->L, s);
}

// complex W-DFT / W-IDFT over [phi][n2]; MFHE_OPT_CGEMM_MFMA = 2 (default): factored through 771 = 3 x 257
// (gemm.hip cgemm_mfma_kernel<1 / 2>), half the flops of the dense 512 x 512 product
// planar (factored W-IDFT only, wdft_planar_ok): out as two [phi][n2] double planes, real then imaginary
static bool wdft_planar_ok(const mfhe_ctx* c) { return c->cgemm_mfma >= 2 && c->d_wdZ; }
static int wdft(mfhe_ctx* c, const double2* A, const double2* in, double2* out, hipStream_t s, bool planar = false) {
    const Geo2 g = geo(c);
    if (planar && !(wdft_planar_ok(c) && A == c->d_wdVinv))
        return set_error(MFHE_EINVAL, "wdft: planar output needs the factored W-IDFT");
    if (c->cgemm_mfma >= 2 && c->d_wdZ && (A == c->d_wdV || A == c->d_wdVinv)) {
        CGemmArgs f;
        f.mfma = true;
        f.B = in;
        f.C = out;
        f.aB = f.bB = f.cB = 0;
        f.M = f.K = 256;
        f.Pf = (uint32_t)g.n2;
        f.P = 2 * f.Pf;
        f.scM = g.n2;
        if (A == c->d_wdV) {
            // mode 2: the 257-point DFTs by Rader's algorithm (gemm.hip wdft_rader_kernel, r06); 3: the GEMM
            if (c->cgemm_mfma == 2 && c->d_wdrad && in != out)
                return launch_wdft_rader(in, out, (uint32_t)g.n2, c->d_wdrad, c->d_wdgp, s);
            f.fac = 1;
            f.A = c->d_wdZ;
            return launch_cgemm(f, 1, s);
        }
        if (c->cgemm_mfma == 2 && c->d_wdrad && in != out)   // Rader (gemm.hip wdft_rader_inv_kernel, r06)
            return launch_wdft_rader_inv(in, out, planar ? (double*)out + 512ull * g.n2 : nullptr, (uint32_t)g.n2,
                                         c->d_wdrad + 256, c->d_wdgp, c->d_wdlam, c->d_wdphi, s);
        const size_t need = (size_t)g.n2 * 2 * sizeof(double2);
        if (c->wd_ws_bytes < need) {
            if (c->wd_ws) MFHE_HIP(hipFree(c->wd_ws));
            c->wd_ws = nullptr;
            c->wd_ws_bytes = 0;
            MFHE_HIP(hipMalloc(&c->wd_ws, need));
            c->wd_ws_bytes = need;
        }
        f.fac = 2;
        if (planar) f.Cim = (double*)out + 512ull * g.n2;
        f.A = c->d_wdZi;
        f.cc = (const double2*)c->wd_ws;
        f.lam = c->d_wdlam;
        f.phi = c->d_wdphi;
        RC(launch_cwdft_inv_dots(f, in, c->d_wdxp, s));
        return launch_cgemm(f, 1, s);
    }
    CGemmArgs a;
    a.mfma = c->cgemm_mfma != 0;
    a.A = A; a.B = in; a.C = out;
    a.aB = a.bB = a.cB = 0;
    a.M = a.K = 512;
    a.P = (uint32_t)g.n2;
    a.log_n = 2 * g.logn;
    a.sbK = g.n2; a.sbY = 0; a.scM = g.n2; a.scY = 0;
    return launch_cgemm(a, 1, s);
}

// per-lane XY: out = A * M * B over `lanes` n x n matrices (tmp: lanes*n2 complex)
static int xy3(const mfhe_ctx* c, const double2* A, const double2* in, const double2* B, double2* tmp, double2* out,
               size_t lanes, hipStream_t s) {
    const Geo2 g = geo(c);
    // n = 64: mode 2 by 64-point FFTs (gemm.hip xy_fft_kernel, equal to rounding); mode 3 both GEMMs in one launch
    // (gemm.hip xy_fused_kernel), the same doubles as the two launches of mode 1
    if (c->cgemm_mfma == 2 && g.n == 64) {
        if (A == c->d_encV && B == c->d_encVT) return launch_xy_fft(in, out, false, (int)lanes, s);
        if (A == c->d_encVi && B == c->d_encViT) return launch_xy_fft(in, out, true, (int)lanes, s);
    }
    if (c->cgemm_mfma >= 2 && g.n == 64 && in != out) return launch_xy_fused(A, in, B, out, (int)lanes, s);
    CGemmArgs a;
    a.mfma = c->cgemm_mfma != 0;
    a.M = a.K = (int)g.n;
    a.P = (uint32_t)g.n;
    a.log_n = g.logn;
    a.sbK = g.n; a.sbY = 0; a.scM = g.n; a.scY = 0;
    a.A = A; a.aB = 0; a.B = in; a.bB = g.n2; a.C = tmp; a.cB = g.n2;        // T = A M
    int rc = launch_cgemm(a, (int)lanes, s);
    if (rc) return rc;
    a.A = tmp; a.aB = g.n2; a.B = B; a.bB = 0; a.C = out; a.cB = g.n2;       // out = T B
    return launch_cgemm(a, (int)lanes, s);
}

static int layout(const mfhe_ctx* c, const uint64_t* in, uint64_t* out, bool to_poly, hipStream_t s) {
    const Geo2 g = geo(c);
    if (to_poly) hipLaunchKernelGGL(layout_kernel<true>, g1(g.words), dim3(256), 0, s, in, out, g.logn, g.L, g.words);
    else hipLaunchKernelGGL(layout_kernel<false>, g1(g.words), dim3(256), 0, s, in, out, g.logn, g.L, g.words);
    MFHE_CHECK_LAUNCH("layout_kernel");
    return MFHE_OK;
}


// Two independent chains of one call (encode's re / im W-CRT, encrypt's a / e W-CRT, decode's re / im W-INTT +
// compose): the second runs on the context's side stream, forked from and joined back into the caller's stream by
// events, so the digitize (memory / FP64-VALU bound) of one overlaps the i8-MFMA GEMM of the other and each GEMM's
// tail.  The side chain's GEMM uses its own digit planes (wcrt_gemm slot 1).  MFHE_OPT_HE_STREAMS 0: x = s.
static int he_side_stream(mfhe_ctx* c) {   // created once (mfhe_ctx_reserve_workspace, or the first forked call)
    if (c->he_side) return MFHE_OK;
    MFHE_HIP(hipEventCreateWithFlags(&c->he_fork, hipEventDisableTiming));
    MFHE_HIP(hipEventCreateWithFlags(&c->he_join, hipEventDisableTiming));
    MFHE_HIP(hipStreamCreateWithFlags(&c->he_side, hipStreamNonBlocking));
    return MFHE_OK;
}
struct HeFork {
    hipStream_t s = nullptr, x = nullptr;
    mfhe_ctx* c = nullptr;
    bool on = false;
    int begin(mfhe_ctx* c_, hipStream_t s_, bool enable) {
        c = c_;
        s = x = s_;
        if (!enable) return MFHE_OK;
        RC(he_side_stream(c));
        MFHE_HIP(hipEventRecord(c->he_fork, s));
        MFHE_HIP(hipStreamWaitEvent(c->he_side, c->he_fork, 0));
        x = c->he_side;
        on = true;
        return MFHE_OK;
    }
    // every later use of the side chain's results (and of its workspace) is ordered after this on s
    int join() {
        if (!on) return MFHE_OK;
        on = false;
        MFHE_HIP(hipEventRecord(c->he_join, x));
        MFHE_HIP(hipStreamWaitEvent(s, c->he_join, 0));
        return MFHE_OK;
    }
    ~HeFork() { (void)join(); }   // an early error return still joins the side stream into s
};

static int encode_impl(mfhe_ctx* c, const double* msg, uint64_t* out_re, uint64_t* out_im, hipStream_t s) {
    RC(need_wcrt(c));
    if (!msg || !out_re || !out_im) return set_error(MFHE_EINVAL, "mfhe_encode: null pointer");
    RC(ensure_xy(c));
    RC(ensure_ws(c));
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    double2* xy = b.get<double2>(g.cnt);
    double2* tmp = b.get<double2>(g.cnt);
    uint64_t* cre = b.get<uint64_t>(g.words);
    // 1) XY-IDFT per lane (Encoder::idft2, encoder.cu:460-467)
    RC(xy3(c, c->d_encVi, (const double2*)msg, c->d_encViT, tmp, xy, 512, s));
    // 2) W-IDFT (w_idft_kernel, batched_encoder.cu:104-123); planar (real plane, then imaginary) when the fused
    // digitize reads it, so each of its per-limb passes reads whole 8-byte lanes (r06)
    const bool planar = quant_fused_ok(c) && wdft_planar_ok(c);
    RC(wdft(c, c->d_wdVinv, xy, tmp, s, planar));
    // 3) quantize + RNS split, 4) W-CRT -> matrix-major eval (re, then im); fused into the W-CRT's digitize
    // kernel when the factored forward runs (the residues never reach HBM)
    if (quant_fused_ok(c)) {
        const double* qre = (const double*)tmp;
        const double* qim = planar ? qre + 512ull * g.n2 : qre + 1;
        const uint64_t qstep = planar ? 1 : 2;
        if (c->he_streams >= 2) {   // modes 2, 3: re and im as one launch per step (gemm.hip launch_mod_gemm_pair)
            ModGemmArgs ar, ai;
            RC(wcrt_args(c, ar, c->d_wV, (const uint64_t*)tmp, false, out_re, WOut::Matrix, false, 1, qre, qstep));
            RC(wcrt_args(c, ai, c->d_wV, (const uint64_t*)tmp, false, out_im, WOut::Matrix, false, 1, qim, qstep,
                         nullptr, 1));
            return launch_mod_gemm_pair(ar, ai, g.L, s);
        }
        HeFork f;
        RC(f.begin(c, s, c->he_streams == 1));
        RC(wcrt_gemm(c, c->d_wV, (const uint64_t*)tmp, false, out_re, WOut::Matrix, false, s, 1, qre, qstep));
        RC(wcrt_gemm(c, c->d_wV, (const uint64_t*)tmp, false, out_im, WOut::Matrix, false, f.x, 1, qim, qstep,
                     nullptr, f.on ? 1 : 0));
        return f.join();
    }
    RC(mfhe_rns_decompose(c, (const double*)tmp, 2, 512, g.n2, cre, (mfhe_stream_t)s));
    RC(wcrt_gemm(c, c->d_wV, cre, false, out_re, WOut::Matrix, false, s));
    RC(mfhe_rns_decompose(c, (const double*)tmp + 1, 2, 512, g.n2, cre, (mfhe_stream_t)s));
    RC(wcrt_gemm(c, c->d_wV, cre, false, out_im, WOut::Matrix, false, s));
    return MFHE_OK;
}

// dec: ev_re / ev_im are the ciphertexts, decrypted inside the W-INTT's digitize (dec_fused_ok only)
static int decode_impl(mfhe_ctx* c, const uint64_t* ev_re, const uint64_t* ev_im, double* msg, hipStream_t s,
                       Bump* pb = nullptr, const RingArgs* dec = nullptr) {
    RC(need_wcrt(c));
    if (!ev_re || !ev_im || !msg) return set_error(MFHE_EINVAL, "mfhe_decode: null pointer");
    RC(ensure_xy(c));
    Bump b0{(char*)c->ws};
    if (!pb) {
        RC(ensure_ws(c));
        pb = &b0;
    }
    const Geo2 g = geo(c);
    uint64_t* coeff = pb->get<uint64_t>(g.words);
    double2* ccx = pb->get<double2>(g.cnt);
    double2* ecx = pb->get<double2>(g.cnt);
    // W-INTT (poly-major in -> matrix-major coeff), CRT compose + centre + /delta fused, into re / im (im on the side
    // stream with its own coefficient buffer; the two composes write alternate doubles of ccx)
    if (c->he_streams == 2) {
        // re and im as one launch per step: W-INTT pair (gemm.hip launch_mod_gemm_pair), then one compose launch
        uint64_t* coeff_im = pb->get<uint64_t>(g.words);
        ModGemmArgs ar, ai;
        RC(wcrt_args(c, ar, c->d_wVinv, ev_re, true, coeff, WOut::Matrix, false, 0, nullptr, 1, dec));
        RC(wcrt_args(c, ai, c->d_wVinv, ev_im, true, coeff_im, WOut::Matrix, false, 0, nullptr, 1, dec, 1));
        RC(launch_mod_gemm_pair(ar, ai, g.L, s));
        RC(crt_compose_f64_pair(c, coeff, coeff_im, 512, g.n2, (double*)ccx, (double*)ccx + 1, 2, s));
        RC(wdft(c, c->d_wdV, ccx, ecx, s));
        return xy3(c, c->d_encV, ecx, c->d_encVT, ccx, (double2*)msg, 512, s);
    }
    HeFork f;
    RC(f.begin(c, s, c->he_streams == 1 || c->he_streams == 3));
    uint64_t* coeff_im = f.on ? pb->get<uint64_t>(g.words) : coeff;
    RC(wcrt_gemm(c, c->d_wVinv, ev_re, true, coeff, WOut::Matrix, false, s, 0, nullptr, 1, dec));
    RC(mfhe_crt_compose_f64(c, coeff, 512, g.n2, (double*)ccx, 2, (mfhe_stream_t)s));
    RC(wcrt_gemm(c, c->d_wVinv, ev_im, true, coeff_im, WOut::Matrix, false, f.x, 0, nullptr, 1, dec, f.on ? 1 : 0));
    RC(mfhe_crt_compose_f64(c, coeff_im, 512, g.n2, (double*)ccx + 1, 2, (mfhe_stream_t)f.x));
    RC(f.join());
    // W-DFT, then XY-DFT per lane: M = V E V^T
    RC(wdft(c, c->d_wdV, ccx, ecx, s));
    RC(xy3(c, c->d_encV, ecx, c->d_encVT, ccx, (double2*)msg, 512, s));
    return MFHE_OK;
}

static int keygen_impl(mfhe_ctx* c, uint64_t* sk, hipStream_t s) {
    RC(need_wcrt(c));
    if (!(c->conv & MFHE_CONV_PHANTOM)) return set_error(MFHE_ENOTREADY, "keygen needs MFHE_CONV_PHANTOM (X-NTT)");
    if (!sk) return set_error(MFHE_EINVAL, "mfhe_keygen: null pointer");
    RC(ensure_ws(c));
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    uint64_t* sc = b.get<uint64_t>(512ull * g.L * g.n);
    const uint64_t total = 512ull * g.L * g.n;
    hipLaunchKernelGGL(ternary_kernel, g1(total), dim3(256), 0, s, sc, c->d_rns_mu, g.L, g.logn, total);
    MFHE_CHECK_LAUNCH("ternary_kernel");
    RC(wcrt_gemm(c, c->d_wV, sc, false, sk, WOut::Vector, true, s));
    return mfhe_ntt_fwd(c, sk, 512, 0, g.L, (mfhe_stream_t)s);
}

// encrypt (HE.cu:1370-1453) / encrypt_pair (HE.cu:1455-1552)
static int encrypt_impl(mfhe_ctx* c, const uint64_t* m_re, const uint64_t* m_im, const uint64_t* sk, uint64_t* ct_re,
                        uint64_t* ct_im, hipStream_t s) {
    RC(need_wcrt(c));
    if (!(c->conv & MFHE_CONV_PHANTOM)) return set_error(MFHE_ENOTREADY, "encrypt needs MFHE_CONV_PHANTOM (X-NTT)");
    if (!m_re || !sk || !ct_re || (m_im && !ct_im)) return set_error(MFHE_EINVAL, "mfhe_encrypt: null pointer");
    RC(ensure_ws(c));
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    uint64_t* ap = b.get<uint64_t>(g.words);
    uint64_t* aev = b.get<uint64_t>(g.words);
    uint64_t* ant = b.get<uint64_t>(g.words);
    uint64_t* ep = b.get<uint64_t>(g.words);
    uint64_t* eev = b.get<uint64_t>(g.words);
    const uint64_t W = g.words;
    const bool a_mm = quant_fused_ok(c) && ring_fused_ok(c, g.logn) && c->enc_a_direct;
    // shared a: W coeff -> W-CRT eval (poly-major) -> X-NTT
    // e: identical for re and im (seed depends only on the coefficient, HE.cu:605-608)
    if (quant_fused_ok(c)) {
        // the samplers evaluated inside the factored W-CRT's digitize: a in place, e from one draw per coefficient;
        // with the fused ring, a straight into both ciphertexts' a halves (matrix-major), where enc_ring reads it.
        // MFHE_OPT_HE_STREAMS 2: the two GEMMs as one launch (gemm.hip launch_mod_gemm_pair; measured no faster than
        // two: 301 vs 160 + 138 us, profiles/r05_he_stream_modes.txt, so mode 3 keeps two)
        const bool pair = c->he_streams == 2;
        ModGemmArgs aa, ae;
        if (a_mm) RC(wcrt_args(c, aa, c->d_wV, ap, false, ct_re + W, WOut::Matrix, false, 2, nullptr, 1, nullptr, 0,
                               m_im ? ct_im + W : nullptr));
        else RC(wcrt_args(c, aa, c->d_wV, ap, false, aev, WOut::Poly, false, 2));
        // the noise: its W-CRT forward as the dense product with its one signed digit (MFHE_OPT_ENC_E_SMALL, gemm.hip
        // mod_gemm_mfma_smallb_kernel) where the dense V planes have 5-6 digits; else factored from its residues
        const bool e_small = c->enc_e_small && !pair && c->d_wVdig && c->wD >= 5 && c->wD <= 6 && g.n2 % 64 == 0;
        if (e_small) {
            RC(wcrt_args(c, ae, c->d_wV, ep, false, eev, WOut::Poly, false));
            ae.Adig = c->d_wVdig;   // the dense V planes (use_mfma chose the factored ones)
            ae.adL = (uint64_t)c->wD * 512 * 512;
            ae.fold = nullptr;
            RC(launch_mod_gemm(aa, g.L, s));
            int8_t* b8 = (int8_t*)ep;   // 512 x n^2 bytes, inside the unused residue buffer
            hipLaunchKernelGGL(gaussian_i8_kernel, g1(128ull * g.n2), dim3(256), 0, s, b8, g.logn, (uint32_t)g.n2);
            MFHE_CHECK_LAUNCH("gaussian_i8_kernel");
            RC(launch_mod_gemm_smallb(ae, b8, g.L, s));
        } else {
            RC(wcrt_args(c, ae, c->d_wV, ep, false, eev, WOut::Poly, false, 3, (const double*)ep, 1, nullptr,
                         pair ? 1 : 0));
            if (!pair) RC(launch_mod_gemm(aa, g.L, s));
            hipLaunchKernelGGL(gaussian_compact_kernel, g1(W / g.L), dim3(256), 0, s, (double*)ep, g.logn, W / g.L);
            MFHE_CHECK_LAUNCH("gaussian_compact_kernel");
            if (pair) RC(launch_mod_gemm_pair(aa, ae, g.L, s));
            else RC(launch_mod_gemm(ae, g.L, s));
        }
    } else {
        hipLaunchKernelGGL(uniform_kernel, g1(W), dim3(256), 0, s, ap, c->d_rns_mu, g.L, g.logn, W, c->limb_base,
                           c->limbs_total ? c->limbs_total : g.L);
        MFHE_CHECK_LAUNCH("uniform_kernel");
        RC(wcrt_gemm(c, c->d_wV, ap, false, aev, WOut::Poly, false, s));
        hipLaunchKernelGGL(gaussian_kernel, g1(W / g.L), dim3(256), 0, s, ep, c->d_rns_mu, g.L, g.logn, W / g.L);
        MFHE_CHECK_LAUNCH("gaussian_kernel");
        RC(wcrt_gemm(c, c->d_wV, ep, false, eev, WOut::Poly, false, s));
    }
    if (ring_fused_ok(c, g.logn)) {
        const uint64_t rows = W / g.n;
        const RingArgs ra = ring_args(c, sk, g.L, rows);
        MFHE_RING_DISPATCH(enc_ring_kernel, g.logn, g1(rows * (g.n / 4)), s, ra, a_mm ? ct_re + W : aev, eev, m_re, m_im,
                           ct_re, ct_im, (int)a_mm);
        MFHE_CHECK_LAUNCH("enc_ring_kernel");
        return MFHE_OK;
    }
    MFHE_HIP(hipMemcpyAsync(ant, aev, W * 8, hipMemcpyDeviceToDevice, s));
    RC(mfhe_ntt_fwd(c, ant, 512 * g.n, 0, g.L, (mfhe_stream_t)s));
    // t = INTT(a_ntt * s)  (reuse ep as t)
    uint64_t* t = ep;
    if (W >= (1ull << 32)) return set_error(MFHE_EUNSUPPORTED, "ciphertext of 2^32 words or more");
    hipLaunchKernelGGL(mul_s_kernel, g1(W), dim3(256), 0, s, ant, sk, t, c->d_rns_mu, c->d_r64,
                       c->f64_ok ? c->d_limbs : nullptr, g.L, g.logn, (uint32_t)W);
    MFHE_CHECK_LAUNCH("mul_s_kernel");
    RC(mfhe_ntt_inv(c, t, 512 * g.n, 0, g.L, (mfhe_stream_t)s));
    hipLaunchKernelGGL(enc_combine_kernel, g1(W), dim3(256), 0, s, m_re, m_im, t, eev, aev, ct_re, ct_im,
                       c->d_rns_mu, g.logn, g.L, W);
    MFHE_CHECK_LAUNCH("enc_combine_kernel");
    return MFHE_OK;
}

static int decrypt_impl(mfhe_ctx* c, const uint64_t* ct, const uint64_t* sk, uint64_t* out, hipStream_t s, Bump* pb) {
    const Geo2 g = geo(c);
    const uint64_t W = g.words;
    if (ring_fused_ok(c, g.logn)) {
        const uint64_t rows = W / g.n;
        const RingArgs ra = ring_args(c, sk, g.L, rows);
        MFHE_RING_DISPATCH(dec_ring_kernel, g.logn, g1(rows * (g.n / 4)), s, ra, ct, out);
        MFHE_CHECK_LAUNCH("dec_ring_kernel");
        return MFHE_OK;
    }
    uint64_t* ap = pb->get<uint64_t>(W);
    uint64_t* t = pb->get<uint64_t>(W);
    RC(layout(c, ct + W, ap, true, s));
    RC(mfhe_ntt_fwd(c, ap, 512 * g.n, 0, g.L, (mfhe_stream_t)s));
    if (W >= (1ull << 32)) return set_error(MFHE_EUNSUPPORTED, "ciphertext of 2^32 words or more");
    hipLaunchKernelGGL(mul_s_kernel, g1(W), dim3(256), 0, s, ap, sk, t, c->d_rns_mu, c->d_r64,
                       c->f64_ok ? c->d_limbs : nullptr, g.L, g.logn, (uint32_t)W);
    MFHE_CHECK_LAUNCH("mul_s_kernel");
    RC(mfhe_ntt_inv(c, t, 512 * g.n, 0, g.L, (mfhe_stream_t)s));
    hipLaunchKernelGGL(dec_combine_kernel, g1(W), dim3(256), 0, s, ct, t, out, c->d_rns_mu, g.logn, g.L, W);
    MFHE_CHECK_LAUNCH("dec_combine_kernel");
    return MFHE_OK;
}

// Residue-sharded decode (BASELINE C4): this rank's W-INTT of its limbs, the RCCL recombine of every lane's
// L residues (dist.cpp) into this rank's lane slice of the centred / delta values, an all-gather of those
// f64 slices, then the W-DFT and XY-DFT of the whole batch (FP64, replicated on every rank).  Replaces
// decode_eval_pair_to_complex (HE.cu:1619-1689) whose per-lane compose loop (:1653-1668) is the exchange step.
static int decode_sharded_impl(mfhe_ctx* c, mfhe_ctx* call, mfhe_comm* comm, int mode, const uint64_t* ev_re,
                               const uint64_t* ev_im, double* msg, hipStream_t s, Bump* pb,
                               const RingArgs* dec = nullptr) {
    const Geo2 g = geo(c);
    int G = 1, rank = 0;
    RC(comm_size_rank(comm, &G, &rank));
    uint64_t* coeff_re = pb->get<uint64_t>(g.words);
    uint64_t* coeff_im = pb->get<uint64_t>(g.words);
    double2* ccx = pb->get<double2>(g.cnt);
    double2* ecx = pb->get<double2>(g.cnt);
    // both W-INTTs first, then the two chunked recombines back to back; the im call passes MFHE_RECOMBINE_AFTER_PREV
    // (coeff_im was complete when the re call was entered), so the exchange stream runs the im chunks right after the
    // re chunks, waiting only for the composes whose receive half it refills (dist.cpp mfhe_crt_recombine_chunked).
    // Rows land at their
    // lane index (MFHE_RECOMBINE_ROWS_GLOBAL), so each chunk's lanes [p0, p0 + cp) are [rank][cp / G] in lane order
    // and one in-place all-gather per chunk completes them on every rank.
    const size_t cp = mfhe_ctx::PHI / 4 >= (size_t)G ? mfhe_ctx::PHI / 4 / G * G : (size_t)G;
    RC(wcrt_gemm(c, c->d_wVinv, ev_re, true, coeff_re, WOut::Matrix, false, s, 0, nullptr, 1, dec));
    RC(wcrt_gemm(c, c->d_wVinv, ev_im, true, coeff_im, WOut::Matrix, false, s, 0, nullptr, 1, dec));
    // Both recombines are always issued and their statuses agreed on once at the end: a rank whose re call fails
    // locally after its exchanges started still joins the im call's collectives and the agreement, so no peer is left
    // waiting in a collective this rank skipped; every rank then returns the error.
    const int rre = mfhe_crt_recombine_chunked(call, comm, mode, coeff_re, 512, g.n2, cp, (double*)ccx, 2,
                                               MFHE_RECOMBINE_ROWS_GLOBAL, (mfhe_stream_t)s);
    const std::string ere = rre ? mfhe_last_error() : "";
    const int rim = mfhe_crt_recombine_chunked(call, comm, mode, coeff_im, 512, g.n2, cp, (double*)ccx + 1, 2,
                                               MFHE_RECOMBINE_ROWS_GLOBAL | MFHE_RECOMBINE_AFTER_PREV, (mfhe_stream_t)s);
    RC(comm_agree(comm, rre ? set_error(rre, ere) : rim, s));
    for (size_t p0 = 0; p0 < 512; p0 += cp) {
        const size_t bs = (512 - p0 < cp ? 512 - p0 : cp) / (size_t)G;
        RC(comm_allgather_bytes(comm, ccx + (p0 + (size_t)rank * bs) * g.n2, ccx + p0 * g.n2,
                                bs * g.n2 * sizeof(double2), s));   // in place
    }
    RC(wdft(c, c->d_wdV, ccx, ecx, s));
    RC(xy3(c, c->d_encV, ecx, c->d_encVT, ccx, (double2*)msg, 512, s));
    return MFHE_OK;
}

}  // namespace mfhe

using namespace mfhe;

extern "C" int mfhe_ctx_reserve_workspace(mfhe_ctx* c) {
    RC(need_wcrt(c));
    RC(ensure_ws(c));
    // both GEMM digit-plane workspaces (the caller's stream and the side stream of MFHE_OPT_HE_STREAMS) at the
    // matrix transforms' size, so no W-CRT call allocates afterwards
    if (c->wcrt_mfma && c->wD) {
        const Geo2 g = geo(c);
        ModGemmArgs a;
        a.P = (uint32_t)g.n2;
        a.aL = 512ull * 512;
        RC(use_mfma(c, a, c->d_wV, g.L, 0));
        RC(use_mfma(c, a, c->d_wV, g.L, 1));
    }
    return he_side_stream(c);
}

extern "C" int mfhe_wcrt_fwd(mfhe_ctx* c, const uint64_t* in, uint64_t* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out) return set_error(MFHE_EINVAL, "mfhe_wcrt_fwd: null pointer");
    return wcrt_gemm(c, c->d_wV, in, false, out, WOut::Poly, false, (hipStream_t)s);
}
extern "C" int mfhe_wcrt_inv(mfhe_ctx* c, const uint64_t* in, uint64_t* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out) return set_error(MFHE_EINVAL, "mfhe_wcrt_inv: null pointer");
    return wcrt_gemm(c, c->d_wVinv, in, true, out, WOut::Matrix, false, (hipStream_t)s);
}
extern "C" int mfhe_wcrt_fwd_vector(mfhe_ctx* c, const uint64_t* in, uint64_t* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out) return set_error(MFHE_EINVAL, "mfhe_wcrt_fwd_vector: null pointer");
    return wcrt_gemm(c, c->d_wV, in, false, out, WOut::Vector, true, (hipStream_t)s);
}

extern "C" int mfhe_wcrt_fwd_centered(mfhe_ctx* c, const int64_t* in, int64_t* out, mfhe_stream_t s_) {
    RC(need_wcrt(c));
    if (!in || !out) return set_error(MFHE_EINVAL, "mfhe_wcrt_fwd_centered: null pointer");
    RC(ensure_ws(c));
    hipStream_t s = (hipStream_t)s_;
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    uint64_t* rns = b.get<uint64_t>(g.words);
    uint64_t* ev = b.get<uint64_t>(g.words);
    uint64_t* mag = b.get<uint64_t>(g.cnt * c->W);
    uint8_t* neg = b.get<uint8_t>(g.cnt);
    hipLaunchKernelGGL(centered_to_rns_kernel, g1(g.words), dim3(256), 0, s, in, rns, c->d_rns_mu, g.L, g.n2, g.words);
    MFHE_CHECK_LAUNCH("centered_to_rns_kernel");
    RC(wcrt_gemm(c, c->d_wV, rns, false, ev, WOut::Matrix, false, s));
    RC(mfhe_crt_compose(c, ev, 512, g.n2, mag, neg, s_));
    hipLaunchKernelGGL(big_to_i64_kernel, g1(g.cnt), dim3(256), 0, s, mag, neg, c->W, out, g.cnt);
    MFHE_CHECK_LAUNCH("big_to_i64_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_wcrt_inv_centered(mfhe_ctx* c, const int64_t* in, int64_t* out, mfhe_stream_t s_) {
    RC(need_wcrt(c));
    if (!in || !out) return set_error(MFHE_EINVAL, "mfhe_wcrt_inv_centered: null pointer");
    RC(ensure_ws(c));
    hipStream_t s = (hipStream_t)s_;
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    uint64_t* rns = b.get<uint64_t>(g.cnt);
    uint64_t* co = b.get<uint64_t>(g.cnt);
    // limb 0 only (HE.cu:1101): treat the input as a 1-limb matrix-major array
    hipLaunchKernelGGL(centered_to_rns_kernel, g1(g.cnt), dim3(256), 0, s, in, rns, c->d_rns_mu, 1, g.n2, g.cnt);
    MFHE_CHECK_LAUNCH("centered_to_rns_kernel");
    ModGemmArgs a;
    a.A = c->d_wVinv; a.aL = 0; a.M = a.K = 512; a.qmu = c->d_rns_mu; a.r64 = c->d_r64;
    a.B = rns; a.bL = 0; a.sbK = g.n2; a.sbY = g.n; a.log_n = g.logn; a.P = (uint32_t)g.n2;
    a.C = co; a.cL = 0; a.scM = g.n2; a.scY = g.n;
    RC(use_mfma(c, a, c->d_wVinv, 1));
    RC(launch_mod_gemm(a, 1, s));
    hipLaunchKernelGGL(center_limb0_kernel, g1(g.cnt), dim3(256), 0, s, co, out, c->moduli[0], g.cnt);
    MFHE_CHECK_LAUNCH("center_limb0_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_wdft_fwd(mfhe_ctx* c, const double* in, double* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out || in == out) return set_error(MFHE_EINVAL, "mfhe_wdft_fwd: need distinct in/out");
    return wdft(c, c->d_wdV, (const double2*)in, (double2*)out, (hipStream_t)s);
}
extern "C" int mfhe_wdft_inv(mfhe_ctx* c, const double* in, double* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out || in == out) return set_error(MFHE_EINVAL, "mfhe_wdft_inv: need distinct in/out");
    return wdft(c, c->d_wdVinv, (const double2*)in, (double2*)out, (hipStream_t)s);
}

static int xy_entry(mfhe_ctx* c, const double* in, double* out, size_t lanes, mfhe_stream_t s, bool inv) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (lanes == 0) return MFHE_OK;
    if (!in || !out || in == out) return set_error(MFHE_EINVAL, "mfhe_xy_(i)dft: need distinct in/out");
    if (lanes > 65535) return set_error(MFHE_EINVAL, "mfhe_xy_(i)dft: at most 65535 lanes per call");
    RC(ensure_xy(c));
    RC(ensure_ws(c));
    double2* tmp = (double2*)c->ws;
    const Geo2 g = geo(c);
    if (lanes * g.n2 * 16 > c->ws_bytes) return set_error(MFHE_EINVAL, "too many lanes for the workspace");
    return inv ? xy3(c, c->d_encVi, (const double2*)in, c->d_encViT, tmp, (double2*)out, lanes, (hipStream_t)s)
               : xy3(c, c->d_encV, (const double2*)in, c->d_encVT, tmp, (double2*)out, lanes, (hipStream_t)s);
}
extern "C" int mfhe_xy_idft(mfhe_ctx* c, const double* in, double* out, size_t lanes, mfhe_stream_t s) {
    return xy_entry(c, in, out, lanes, s, true);
}
extern "C" int mfhe_xy_dft(mfhe_ctx* c, const double* in, double* out, size_t lanes, mfhe_stream_t s) {
    return xy_entry(c, in, out, lanes, s, false);
}

extern "C" int mfhe_matrix_to_poly(mfhe_ctx* c, const uint64_t* in, uint64_t* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out || in == out) return set_error(MFHE_EINVAL, "layout needs distinct in/out");
    return layout(c, in, out, true, (hipStream_t)s);
}
extern "C" int mfhe_poly_to_matrix(mfhe_ctx* c, const uint64_t* in, uint64_t* out, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!in || !out || in == out) return set_error(MFHE_EINVAL, "layout needs distinct in/out");
    return layout(c, in, out, false, (hipStream_t)s);
}

extern "C" int mfhe_encode(mfhe_ctx* c, const double* msg, uint64_t* re, uint64_t* im, mfhe_stream_t s) {
    return encode_impl(c, msg, re, im, (hipStream_t)s);
}
extern "C" int mfhe_decode(mfhe_ctx* c, const uint64_t* re, const uint64_t* im, double* msg, mfhe_stream_t s) {
    return decode_impl(c, re, im, msg, (hipStream_t)s);
}
extern "C" int mfhe_keygen(mfhe_ctx* c, uint64_t* sk, mfhe_stream_t s) { return keygen_impl(c, sk, (hipStream_t)s); }
extern "C" int mfhe_encrypt(mfhe_ctx* c, const uint64_t* m, const uint64_t* sk, uint64_t* ct, mfhe_stream_t s) {
    return encrypt_impl(c, m, nullptr, sk, ct, nullptr, (hipStream_t)s);
}
extern "C" int mfhe_encrypt_pair(mfhe_ctx* c, const uint64_t* mre, const uint64_t* mim, const uint64_t* sk,
                                 uint64_t* cre, uint64_t* cim, mfhe_stream_t s) {
    if (!mim || !cim) return set_error(MFHE_EINVAL, "mfhe_encrypt_pair: null pointer");
    return encrypt_impl(c, mre, mim, sk, cre, cim, (hipStream_t)s);
}
extern "C" int mfhe_decrypt_to_eval(mfhe_ctx* c, const uint64_t* ct, const uint64_t* sk, uint64_t* out,
                                    mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!(c->conv & MFHE_CONV_PHANTOM)) return set_error(MFHE_ENOTREADY, "decrypt needs MFHE_CONV_PHANTOM (X-NTT)");
    if (!ct || !sk || !out) return set_error(MFHE_EINVAL, "mfhe_decrypt_to_eval: null pointer");
    RC(ensure_ws(c));
    Bump b{(char*)c->ws};
    return decrypt_impl(c, ct, sk, out, (hipStream_t)s, &b);
}
extern "C" int mfhe_decrypt_and_decode(mfhe_ctx* c, const uint64_t* cre, const uint64_t* cim, const uint64_t* sk,
                                       double* msg, mfhe_stream_t s) {
    RC(need_wcrt(c));
    if (!(c->conv & MFHE_CONV_PHANTOM)) return set_error(MFHE_ENOTREADY, "decrypt needs MFHE_CONV_PHANTOM (X-NTT)");
    if (!cre || !cim || !sk || !msg) return set_error(MFHE_EINVAL, "mfhe_decrypt_and_decode: null pointer");
    RC(ensure_ws(c));
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    if (dec_fused_ok(c, g.logn)) {
        RingArgs ra = ring_args(c, sk, g.L, g.words / g.n);
        return decode_impl(c, cre, cim, msg, (hipStream_t)s, &b, &ra);
    }
    uint64_t* er = b.get<uint64_t>(g.words);
    uint64_t* ei = b.get<uint64_t>(g.words);
    Bump inner = b;
    RC(decrypt_impl(c, cre, sk, er, (hipStream_t)s, &inner));
    inner = b;
    RC(decrypt_impl(c, cim, sk, ei, (hipStream_t)s, &inner));
    inner = b;
    return decode_impl(c, er, ei, msg, (hipStream_t)s, &inner);
}

// Every argument check of a sharded decode, run by each rank on its own arguments.
static int sharded_args(mfhe_ctx* c, mfhe_ctx* call, mfhe_comm* comm, const void* a, const void* b, const void* m) {
    RC(need_wcrt(c));
    if (!call || !a || !b || !m) return set_error(MFHE_EINVAL, "sharded decode: null pointer");
    if (call->N != c->N) return set_error(MFHE_EINVAL, "sharded decode: ctx_all has another ring degree");
    // the compose divides by ctx_all's delta: another scale would give silently wrong messages
    if (call->delta != c->delta) return set_error(MFHE_EINVAL, "sharded decode: ctx_all has another scale (delta)");
    int G = 1, rank = 0;
    RC(comm_size_rank(comm, &G, &rank));
    if (512 % G) return set_error(MFHE_EINVAL, "sharded decode: the communicator size must divide 512 lanes");
    if (call->L != (c->limbs_total ? c->limbs_total : c->L) || call->L != c->L * G)
        return set_error(MFHE_EINVAL, "sharded decode: ctx_all must hold the G * L_shard moduli of the whole set");
    // the exchange layout puts rank g's limbs at [g L, (g + 1) L) of ctx_all: the shard must be exactly that
    if (c->limb_base != rank * c->L)
        return set_error(MFHE_EINVAL, "sharded decode: this rank's shard must start at limb rank * L_shard "
                                      "(mfhe_ctx_set_limb_shard)");
    for (int k = 0; k < c->L; ++k)
        if (call->moduli[(size_t)(rank * c->L + k)] != c->moduli[(size_t)k])
            return set_error(MFHE_EINVAL, "sharded decode: the shard's moduli differ from ctx_all's limbs rank * L_shard..");
    RC(ensure_xy(c));
    return ensure_ws(c);
}
extern "C" int mfhe_decode_sharded(mfhe_ctx* c, mfhe_ctx* call, mfhe_comm* comm, int mode, const uint64_t* re,
                                   const uint64_t* im, double* msg, mfhe_stream_t s) {
    if (!comm) return set_error(MFHE_EINVAL, "sharded decode: null communicator");
    // the ranks agree on the verdict before any collective: one rank's bad arguments fail every rank instead of
    // leaving the others blocked in the exchange
    RC(comm_agree(comm, sharded_args(c, call, comm, re, im, msg), (hipStream_t)s));
    Bump b{(char*)c->ws};
    return decode_sharded_impl(c, call, comm, mode, re, im, msg, (hipStream_t)s, &b);
}
extern "C" int mfhe_decrypt_and_decode_sharded(mfhe_ctx* c, mfhe_ctx* call, mfhe_comm* comm, int mode,
                                               const uint64_t* cre, const uint64_t* cim, const uint64_t* sk, double* msg,
                                               mfhe_stream_t s) {
    if (!comm) return set_error(MFHE_EINVAL, "sharded decode: null communicator");
    int rc = sharded_args(c, call, comm, cre, cim, msg);
    if (!rc && !(c->conv & MFHE_CONV_PHANTOM)) rc = set_error(MFHE_ENOTREADY, "decrypt needs MFHE_CONV_PHANTOM (X-NTT)");
    if (!rc && !sk) rc = set_error(MFHE_EINVAL, "sharded decrypt: null key");
    RC(comm_agree(comm, rc, (hipStream_t)s));
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    if (dec_fused_ok(c, g.logn)) {
        RingArgs ra = ring_args(c, sk, g.L, g.words / g.n);
        return decode_sharded_impl(c, call, comm, mode, cre, cim, msg, (hipStream_t)s, &b, &ra);
    }
    uint64_t* er = b.get<uint64_t>(g.words);
    uint64_t* ei = b.get<uint64_t>(g.words);
    Bump inner = b;
    RC(decrypt_impl(c, cre, sk, er, (hipStream_t)s, &inner));
    inner = b;
    RC(decrypt_impl(c, cim, sk, ei, (hipStream_t)s, &inner));
    inner = b;
    return decode_sharded_impl(c, call, comm, mode, er, ei, msg, (hipStream_t)s, &inner);
}

static int wdft_pair(mfhe_ctx* c, const void* re, const void* im, bool i64, double* ore, double* oim, bool inv,
                     hipStream_t s) {
    RC(need_wcrt(c));
    if (!re || !im || !ore || !oim) return set_error(MFHE_EINVAL, "mfhe_wdft_*_pair: null pointer");
    RC(ensure_ws(c));
    const Geo2 g = geo(c);
    Bump b{(char*)c->ws};
    double2* x = b.get<double2>(g.cnt);
    double2* y = b.get<double2>(g.cnt);
    if (i64)
        hipLaunchKernelGGL(pack_i64_pair_kernel, g1(g.cnt), dim3(256), 0, s, (const int64_t*)re, (const int64_t*)im, x,
                           g.cnt);
    else
        hipLaunchKernelGGL(pack_f64_pair_kernel, g1(g.cnt), dim3(256), 0, s, (const double*)re, (const double*)im, x,
                           g.cnt);
    MFHE_CHECK_LAUNCH("pack_pair_kernel");
    RC(wdft(c, inv ? c->d_wdVinv : c->d_wdV, x, y, s));
    hipLaunchKernelGGL(unpack_pair_kernel, g1(g.cnt), dim3(256), 0, s, y, ore, oim, g.cnt);
    MFHE_CHECK_LAUNCH("unpack_pair_kernel");
    return MFHE_OK;
}
extern "C" int mfhe_wdft_fwd_pair_i64(mfhe_ctx* c, const int64_t* re, const int64_t* im, double* ore, double* oim,
                                      mfhe_stream_t s) {
    return wdft_pair(c, re, im, true, ore, oim, false, (hipStream_t)s);
}
extern "C" int mfhe_wdft_inv_pair(mfhe_ctx* c, const double* re, const double* im, double* ore, double* oim,
                                  mfhe_stream_t s) {
    return wdft_pair(c, re, im, false, ore, oim, true, (hipStream_t)s);
}

extern "C" int mfhe_ct_add(mfhe_ctx* c, const uint64_t* x, const uint64_t* y, uint64_t* r, mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (!x || !y || !r) return set_error(MFHE_EINVAL, "mfhe_ct_add: null pointer");
    const Geo2 g = geo(c);
    hipLaunchKernelGGL(ct_add_kernel, g1(2 * g.words), dim3(256), 0, (hipStream_t)s, x, y, r, c->d_rns_mu, g.L,
                       2 * g.logn, g.words);
    MFHE_CHECK_LAUNCH("ct_add_kernel");
    return MFHE_OK;
}
extern "C" int mfhe_ct_mul_tensor(mfhe_ctx* c, const uint64_t* x, const uint64_t* y, uint64_t* d0, uint64_t* d1,
                                  uint64_t* d2, mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (!x || !y || !d0 || !d1 || !d2) return set_error(MFHE_EINVAL, "mfhe_ct_mul_tensor: null pointer");
    const Geo2 g = geo(c);
    hipLaunchKernelGGL(ct_mul_kernel, g1(g.words), dim3(256), 0, (hipStream_t)s, x, y, d0, d1, d2, c->d_rns_mu,
                       c->d_r64, g.L, 2 * g.logn, g.words);
    MFHE_CHECK_LAUNCH("ct_mul_kernel");
    return MFHE_OK;
}
