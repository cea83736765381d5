// trace.hip -- batched trace GEMM: the homomorphic matrix-product stage of the scheme.
//
// Reference: src/core/batched_trace.cu:37-197 (map_Bprime_batched_kernel, trace_gemm_batched_kernel,
// rescale_by_delta_batched_kernel) and src/core/trace.cu:30-161 (the single-matrix versions).
// Planes are [batch][nlimbs][n][n] u64, one array for the real and one for the imaginary part.
//
// The reference does four `unsigned __int128 %` (a software division) per complex MAC, one thread per
// output.  Here a 256-thread workgroup computes a 64 x 64 output tile of one (batch, limb): 16-deep
// k-panels of A and B' go global -> LDS once (centred, as exact doubles), every thread holds a 4 x 4
// complex register tile, and each product is the FP64 error-free modmul of the NTT (ntt_arith.hpp).
// The accumulators are exact integers in doubles, re-reduced every KR k-steps so they stay < 2^53;
// the epilogue multiplies by n and canonicalises.  Same value mod q as the reference, so the canonical
// output is bit-identical.  Moduli >= 2^50 or n not a multiple of 64 take a u128 kernel (one output per
// thread, the reference's order of operations with a Barrett reduction in place of %).
#include <hip/hip_runtime.h>

#include <cmath>

#include "mfhe_ctx.hpp"

namespace mfhe {

namespace {

constexpr int TR_TILE = 64;   // output tile edge
constexpr int TR_KP = 16;     // k-panel depth staged in LDS
constexpr int TR_LDS = 68;    // padded row stride (doubles): 2-way conflicts on the transposing store

// (hi:lo) mod q: fold hi with r64 = 2^64 mod q, then Barrett with mu = floor(2^64 / q)
__device__ __forceinline__ uint64_t tr_mod128(unsigned __int128 v, uint64_t q, uint64_t mu, uint64_t r64) {
    uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
    while (hi) {
        const unsigned __int128 t = (unsigned __int128)hi * r64 + lo;
        hi = (uint64_t)(t >> 64);
        lo = (uint64_t)t;
    }
    uint64_t r = lo - __umul64hi(lo, mu) * q;
    r = r >= q ? r - q : r;
    return r >= q ? r - q : r;
}

// map_Bprime_batched_kernel (batched_trace.cu:37-79): conj(B), row j -> (n - j) mod n, rows j != 0 times -i.

// Per-limb epilogue constants, centred: n, 2^S, 2^2S mod q_l (S = the digit split).  Passed by value in the
// kernel arguments, so concurrent calls with different n / S on different streams never share mutable state.
constexpr int kTraceMaxLimbs = 64;
struct TraceK {
    double k[3 * kTraceMaxLimbs];
};

__global__ void trace_map_kernel(const uint64_t* __restrict__ br, const uint64_t* __restrict__ bi,
                                 uint64_t* __restrict__ opr, uint64_t* __restrict__ opi, const uint64_t* qmu,
                                 int log_n, int L, uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const uint64_t n = 1ull << log_n, n2 = n << log_n;
    const uint64_t mat = idx >> (2 * log_n), pos = idx & (n2 - 1);
    const uint64_t j = pos >> log_n, k = pos & (n - 1);
    const uint64_t q = qmu[2 * (mat % (uint64_t)L)];
    const uint64_t a = br[idx], b = bi[idx];
    const uint64_t na = a ? q - a : 0, nb = b ? q - b : 0;
    const uint64_t dst = mat * n2 + (((n - j) & (n - 1)) << log_n) + k;
    opr[dst] = j == 0 ? a : nb;
    opi[dst] = j == 0 ? nb : na;
}

// trace_gemm_batched_kernel (batched_trace.cu:99-146), FP64 tile kernel (every q < 2^50, n % 64 == 0).
// KR: k-steps between accumulator reductions; each step adds two products of magnitude < 1.5 q, so
// |acc| < (0.5 + 3 KR) q must stay below 2^53 (host picks KR = 16 for q < 2^47.4, else 2).
template <int KR>
__global__ __launch_bounds__(256) void trace_gemm_f64_kernel(
    const uint64_t* __restrict__ Ar, const uint64_t* __restrict__ Ai, const uint64_t* __restrict__ Br,
    const uint64_t* __restrict__ Bi, uint64_t* __restrict__ Cr, uint64_t* __restrict__ Ci,
    const LimbConst* __restrict__ lf, TraceK kc, int log_n, int L) {
    __shared__ double sA[2][TR_KP][TR_LDS];
    __shared__ double sB[2][TR_KP][TR_LDS];
    const int n = 1 << log_n, tdim = n / TR_TILE, tiles = tdim * tdim;
    const uint64_t mat = blockIdx.x / tiles;
    const int tile = blockIdx.x % tiles, tm = tile / tdim, tn = tile % tdim;
    const int l = (int)(mat % (uint64_t)L);
    const ArithF64 ar(lf[l]);
    const double q = ar.q, qh = 0.5 * q;
    const uint64_t base = mat << (2 * log_n);
    const uint64_t* a_re = Ar + base + (uint64_t)(tm * TR_TILE) * n;
    const uint64_t* a_im = Ai + base + (uint64_t)(tm * TR_TILE) * n;
    const uint64_t* b_re = Br + base + (uint64_t)(tn * TR_TILE) * n;
    const uint64_t* b_im = Bi + base + (uint64_t)(tn * TR_TILE) * n;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;

    double accr[4][4], acci[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) accr[i][j] = acci[i][j] = 0.0;

    for (int k0 = 0; k0 < n; k0 += TR_KP) {
        // stage: 64 rows x 16 k of each plane; a thread loads 4 elements per plane (row-contiguous 128 B runs)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int idx = tid + 256 * e, r = idx >> 4, kk = idx & 15;
            const uint64_t g = (uint64_t)r * n + k0 + kk;
            const double v0 = ArithF64::from_u64(a_re[g]), v1 = ArithF64::from_u64(a_im[g]);
            const double v2 = ArithF64::from_u64(b_re[g]), v3 = ArithF64::from_u64(b_im[g]);
            sA[0][kk][r] = v0 > qh ? v0 - q : v0;
            sA[1][kk][r] = v1 > qh ? v1 - q : v1;
            sB[0][kk][r] = v2 > qh ? v2 - q : v2;
            sB[1][kk][r] = v3 > qh ? v3 - q : v3;
        }
        __syncthreads();
#pragma unroll 2
        for (int kk = 0; kk < TR_KP; ++kk) {
            double xr[4], xi[4], yr[4], yi[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xr[i] = sA[0][kk][ty + 16 * i];
                xi[i] = sA[1][kk][ty + 16 * i];
                yr[i] = sB[0][kk][tx + 16 * i];
                yi[i] = sB[1][kk][tx + 16 * i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    accr[i][j] += ar.mulmod(xr[i], yr[j]) - ar.mulmod(xi[i], yi[j]);
                    acci[i][j] += ar.mulmod(xr[i], yi[j]) + ar.mulmod(xi[i], yr[j]);
                }
            if ((kk + 1) % KR == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        accr[i][j] = ar.reduce(accr[i][j]);
                        acci[i][j] = ar.reduce(acci[i][j]);
                    }
            }
        }
        __syncthreads();
    }
    const double nm = kc.k[3 * l];   // n mod q, centred
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t o = base + (uint64_t)(tm * TR_TILE + ty + 16 * i) * n + tn * TR_TILE + tx + 16 * j;
            Cr[o] = ar.canon(ar.mulmod(ar.reduce(accr[i][j]), nm));
            Ci[o] = ar.canon(ar.mulmod(ar.reduce(acci[i][j]), nm));
        }
}

// Split-digit variant (every q < 2^45): each centred operand is cut as x = x1 2^S + x0 with x0 centred in
// [-2^(S-1), 2^(S-1)] (S = ceil(bits(q_max) / 2)), so every digit product is an exact FP64 value <= 2^(bits-1)
// and a complex MAC is 16 plain FMAs into three exact accumulators per part (hi = x1 y1, mid = x1 y0 + x0 y1,
// lo = x0 y0) instead of four error-free modmuls (~28 ops).  |partial sums| <= 4 * 64 * 2^44 < 2^53 over any
// 64 k; the accumulators are reduced mod q every 64 k (n > 64) and folded in the epilogue as
// C = n (hi 2^2S + mid 2^S + lo) mod q with per-limb centred constants c1 = 2^S, c2 = 2^2S mod q.
// 512 threads per 64 x 64 tile, 4 x 2 outputs per thread (48 accumulator doubles).
__global__ __launch_bounds__(512) void trace_gemm_split_kernel(
    const uint64_t* __restrict__ Ar, const uint64_t* __restrict__ Ai, const uint64_t* __restrict__ Br,
    const uint64_t* __restrict__ Bi, uint64_t* __restrict__ Cr, uint64_t* __restrict__ Ci,
    const LimbConst* __restrict__ lf, TraceK kc, int log_n, int L, double two_s,
    double inv_two_s) {
    // [re hi, re lo, im hi, im lo][k][row]
    __shared__ double sA[4][TR_KP][TR_LDS];
    __shared__ double sB[4][TR_KP][TR_LDS];
    const int n = 1 << log_n, tdim = n / TR_TILE, tiles = tdim * tdim;
    const uint64_t mat = blockIdx.x / tiles;
    const int tile = blockIdx.x % tiles, tm = tile / tdim, tn = tile % tdim;
    const int l = (int)(mat % (uint64_t)L);
    const ArithF64 ar(lf[l]);
    const double q = ar.q, qh = 0.5 * q;
    const uint64_t base = mat << (2 * log_n);
    const uint64_t* src[4] = {Ar + base + (uint64_t)(tm * TR_TILE) * n, Ai + base + (uint64_t)(tm * TR_TILE) * n,
                              Br + base + (uint64_t)(tn * TR_TILE) * n, Bi + base + (uint64_t)(tn * TR_TILE) * n};
    const int tid = threadIdx.x, tx = tid & 31, ty = tid >> 5;

    double hr[4][2], mr[4][2], lr[4][2], hi[4][2], mi[4][2], li[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) hr[i][j] = mr[i][j] = lr[i][j] = hi[i][j] = mi[i][j] = li[i][j] = 0.0;

    for (int k0 = 0; k0 < n; k0 += TR_KP) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int idx = tid + 512 * e, r = idx >> 4, kk = idx & 15;
            const uint64_t g = (uint64_t)r * n + k0 + kk;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                double v = ArithF64::from_u64(src[m][g]);
                v = v > qh ? v - q : v;
                const double d1 = ArithF64::round_int(v, inv_two_s);
                const double d0 = __fma_rn(-d1, two_s, v);
                double(*dst)[TR_KP][TR_LDS] = m < 2 ? sA : sB;
                dst[2 * (m & 1)][kk][r] = d1;
                dst[2 * (m & 1) + 1][kk][r] = d0;
            }
        }
        __syncthreads();
#pragma unroll 2
        for (int kk = 0; kk < TR_KP; ++kk) {
            double a1r[4], a0r[4], a1i[4], a0i[4], b1r[2], b0r[2], b1i[2], b0i[2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a1r[i] = sA[0][kk][ty + 16 * i];
                a0r[i] = sA[1][kk][ty + 16 * i];
                a1i[i] = sA[2][kk][ty + 16 * i];
                a0i[i] = sA[3][kk][ty + 16 * i];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                b1r[j] = sB[0][kk][tx + 32 * j];
                b0r[j] = sB[1][kk][tx + 32 * j];
                b1i[j] = sB[2][kk][tx + 32 * j];
                b0i[j] = sB[3][kk][tx + 32 * j];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    hr[i][j] = __fma_rn(a1r[i], b1r[j], __fma_rn(-a1i[i], b1i[j], hr[i][j]));
                    lr[i][j] = __fma_rn(a0r[i], b0r[j], __fma_rn(-a0i[i], b0i[j], lr[i][j]));
                    mr[i][j] = __fma_rn(a1r[i], b0r[j], __fma_rn(a0r[i], b1r[j], mr[i][j]));
                    mr[i][j] = __fma_rn(-a1i[i], b0i[j], __fma_rn(-a0i[i], b1i[j], mr[i][j]));
                    hi[i][j] = __fma_rn(a1r[i], b1i[j], __fma_rn(a1i[i], b1r[j], hi[i][j]));
                    li[i][j] = __fma_rn(a0r[i], b0i[j], __fma_rn(a0i[i], b0r[j], li[i][j]));
                    mi[i][j] = __fma_rn(a1r[i], b0i[j], __fma_rn(a0r[i], b1i[j], mi[i][j]));
                    mi[i][j] = __fma_rn(a1i[i], b0r[j], __fma_rn(a0i[i], b1r[j], mi[i][j]));
                }
        }
        __syncthreads();
        if (((k0 + TR_KP) & 63) == 0 && k0 + TR_KP < n) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    hr[i][j] = ar.reduce(hr[i][j]); mr[i][j] = ar.reduce(mr[i][j]); lr[i][j] = ar.reduce(lr[i][j]);
                    hi[i][j] = ar.reduce(hi[i][j]); mi[i][j] = ar.reduce(mi[i][j]); li[i][j] = ar.reduce(li[i][j]);
                }
        }
    }
    const double nm = kc.k[3 * l], c1 = kc.k[3 * l + 1], c2 = kc.k[3 * l + 2];   // centred n, 2^S, 2^2S mod q
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint64_t o = base + (uint64_t)(tm * TR_TILE + ty + 16 * i) * n + tn * TR_TILE + tx + 32 * j;
            const double vr = ar.mulmod(ar.reduce(hr[i][j]), c2) + ar.mulmod(ar.reduce(mr[i][j]), c1) +
                              ar.reduce(lr[i][j]);
            const double vi = ar.mulmod(ar.reduce(hi[i][j]), c2) + ar.mulmod(ar.reduce(mi[i][j]), c1) +
                              ar.reduce(li[i][j]);
            Cr[o] = ar.canon(ar.mulmod(ar.reduce(vr), nm));
            Ci[o] = ar.canon(ar.mulmod(ar.reduce(vi), nm));
        }
}

// The same split-digit product on the FP64 matrix cores (v_mfma_f64_16x16x4_f64): every digit product and
// partial sum is an exact integer below 2^53, so the MFMA's fused sums are exact too.  512 threads per
// 64 x 64 tile; wave w owns rows 16 (w >> 1) .. +16 and columns 32 (w & 1) .. +32 as two 16 x 16 blocks,
// each with six accumulators (hi / mid / lo for the real and imaginary parts): 16 MFMAs per block per
// 4-deep k-step.  LDS: [plane][row][k] with a 17-double row pitch (fragment loads spread over the banks).
// Fragment maps (f64 16x16x4): A lane l = A[l & 15][k = l >> 4], B lane l = B[k = l >> 4][l & 15],
// C/D reg g of lane l = C[(l >> 4) + 4 g][l & 15].
typedef double tr_v4d __attribute__((ext_vector_type(4)));
constexpr int TR_CAP = TR_KP + 1;

struct TracePost {
    double f[64];   // per limb, centred: n * inv[l] mod q_l (fused product)
};

// FUSE: the B -> B' map is applied while staging (B' row p = f(B row (n - p) mod n)) and the rescale is
// folded into the epilogue constant (mfhe_trace_product); otherwise B' is read as given.
template <bool FUSE>
__global__ __launch_bounds__(512) void trace_gemm_split_mfma_kernel(
    const uint64_t* __restrict__ Ar, const uint64_t* __restrict__ Ai, const uint64_t* __restrict__ Br,
    const uint64_t* __restrict__ Bi, uint64_t* __restrict__ Cr, uint64_t* __restrict__ Ci,
    const LimbConst* __restrict__ lf, TraceK kc, int log_n, int L, double two_s,
    double inv_two_s, TracePost post) {
    // planes: 0 re hi, 1 re lo, 2 im hi, 3 im lo
    __shared__ double sA[4][TR_TILE * TR_CAP];
    __shared__ double sB[4][TR_TILE * TR_CAP];
    const int n = 1 << log_n, tdim = n / TR_TILE, tiles = tdim * tdim;
    const uint64_t mat = blockIdx.x / tiles;
    const int tile = blockIdx.x % tiles, tm = tile / tdim, tn = tile % tdim;
    const int l = (int)(mat % (uint64_t)L);
    const ArithF64 ar(lf[l]);
    const double q = ar.q, qh = 0.5 * q;
    const uint64_t base = mat << (2 * log_n);
    const uint64_t* src[4] = {Ar + base + (uint64_t)(tm * TR_TILE) * n, Ai + base + (uint64_t)(tm * TR_TILE) * n,
                              Br + base + (uint64_t)(tn * TR_TILE) * n, Bi + base + (uint64_t)(tn * TR_TILE) * n};
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = (w >> 1) * 16, wp = (w & 1) * 32, r = lane & 15, kq = lane >> 4;

    // acc[j][0..5] = hr, mr, lr, hi, mi, li of block j
    tr_v4d acc[2][6];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 6; ++t) acc[j][t] = tr_v4d{0, 0, 0, 0};

    for (int k0 = 0; k0 < n; k0 += TR_KP) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int idx = tid + 512 * e, row = idx >> 4, kk = idx & 15;
            const uint64_t g = (uint64_t)row * n + k0 + kk;
            double v[4];
            if (FUSE) {   // map_Bprime_batched_kernel (batched_trace.cu:57-77) on the fly
                const int j = (n - (tn * TR_TILE + row)) & (n - 1);
                const uint64_t gb = base + (uint64_t)j * n + k0 + kk;
                v[0] = ArithF64::from_u64(src[0][g]);
                v[1] = ArithF64::from_u64(src[1][g]);
                v[2] = ArithF64::from_u64(Br[gb]);
                v[3] = ArithF64::from_u64(Bi[gb]);
#pragma unroll
                for (int m = 0; m < 4; ++m) v[m] = v[m] > qh ? v[m] - q : v[m];
                const double br0 = v[2], bi0 = v[3];
                v[2] = j == 0 ? br0 : -bi0;   // conj, then times -i for rows j != 0
                v[3] = j == 0 ? -bi0 : -br0;
            } else {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    v[m] = ArithF64::from_u64(src[m][g]);
                    v[m] = v[m] > qh ? v[m] - q : v[m];
                }
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const double d1 = ArithF64::round_int(v[m], inv_two_s);
                const double d0 = __fma_rn(-d1, two_s, v[m]);
                double(*dst)[TR_TILE * TR_CAP] = m < 2 ? sA : sB;
                dst[2 * (m & 1)][row * TR_CAP + kk] = d1;
                dst[2 * (m & 1) + 1][row * TR_CAP + kk] = d0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < TR_KP / 4; ++ks) {
            const int k = ks * 4 + kq;
            const int ao = (wm + r) * TR_CAP + k;
            const double a1r = sA[0][ao], a0r = sA[1][ao], a1i = sA[2][ao], a0i = sA[3][ao];
            const double n1i = -a1i, n0i = -a0i;
            double b1r[2], b0r[2], b1i[2], b0i[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int bo = (wp + 16 * j + r) * TR_CAP + k;
                b1r[j] = sB[0][bo];
                b0r[j] = sB[1][bo];
                b1i[j] = sB[2][bo];
                b0i[j] = sB[3][bo];
            }
#define TR_MF(acc_, x_, y_) acc_ = __builtin_amdgcn_mfma_f64_16x16x4f64(x_, y_, acc_, 0, 0, 0)
            // interleave the twelve accumulators so no MFMA waits on the previous one
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                TR_MF(acc[j][0], a1r, b1r[j]);
                TR_MF(acc[j][1], a1r, b0r[j]);
                TR_MF(acc[j][2], a0r, b0r[j]);
                TR_MF(acc[j][3], a1r, b1i[j]);
                TR_MF(acc[j][4], a1r, b0i[j]);
                TR_MF(acc[j][5], a0r, b0i[j]);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                TR_MF(acc[j][0], n1i, b1i[j]);
                TR_MF(acc[j][1], a0r, b1r[j]);
                TR_MF(acc[j][2], n0i, b0i[j]);
                TR_MF(acc[j][3], a1i, b1r[j]);
                TR_MF(acc[j][4], a0r, b1i[j]);
                TR_MF(acc[j][5], a0i, b0r[j]);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                TR_MF(acc[j][1], n1i, b0i[j]);
                TR_MF(acc[j][4], a1i, b0r[j]);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                TR_MF(acc[j][1], n0i, b1i[j]);
                TR_MF(acc[j][4], a0i, b1r[j]);
            }
#undef TR_MF
        }
        __syncthreads();
        if (((k0 + TR_KP) & 63) == 0 && k0 + TR_KP < n) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int t = 0; t < 6; ++t)
#pragma unroll
                    for (int g = 0; g < 4; ++g) acc[j][t][g] = ar.reduce(acc[j][t][g]);
        }
    }
    const double nm = FUSE ? post.f[l] : kc.k[3 * l], c1 = kc.k[3 * l + 1], c2 = kc.k[3 * l + 2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const uint64_t o =
                base + (uint64_t)(tm * TR_TILE + wm + kq + 4 * g) * n + tn * TR_TILE + wp + 16 * j + r;
            const double vr = ar.mulmod(ar.reduce(acc[j][0][g]), c2) + ar.mulmod(ar.reduce(acc[j][1][g]), c1) +
                              ar.reduce(acc[j][2][g]);
            const double vi = ar.mulmod(ar.reduce(acc[j][3][g]), c2) + ar.mulmod(ar.reduce(acc[j][4][g]), c1) +
                              ar.reduce(acc[j][5][g]);
            Cr[o] = ar.canon(ar.mulmod(ar.reduce(vr), nm));
            Ci[o] = ar.canon(ar.mulmod(ar.reduce(vi), nm));
        }
}

// Any q < 2^62, any n: one output per thread, the reference's sequence (batched_trace.cu:124-144).
__global__ void trace_gemm_u128_kernel(const uint64_t* __restrict__ Ar, const uint64_t* __restrict__ Ai,
                                       const uint64_t* __restrict__ Br, const uint64_t* __restrict__ Bi,
                                       uint64_t* __restrict__ Cr, uint64_t* __restrict__ Ci, const uint64_t* qmu,
                                       const uint64_t* r64, int log_n, int L, uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int n = 1 << log_n;
    const uint64_t mat = idx >> (2 * log_n), pos = idx & ((1ull << (2 * log_n)) - 1);
    const uint64_t row = pos >> log_n, col = pos & (n - 1), base = mat << (2 * log_n);
    const int l = (int)(mat % (uint64_t)L);
    const uint64_t q = qmu[2 * l], mu = qmu[2 * l + 1], rr = r64[l];
    using u128 = unsigned __int128;
    uint64_t acc_r = 0, acc_i = 0;
    for (int t = 0; t < n; ++t) {
        const uint64_t ar = Ar[base + row * n + t], ai = Ai[base + row * n + t];
        const uint64_t br = Br[base + col * n + t], bi = Bi[base + col * n + t];
        const uint64_t rrp = tr_mod128((u128)ar * br, q, mu, rr), iip = tr_mod128((u128)ai * bi, q, mu, rr);
        const uint64_t rip = tr_mod128((u128)ar * bi, q, mu, rr), irp = tr_mod128((u128)ai * br, q, mu, rr);
        const uint64_t pr = rrp >= iip ? rrp - iip : q - (iip - rrp);
        uint64_t pi = rip + irp;
        pi = pi >= q ? pi - q : pi;
        uint64_t s = acc_r + pr;
        acc_r = s >= q ? s - q : s;
        s = acc_i + pi;
        acc_i = s >= q ? s - q : s;
    }
    const uint64_t nm = (uint64_t)n % q;
    Cr[idx] = tr_mod128((u128)acc_r * nm, q, mu, rr);
    Ci[idx] = tr_mod128((u128)acc_i * nm, q, mu, rr);
}

struct RescaleArgs {
    uint64_t w[64];    // inv[l] mod q_l
    uint64_t ws[64];   // floor(w 2^64 / q_l) (Shoup)
};

// rescale_by_delta_batched_kernel (batched_trace.cu:163-183): C *= inv[l] mod q_l
__global__ void trace_rescale_kernel(uint64_t* Cr, uint64_t* Ci, const uint64_t* qmu, RescaleArgs a, int log_n2,
                                     int L, uint64_t total) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= total) return;
    const int l = (int)((idx >> log_n2) % (uint64_t)L);
    const uint64_t q = qmu[2 * l], w = a.w[l], ws = a.ws[l];
    uint64_t x = Cr[idx], r = x * w - __umul64hi(x, ws) * q;
    Cr[idx] = r >= q ? r - q : r;
    x = Ci[idx];
    r = x * w - __umul64hi(x, ws) * q;
    Ci[idx] = r >= q ? r - q : r;
}

inline dim3 g1(uint64_t total, uint32_t th = 256) { return dim3((uint32_t)((total + th - 1) / th)); }

int trace_check(const mfhe_ctx* c, int n, int nlimbs, size_t batch, const char* what) {
    if (!c) return set_error(MFHE_EINVAL, std::string(what) + ": null ctx");
    if (n < 2 || n > 1024 || (n & (n - 1)))
        return set_error(MFHE_EINVAL, std::string(what) + ": n must be a power of two in [2, 1024]");
    if (nlimbs < 1 || nlimbs > c->L)
        return set_error(MFHE_EINVAL, std::string(what) + ": nlimbs must be in [1, ctx limbs]");
    if (batch == 0) return set_error(MFHE_EINVAL, std::string(what) + ": batch must be >= 1");
    return MFHE_OK;
}

int ilog2(int n) { return 31 - __builtin_clz((unsigned)n); }

TraceK trace_consts(const mfhe_ctx* c, int n, int S, int nlimbs) {
    auto centred = [](uint64_t v, uint64_t q) { return v > q / 2 ? (double)v - (double)q : (double)v; };
    TraceK k{};
    for (int l = 0; l < nlimbs && l < kTraceMaxLimbs; ++l) {
        const uint64_t q = c->moduli[l];
        const uint64_t t1 = (uint64_t)(((unsigned __int128)1 << S) % q);
        k.k[3 * l] = centred((uint64_t)n % q, q);
        k.k[3 * l + 1] = centred(t1, q);
        k.k[3 * l + 2] = centred((uint64_t)((unsigned __int128)t1 * t1 % q), q);
    }
    return k;
}

}  // namespace
}  // namespace mfhe

using namespace mfhe;

extern "C" int mfhe_trace_map_bprime(mfhe_ctx* c, const uint64_t* br, const uint64_t* bi, uint64_t* opr,
                                     uint64_t* opi, int n, int nlimbs, size_t batch, mfhe_stream_t s) {
    if (int rc = trace_check(c, n, nlimbs, batch, "mfhe_trace_map_bprime")) return rc;
    if (!br || !bi || !opr || !opi) return set_error(MFHE_EINVAL, "mfhe_trace_map_bprime: null pointer");
    if (br == opr || bi == opi || br == opi || bi == opr)
        return set_error(MFHE_EINVAL, "mfhe_trace_map_bprime: output must not alias input");
    const uint64_t total = (uint64_t)batch * nlimbs * n * n;
    hipLaunchKernelGGL(trace_map_kernel, g1(total), dim3(256), 0, (hipStream_t)s, br, bi, opr, opi, c->d_rns_mu,
                       ilog2(n), nlimbs, total);
    MFHE_CHECK_LAUNCH("trace_map_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_trace_gemm(mfhe_ctx* c, const uint64_t* ar, const uint64_t* ai, const uint64_t* bpr,
                               const uint64_t* bpi, uint64_t* cr, uint64_t* ci, int n, int nlimbs, size_t batch,
                               mfhe_stream_t s) {
    if (int rc = trace_check(c, n, nlimbs, batch, "mfhe_trace_gemm")) return rc;
    if (!ar || !ai || !bpr || !bpi || !cr || !ci) return set_error(MFHE_EINVAL, "mfhe_trace_gemm: null pointer");
    for (const uint64_t* o : {cr, ci})
        if (o == ar || o == ai || o == bpr || o == bpi)
            return set_error(MFHE_EINVAL, "mfhe_trace_gemm: outputs must not overlap the inputs (other tiles still read them)");
    const uint64_t total = (uint64_t)batch * nlimbs * n * n;
    const int log_n = ilog2(n);
    if (c->f64_ok && n % TR_TILE == 0 && nlimbs <= kTraceMaxLimbs) {
        uint64_t qmax = 0;
        for (int l = 0; l < nlimbs; ++l) qmax = c->moduli[l] > qmax ? c->moduli[l] : qmax;
        const int qbits = 64 - __builtin_clzll(qmax);
        const int S = (qbits + 1) / 2;
        const bool split = c->trace_split && qbits <= 45;
        const TraceK kc = trace_consts(c, n, S, nlimbs);
        const uint64_t blocks = (uint64_t)batch * nlimbs * (n / TR_TILE) * (n / TR_TILE);
        if (blocks > 0x7fffffffull) return set_error(MFHE_EINVAL, "mfhe_trace_gemm: batch too large");
        if (split && c->trace_split == 2) {
            hipLaunchKernelGGL(trace_gemm_split_mfma_kernel<false>, dim3((uint32_t)blocks), dim3(512), 0,
                               (hipStream_t)s, ar, ai, bpr, bpi, cr, ci, c->d_limbs, kc, log_n, nlimbs,
                               std::ldexp(1.0, S), std::ldexp(1.0, -S), TracePost{});
            MFHE_CHECK_LAUNCH("trace_gemm_split_mfma_kernel");
            return MFHE_OK;
        }
        if (split) {
            hipLaunchKernelGGL(trace_gemm_split_kernel, dim3((uint32_t)blocks), dim3(512), 0, (hipStream_t)s, ar, ai,
                               bpr, bpi, cr, ci, c->d_limbs, kc, log_n, nlimbs, std::ldexp(1.0, S),
                               std::ldexp(1.0, -S));
            MFHE_CHECK_LAUNCH("trace_gemm_split_kernel");
            return MFHE_OK;
        }
        if ((double)qmax * 48.5 < 9007199254740992.0)   // (0.5 + 3 * 16) q < 2^53
            hipLaunchKernelGGL(trace_gemm_f64_kernel<16>, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)s, ar,
                               ai, bpr, bpi, cr, ci, c->d_limbs, kc, log_n, nlimbs);
        else
            hipLaunchKernelGGL(trace_gemm_f64_kernel<2>, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)s, ar,
                               ai, bpr, bpi, cr, ci, c->d_limbs, kc, log_n, nlimbs);
        MFHE_CHECK_LAUNCH("trace_gemm_f64_kernel");
        return MFHE_OK;
    }
    hipLaunchKernelGGL(trace_gemm_u128_kernel, g1(total), dim3(256), 0, (hipStream_t)s, ar, ai, bpr, bpi, cr, ci,
                       c->d_rns_mu, c->d_r64, log_n, nlimbs, total);
    MFHE_CHECK_LAUNCH("trace_gemm_u128_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_trace_rescale(mfhe_ctx* c, uint64_t* cr, uint64_t* ci, int n, int nlimbs, size_t batch,
                                  const uint64_t* inv, mfhe_stream_t s) {
    if (int rc = trace_check(c, n, nlimbs, batch, "mfhe_trace_rescale")) return rc;
    if (!cr || !ci || !inv) return set_error(MFHE_EINVAL, "mfhe_trace_rescale: null pointer");
    if (nlimbs > 64) return set_error(MFHE_EINVAL, "mfhe_trace_rescale: at most 64 limbs");
    RescaleArgs a{};
    for (int l = 0; l < nlimbs; ++l) {
        const uint64_t q = c->moduli[l];
        a.w[l] = inv[l] % q;
        a.ws[l] = (uint64_t)(((unsigned __int128)a.w[l] << 64) / q);
    }
    const uint64_t total = (uint64_t)batch * nlimbs * n * n;
    hipLaunchKernelGGL(trace_rescale_kernel, g1(total), dim3(256), 0, (hipStream_t)s, cr, ci, c->d_rns_mu, a,
                       2 * ilog2(n), nlimbs, total);
    MFHE_CHECK_LAUNCH("trace_rescale_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_trace_product(mfhe_ctx* c, const uint64_t* ar, const uint64_t* ai, const uint64_t* br,
                                  const uint64_t* bi, uint64_t* cr, uint64_t* ci, int n, int nlimbs, size_t batch,
                                  const uint64_t* inv, mfhe_stream_t s) {
    if (int rc = trace_check(c, n, nlimbs, batch, "mfhe_trace_product")) return rc;
    if (!ar || !ai || !br || !bi || !cr || !ci) return set_error(MFHE_EINVAL, "mfhe_trace_product: null pointer");
    for (const uint64_t* o : {cr, ci})
        if (o == ar || o == ai || o == br || o == bi)
            return set_error(MFHE_EINVAL, "mfhe_trace_product: outputs must not overlap the inputs (other tiles still read them)");
    uint64_t qmax = 0;
    for (int l = 0; l < nlimbs; ++l) qmax = c->moduli[l] > qmax ? c->moduli[l] : qmax;
    if (!c->f64_ok || n % TR_TILE != 0 || 64 - __builtin_clzll(qmax) > 45 || nlimbs > kTraceMaxLimbs)
        return set_error(MFHE_EUNSUPPORTED, "mfhe_trace_product: needs n % 64 == 0, every q < 2^45, nlimbs <= 64 "
                                            "(use mfhe_trace_map_bprime + mfhe_trace_gemm + mfhe_trace_rescale)");
    // per-limb constants for this n and digit split (same table as mfhe_trace_gemm)
    const int qbits = 64 - __builtin_clzll(qmax), S = (qbits + 1) / 2;
    const TraceK kc = trace_consts(c, n, S, nlimbs);
    TracePost post{};
    for (int l = 0; l < nlimbs; ++l) {
        const uint64_t q = c->moduli[l], nm = (uint64_t)n % q;
        const uint64_t f = inv ? (uint64_t)((unsigned __int128)nm * (inv[l] % q) % q) : nm;
        post.f[l] = f > q / 2 ? (double)f - (double)q : (double)f;
    }
    const uint64_t blocks = (uint64_t)batch * nlimbs * (n / TR_TILE) * (n / TR_TILE);
    if (blocks > 0x7fffffffull) return set_error(MFHE_EINVAL, "mfhe_trace_product: batch too large");
    hipLaunchKernelGGL(trace_gemm_split_mfma_kernel<true>, dim3((uint32_t)blocks), dim3(512), 0, (hipStream_t)s, ar,
                       ai, br, bi, cr, ci, c->d_limbs, kc, ilog2(n), nlimbs, std::ldexp(1.0, S),
                       std::ldexp(1.0, -S), post);
    MFHE_CHECK_LAUNCH("trace_gemm_split_mfma_kernel<fused>");
    return MFHE_OK;
}
