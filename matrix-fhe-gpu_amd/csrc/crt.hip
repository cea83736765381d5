// crt.hip -- RNS decompose and wide CRT compose / centre-lift / f64 for gfx950.
//
// Reference semantics:
//   decompose : quantize_coeff_to_rns_kernel (batched_encoder.cu:125-152):
//               x = llround(z*delta) as int64; r = x % q (C truncation) + q if negative
//   compose   : crt_compose_centerlift_big_kernel (encoder.cu:191-230):
//               acc = sum_k M_k * ((x_k * inv_k) mod q_k) mod Q; centre-lift against Q/2
//   to_f64    : he_big_to_f64 + compose_big_pair_to_complex_by_delta (HE.cu:917-924, 1007-1027)
//
// Design: one thread per coefficient, all W words of the accumulator in
// registers (W is a template parameter, 1..32), the mod-Q reduction done once
// with an FP64 quotient estimate floor(sum_k t_k/q_k) and a single +-Q
// correction instead of the reference's per-limb compare/subtract.  Inputs are
// read limb-major so every load instruction is coalesced; the per-limb tables
// (M_k, inv_k, 1/q_k) are wave-uniform and come through the scalar cache.
#include <hip/hip_runtime.h>

#include "mfhe_ctx.hpp"

namespace mfhe {

using u128 = unsigned __int128;

// (poly, coefficient) of a flat index: a shift for power-of-two ncoeff (lg >= 0), else a 64-bit division
__device__ __forceinline__ void split_index(uint64_t i, uint64_t n, int lg, uint64_t& p, uint64_t& c) {
    if (lg >= 0) {
        p = i >> lg;
        c = i & (n - 1);
    } else {
        p = i / n;
        c = i - p * n;
    }
}
static inline int log2_or_neg(uint64_t n) {
    return (n && !(n & (n - 1))) ? __builtin_ctzll(n) : -1;
}

// ---------------- RNS decompose ----------------
__global__ __launch_bounds__(256) void rns_decompose_kernel(const double* __restrict__ in, uint64_t in_stride,
                                                            uint64_t total, uint64_t ncoeff, int lg, int L,
                                                            const uint64_t* __restrict__ qmu, double delta,
                                                            uint64_t* __restrict__ out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    uint64_t p, c;
    split_index(i, ncoeff, lg, p, c);
    const double z = in[i * in_stride] * delta;
    const long long x = llround(z);
    const bool neg = x < 0;
    const uint64_t ax = neg ? (uint64_t)0 - (uint64_t)x : (uint64_t)x;
    uint64_t* o = out + p * (uint64_t)L * ncoeff + c;
    for (int l = 0; l < L; ++l) {
        const uint64_t q = qmu[2 * l], mu = qmu[2 * l + 1];
        uint64_t r = ax - __umul64hi(ax, mu) * q;   // Barrett: [0, 2q)
        r = r >= q ? r - q : r;
        r = (neg && r) ? q - r : r;
        o[(uint64_t)l * ncoeff] = r;
    }
}

// Two coefficients per thread (ncoeff even, unit input stride, 16-B aligned buffers): one 16-B load and L
// 16-B stores per thread instead of one and L 8-B ones -- half the memory instructions for the same bytes.
__global__ __launch_bounds__(256) void rns_decompose_x2_kernel(const double2* __restrict__ in, uint64_t total2,
                                                               uint64_t ncoeff2, int lg2, int L,
                                                               const uint64_t* __restrict__ qmu, double delta,
                                                               ulonglong2* __restrict__ out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= total2) return;
    uint64_t p, c;
    split_index(i, ncoeff2, lg2, p, c);
    const double2 z = in[i];
    const long long x0 = llround(z.x * delta), x1 = llround(z.y * delta);
    const bool n0 = x0 < 0, n1 = x1 < 0;
    const uint64_t a0 = n0 ? (uint64_t)0 - (uint64_t)x0 : (uint64_t)x0;
    const uint64_t a1 = n1 ? (uint64_t)0 - (uint64_t)x1 : (uint64_t)x1;
    ulonglong2* o = out + p * (uint64_t)L * ncoeff2 + c;
    for (int l = 0; l < L; ++l) {
        const uint64_t q = qmu[2 * l], mu = qmu[2 * l + 1];
        uint64_t r0 = a0 - __umul64hi(a0, mu) * q, r1 = a1 - __umul64hi(a1, mu) * q;   // Barrett: [0, 2q)
        r0 = r0 >= q ? r0 - q : r0;
        r1 = r1 >= q ? r1 - q : r1;
        r0 = (n0 && r0) ? q - r0 : r0;
        r1 = (n1 && r1) ? q - r1 : r1;
        o[(uint64_t)l * ncoeff2] = make_ulonglong2(r0, r1);
    }
}

// ---------------- wide CRT compose ----------------
// Limb k of the coefficient is read from in[(k / Lg) * shard_stride + (k % Lg) * ncoeff]: Lg = L and
// shard_stride = 0 is the plain [npoly][L][ncoeff] layout; Lg < L reads residue shards gathered from
// several GPUs ([shard][npoly][Lg][ncoeff]) in place, without a transpose.
template <int W>
__device__ __forceinline__ void compose_slow(const uint64_t* __restrict__ in, uint64_t ncoeff, int L, int Lg,
                                          uint64_t shard_stride, const uint64_t* __restrict__ qmu,
                                          const uint64_t* __restrict__ inv, const double* __restrict__ qinv,
                                          const uint64_t* __restrict__ M, const uint64_t* __restrict__ Q,
                                          const uint64_t* __restrict__ Qh, uint64_t (&mag)[W], bool& neg) {
    uint64_t acc[W + 1];
#pragma unroll
    for (int i = 0; i <= W; ++i) acc[i] = 0;
    double est = 0.0;
    for (int k = 0, j = 0; k < L; ++k) {
        const uint64_t q = qmu[2 * k];
        const uint64_t x = in[(uint64_t)j * ncoeff];
        if (++j == Lg) {
            j = 0;
            in += shard_stride;
        }
        uint64_t t = x * inv[2 * k] - __umul64hi(x, inv[2 * k + 1]) * q;   // Shoup: [0, 2q)
        t = t >= q ? t - q : t;
        est += (double)t * qinv[k];
        const uint64_t* Mk = M + (size_t)k * W;
        uint64_t carry = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const u128 pr = (u128)t * Mk[i] + acc[i] + carry;
            acc[i] = (uint64_t)pr;
            carry = (uint64_t)(pr >> 64);
        }
        acc[W] += carry;
    }
    // subtract e*Q, e = floor(sum t_k / q_k) (exact or off by one)
    const uint64_t e = (uint64_t)__builtin_floor(est);
    {
        uint64_t carry = 0, borrow = 0;
#pragma unroll
        for (int i = 0; i <= W; ++i) {
            const u128 pr = (u128)e * (i < W ? Q[i] : 0) + carry;
            const uint64_t s = (uint64_t)pr;
            carry = (uint64_t)(pr >> 64);
            const uint64_t a = acc[i];
            const uint64_t d = a - s - borrow;
            borrow = (a < s) || (a - s < borrow);
            acc[i] = d;
        }
    }
    // result r in (-Q, 2Q): fix to [0, Q)
    if ((int64_t)acc[W] < 0) {
        uint64_t c = 0;
#pragma unroll
        for (int i = 0; i <= W; ++i) {
            const u128 s = (u128)acc[i] + (i < W ? Q[i] : 0) + c;
            acc[i] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
    } else {
        bool ge = acc[W] != 0;
        if (!ge) {
            ge = true;  // equal counts as >=
#pragma unroll
            for (int i = W - 1; i >= 0; --i) {
                if (acc[i] != Q[i]) { ge = acc[i] > Q[i]; break; }
            }
        }
        if (ge) {
            uint64_t b = 0;
#pragma unroll
            for (int i = 0; i < W; ++i) {
                const uint64_t a = acc[i], s = Q[i];
                acc[i] = a - s - b;
                b = (a < s) || (a - s < b);
            }
        }
    }
    // centre lift against Q_half = floor(Q/2)
    bool gt = false;
#pragma unroll
    for (int i = W - 1; i >= 0; --i) {
        if (acc[i] != Qh[i]) { gt = acc[i] > Qh[i]; break; }
    }
    neg = gt;
    if (gt) {
        uint64_t b = 0;
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint64_t a = Q[i], s = acc[i];
            mag[i] = a - s - b;
            b = (a < s) || (a - s < b);
        }
    } else {
#pragma unroll
        for (int i = 0; i < W; ++i) mag[i] = acc[i];
    }
}

// One limb of the FP64 fast path: t = x * inv mod q as an exact integer in (-q, q), est += t / q,
// lo += t * M0 (wrapping).
__device__ __forceinline__ void fast_f64_term(uint64_t x, const CrtLimbF& f, double& est, uint64_t& lo) {
    constexpr double kMagic = 6755399441055744.0;   // 1.5 * 2^52
    const int64_t kMagicBits = __double_as_longlong(kMagic);
    const double xv = __longlong_as_double((long long)(x | 0x4330000000000000ULL)) - 4503599627370496.0;
    const double hi = xv * f.invf;
    const double elo = __fma_rn(xv, f.invf, -hi);
    const double kq = __fma_rn(hi, f.qinvf, kMagic) - kMagic;
    const double t = __fma_rn(-kq, f.qf, hi) + elo;       // exact, |t| < q
    est = __fma_rn(t, f.qinvf, est);
    const int64_t ti = __double_as_longlong(t + kMagic) - kMagicBits;
    lo += (uint64_t)ti * f.M0;                               // wrapping
}
__device__ __forceinline__ int64_t fast_f64_candidate(double est, uint64_t lo, uint64_t Q0) {
    const int64_t u = (int64_t)__builtin_rint(est);
    return (int64_t)(lo - (uint64_t)u * Q0);
}
// q | (c - x), exactly (q odd)
__device__ __forceinline__ bool fast_f64_divides(int64_t c, uint64_t x, const CrtLimbF& f) {
    const int64_t d = c - (int64_t)x;
    const uint64_t ad = d < 0 ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
    return ad * f.qinv64 <= f.lim;
}

// FP64 small-value fast path (every q < 2^50 and odd; ctx table CrtLimbF).  Same acceptance rule as the
// integer fast path below, cheaper arithmetic: t_k = x_k * inv_k mod q_k comes from one FP64 error-free
// product as an exact integer in (-q, q) -- not canonicalised: any representative of the class gives the
// same CRT value -- est = sum_k t_k / q_k, u = rint(est), c = low64(sum_k t_k M_k - u Q) in wrapping
// int64.  c is accepted iff |c| < 2^62, |c| <= Q_half and q_k | (c - x_k) for every k, tested exactly
// as |c - x_k| * q_k^-1 mod 2^64 <= floor((2^64-1)/q_k) (q_k odd); by CRT uniqueness c is then THE
// centred value, bit-identical to compose_slow.  Residues are loaded CH limbs at a time so each thread
// has CH loads in flight; for L <= CH the divisibility pass reuses the registers.
#ifndef MFHE_CRT_NT
#define MFHE_CRT_NT 1   // the fast compose's residue loads nontemporal (read once; 0 for A/B)
#endif
template <int CH>
__device__ __forceinline__ bool compose_fast_f64(const uint64_t* __restrict__ in, uint64_t ncoeff, int L, int Lg,
                                                 uint64_t shard_stride, const CrtLimbF* __restrict__ lf,
                                                 uint64_t Q0, uint64_t Qh0, bool qbig, uint64_t& mag0, bool& neg) {
    uint64_t xs[CH];
    double est = 0.0;
    uint64_t lo = 0;
    const uint64_t* p = in;
    int j = 0;
    for (int k0 = 0; k0 < L; k0 += CH) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if (k0 + i < L) {
                xs[i] = MFHE_CRT_NT ? __builtin_nontemporal_load(p + (uint64_t)j * ncoeff) : p[(uint64_t)j * ncoeff];
                if (++j == Lg) {
                    j = 0;
                    p += shard_stride;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < CH; ++i)
            if (k0 + i < L) fast_f64_term(xs[i], lf[k0 + i], est, lo);
    }
    const int64_t c = fast_f64_candidate(est, lo, Q0);
    const uint64_t a = c < 0 ? (uint64_t)0 - (uint64_t)c : (uint64_t)c;
    bool ok = a < (1ull << 62) && (qbig || a <= Qh0);
    auto divides = [&](uint64_t x, const CrtLimbF& f) { return fast_f64_divides(c, x, f); };
    if (ok) {
        if (L <= CH) {
#pragma unroll
            for (int i = 0; i < CH; ++i)
                if (i < L) ok &= divides(xs[i], lf[i]);
        } else {
            p = in;
            j = 0;
            for (int k = 0; k < L && ok; ++k) {
                ok = divides(p[(uint64_t)j * ncoeff], lf[k]);
                if (++j == Lg) {
                    j = 0;
                    p += shard_stride;
                }
            }
        }
    }
    mag0 = a;
    neg = c < 0;
    return ok;
}

// Limbs loaded per round of the fast path: every limb of a context with L <= CH is loaded at once and its residue
// check reads the registers (the reference's L = 11: one memory round trip instead of three -- 8 + 3 loads, then the
// check's re-reads).  CH = 16 below 11 words; 32 from 11 words up (Q of >= 641 bits: the 32 x 50-bit primes of
// BASELINE C5), where 16 made the check re-read all 32 residues -- with the nontemporal first reads, from HBM: twice
// the compose's bytes (r06).
#ifndef MFHE_CRT_FAST_CH
#define MFHE_CRT_FAST_CH 16
#endif
template <int W>
constexpr int crt_fast_ch() { return W >= 11 ? 32 : MFHE_CRT_FAST_CH; }

// Small-value fast path.  With u = nearest integer to sum_k t_k/q_k, the centred CRT value is
// X = sum_k t_k M_k - u Q; its low 64 bits cost one wrapping multiply-add per limb.  The candidate
// c = (int64) low64(X) is accepted only if |c| <= Q_half and c = x_k (mod q_k) for every k: by CRT
// uniqueness it then IS the centred value, bit-identical to compose_slow.  Decoded messages (|X| ~
// delta * |m| + noise) always take it; inputs that fail the check (random residues) take the full
// W-word path.
template <int W>
__device__ __forceinline__ void compose_one(const uint64_t* __restrict__ in, uint64_t ncoeff, int L, int Lg,
                                            uint64_t shard_stride, const uint64_t* __restrict__ qmu,
                                            const uint64_t* __restrict__ inv, const double* __restrict__ qinv,
                                            const uint64_t* __restrict__ M, const uint64_t* __restrict__ Q,
                                            const uint64_t* __restrict__ Qh, uint64_t (&mag)[W], bool& neg,
                                            const CrtLimbF* __restrict__ lf, bool qbig) {
    if (lf) {
        uint64_t a0;
        if (compose_fast_f64<crt_fast_ch<W>()>(in, ncoeff, L, Lg, shard_stride, lf, Q[0], Qh[0], qbig, a0, neg)) {
            mag[0] = a0;
#pragma unroll
            for (int i = 1; i < W; ++i) mag[i] = 0;
            return;
        }
        compose_slow<W>(in, ncoeff, L, Lg, shard_stride, qmu, inv, qinv, M, Q, Qh, mag, neg);
        return;
    }
    uint64_t lo = 0;
    double est = 0.0;
    {
        const uint64_t* p = in;
        for (int k = 0, j = 0; k < L; ++k) {
            const uint64_t q = qmu[2 * k];
            const uint64_t x = p[(uint64_t)j * ncoeff];
            if (++j == Lg) {
                j = 0;
                p += shard_stride;
            }
            uint64_t t = x * inv[2 * k] - __umul64hi(x, inv[2 * k + 1]) * q;   // Shoup: [0, 2q)
            t = t >= q ? t - q : t;
            est += (double)t * qinv[k];
            lo += t * M[(size_t)k * W];                                       // wrapping
        }
    }
    const uint64_t u = (uint64_t)__builtin_rint(est);
    const int64_t c = (int64_t)(lo - u * Q[0]);
    const uint64_t a = c < 0 ? (uint64_t)0 - (uint64_t)c : (uint64_t)c;
    bool ok = a < (1ull << 62) && (qbig || a <= Qh[0]);
    {
        const uint64_t* p = in;
        for (int k = 0, j = 0; k < L && ok; ++k) {
            const uint64_t q = qmu[2 * k], mu = qmu[2 * k + 1];
            const uint64_t x = p[(uint64_t)j * ncoeff];
            if (++j == Lg) {
                j = 0;
                p += shard_stride;
            }
            uint64_t r = a - __umul64hi(a, mu) * q;   // Barrett: [0, 2q)
            r = r >= q ? r - q : r;
            r = (c < 0 && r) ? q - r : r;
            ok = r == x;
        }
    }
    if (ok) {
        mag[0] = a;
#pragma unroll
        for (int i = 1; i < W; ++i) mag[i] = 0;
        neg = c < 0;
        return;
    }
    compose_slow<W>(in, ncoeff, L, Lg, shard_stride, qmu, inv, qinv, M, Q, Qh, mag, neg);
}

template <int W>
__device__ __forceinline__ double big_to_f64(const uint64_t (&mag)[W], bool neg, double delta) {
    const double two64 = 18446744073709551616.0;
    double v = 0.0;
#pragma unroll
    for (int i = W - 1; i >= 0; --i) v = v * two64 + (double)mag[i];
    if (neg) v = -v;
    return v / delta;
}

struct CrtArgs {
    const uint64_t* in;
    uint64_t ncoeff, total;
    int L, Lg;                // limbs per shard (Lg = L: unsharded)
    uint64_t shard_stride;    // words between shards
    const uint64_t *qmu, *inv;
    const double* qinv;
    const uint64_t *M, *Q, *Qh;
    const CrtLimbF* lf;       // FP64 fast-path constants (null: integer fast path)
    bool qbig;                // Q_half >= 2^64: every |c| < 2^62 is inside (-Q/2, Q/2)
    int lg_nc;                // log2(ncoeff), or -1 when ncoeff is not a power of two
};

template <int W>
__global__ __launch_bounds__(256) void crt_compose_kernel(CrtArgs a, uint64_t* __restrict__ out_mag,
                                                          uint8_t* __restrict__ out_neg) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= a.total) return;
    uint64_t p, c;
    split_index(i, a.ncoeff, a.lg_nc, p, c);
    uint64_t mag[W];
    bool neg;
    compose_one<W>(a.in + p * (uint64_t)a.Lg * a.ncoeff + c, a.ncoeff, a.L, a.Lg, a.shard_stride, a.qmu, a.inv,
                   a.qinv, a.M, a.Q, a.Qh, mag, neg, a.lf, a.qbig);
    uint64_t* o = out_mag + i * W;
#pragma unroll
    for (int w = 0; w < W; ++w) o[w] = mag[w];
    out_neg[i] = neg ? 1 : 0;
}

// crt_compose_centerlift_kernel (encoder.cu:152-189): the centred value truncated to its low word,
// v = (int64)mag[0], out = neg ? -v : v (wrapping, as the reference's int64 negation does on the GPU)
template <int W>
__global__ __launch_bounds__(256) void crt_compose_i64_kernel(CrtArgs a, int64_t* __restrict__ out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= a.total) return;
    uint64_t p, c;
    split_index(i, a.ncoeff, a.lg_nc, p, c);
    uint64_t mag[W];
    bool neg;
    compose_one<W>(a.in + p * (uint64_t)a.Lg * a.ncoeff + c, a.ncoeff, a.L, a.Lg, a.shard_stride, a.qmu, a.inv,
                   a.qinv, a.M, a.Q, a.Qh, mag, neg, a.lf, a.qbig);
    out[i] = (int64_t)(neg ? (uint64_t)0 - mag[0] : mag[0]);
}

template <int W>
__global__ __launch_bounds__(256) void crt_compose_f64_kernel(CrtArgs a, double delta, double* __restrict__ out,
                                                              uint64_t out_stride) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= a.total) return;
    uint64_t p, c;
    split_index(i, a.ncoeff, a.lg_nc, p, c);
    uint64_t mag[W];
    bool neg;
    compose_one<W>(a.in + p * (uint64_t)a.Lg * a.ncoeff + c, a.ncoeff, a.L, a.Lg, a.shard_stride, a.qmu, a.inv,
                   a.qinv, a.M, a.Q, a.Qh, mag, neg, a.lf, a.qbig);
    out[i * out_stride] = big_to_f64<W>(mag, neg, delta);
}

// two composes of the same shape in one grid (he.hip decode: re into the even doubles, im into the odd ones): blocks
// [0, nb) compose a into oa, blocks [nb, 2 nb) compose b into ob
template <int W>
__global__ __launch_bounds__(256) void crt_compose_f64_pair_kernel(CrtArgs a, CrtArgs b, double delta, double* oa,
                                                                   double* ob, uint64_t out_stride, uint32_t nb) {
    const bool hi = blockIdx.x >= nb;
    const CrtArgs& x = hi ? b : a;
    const uint64_t i = (blockIdx.x - (hi ? nb : 0)) * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= x.total) return;
    uint64_t p, c;
    split_index(i, x.ncoeff, x.lg_nc, p, c);
    uint64_t mag[W];
    bool neg;
    compose_one<W>(x.in + p * (uint64_t)x.Lg * x.ncoeff + c, x.ncoeff, x.L, x.Lg, x.shard_stride, x.qmu, x.inv,
                   x.qinv, x.M, x.Q, x.Qh, mag, neg, x.lf, x.qbig);
    (hi ? ob : oa)[i * out_stride] = big_to_f64<W>(mag, neg, delta);
}

template <int W>
__global__ __launch_bounds__(256) void crt_to_f64_kernel(const uint64_t* __restrict__ mag_in,
                                                         const uint8_t* __restrict__ neg_in, uint64_t total,
                                                         double delta, double* __restrict__ out, uint64_t out_stride) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    uint64_t mag[W];
#pragma unroll
    for (int w = 0; w < W; ++w) mag[w] = mag_in[i * W + w];
    out[i * out_stride] = big_to_f64<W>(mag, neg_in[i] != 0, delta);
}

#define MFHE_W_CASES(X) \
    X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
    X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

static CrtArgs crt_args(const mfhe_ctx* c, const uint64_t* in, uint64_t npoly, uint64_t ncoeff) {
    CrtArgs a;
    a.in = in;
    a.ncoeff = ncoeff;
    a.total = npoly * ncoeff;
    a.lg_nc = log2_or_neg(ncoeff);
    a.L = c->L;
    a.Lg = c->L;
    a.shard_stride = 0;
    a.qmu = c->d_rns_mu;
    a.inv = c->d_crt_inv;
    a.qinv = c->d_crt_qinv;
    a.M = c->d_crt_M;
    a.Q = c->d_crt_Q;
    a.Qh = c->d_crt_Qhalf;
    a.lf = c->d_crt_lf;
    a.qbig = c->crt_qbig;
    return a;
}

static inline dim3 grid1d(uint64_t total, uint32_t th) { return dim3((uint32_t)((total + th - 1) / th)); }

}  // namespace mfhe

using namespace mfhe;

extern "C" int mfhe_rns_decompose(mfhe_ctx* c, const double* in, size_t in_stride, size_t npoly, size_t ncoeff,
                                  uint64_t* out, mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    const uint64_t total = (uint64_t)npoly * ncoeff;
    if (total == 0) return MFHE_OK;
    if (!in || !out || in_stride == 0) return set_error(MFHE_EINVAL, "mfhe_rns_decompose: bad pointer/stride");
    if (in_stride == 1 && ncoeff % 2 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0)
        hipLaunchKernelGGL(rns_decompose_x2_kernel, grid1d(total / 2, 256), dim3(256), 0, (hipStream_t)s,
                           (const double2*)in, total / 2, (uint64_t)ncoeff / 2, log2_or_neg(ncoeff / 2), c->L,
                           c->d_rns_mu, c->delta, (ulonglong2*)out);
    else
        hipLaunchKernelGGL(rns_decompose_kernel, grid1d(total, 256), dim3(256), 0, (hipStream_t)s, in,
                           (uint64_t)in_stride, total, (uint64_t)ncoeff, log2_or_neg(ncoeff), c->L, c->d_rns_mu,
                           c->delta, out);
    MFHE_CHECK_LAUNCH("rns_decompose_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_crt_compose(mfhe_ctx* c, const uint64_t* in, size_t npoly, size_t ncoeff, uint64_t* mag,
                                uint8_t* neg, mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    const uint64_t total = (uint64_t)npoly * ncoeff;
    if (total == 0) return MFHE_OK;
    if (!in || !mag || !neg) return set_error(MFHE_EINVAL, "mfhe_crt_compose: null pointer");
    const CrtArgs a = crt_args(c, in, npoly, ncoeff);
    switch (c->W) {
#define X(w) \
    case w: hipLaunchKernelGGL(crt_compose_kernel<w>, grid1d(total, 256), dim3(256), 0, (hipStream_t)s, a, mag, neg); break;
        MFHE_W_CASES(X)
#undef X
        default: return set_error(MFHE_EUNSUPPORTED, "crt words > 32");
    }
    MFHE_CHECK_LAUNCH("crt_compose_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_crt_compose_i64(mfhe_ctx* c, const uint64_t* in, size_t npoly, size_t ncoeff, int64_t* out,
                                    mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    const uint64_t total = (uint64_t)npoly * ncoeff;
    if (total == 0) return MFHE_OK;
    if (!in || !out) return set_error(MFHE_EINVAL, "mfhe_crt_compose_i64: null pointer");
    const CrtArgs a = crt_args(c, in, npoly, ncoeff);
    switch (c->W) {
#define X(w) \
    case w: hipLaunchKernelGGL(crt_compose_i64_kernel<w>, grid1d(total, 256), dim3(256), 0, (hipStream_t)s, a, out); break;
        MFHE_W_CASES(X)
#undef X
        default: return set_error(MFHE_EUNSUPPORTED, "crt words > 32");
    }
    MFHE_CHECK_LAUNCH("crt_compose_i64_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_crt_compose_f64(mfhe_ctx* c, const uint64_t* in, size_t npoly, size_t ncoeff, double* out,
                                    size_t out_stride, mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    const uint64_t total = (uint64_t)npoly * ncoeff;
    if (total == 0) return MFHE_OK;
    if (!in || !out || out_stride == 0) return set_error(MFHE_EINVAL, "mfhe_crt_compose_f64: bad pointer/stride");
    const CrtArgs a = crt_args(c, in, npoly, ncoeff);
    switch (c->W) {
#define X(w)                                                                                                       \
    case w:                                                                                                        \
        hipLaunchKernelGGL(crt_compose_f64_kernel<w>, grid1d(total, 256), dim3(256), 0, (hipStream_t)s, a, c->delta, \
                           out, (uint64_t)out_stride);                                                            \
        break;
        MFHE_W_CASES(X)
#undef X
        default: return set_error(MFHE_EUNSUPPORTED, "crt words > 32");
    }
    MFHE_CHECK_LAUNCH("crt_compose_f64_kernel");
    return MFHE_OK;
}

namespace mfhe {
// compose a -> oa and b -> ob (same npoly, ncoeff) in one launch (he.hip decode, MFHE_OPT_HE_STREAMS 2)
int crt_compose_f64_pair(mfhe_ctx* c, const uint64_t* a, const uint64_t* b, size_t npoly, size_t ncoeff, double* oa,
                         double* ob, size_t out_stride, hipStream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    const uint64_t total = (uint64_t)npoly * ncoeff;
    if (total == 0) return MFHE_OK;
    if (!a || !b || !oa || !ob || out_stride == 0) return set_error(MFHE_EINVAL, "crt_compose_f64_pair: bad pointer/stride");
    const CrtArgs ca = crt_args(c, a, npoly, ncoeff), cb = crt_args(c, b, npoly, ncoeff);
    const uint64_t nb = (total + 255) / 256;
    if (2 * nb > 0x7FFFFFFFull) return set_error(MFHE_EINVAL, "crt_compose_f64_pair: too large");
    switch (c->W) {
#define X(w)                                                                                                       \
    case w:                                                                                                        \
        hipLaunchKernelGGL(crt_compose_f64_pair_kernel<w>, dim3((uint32_t)(2 * nb)), dim3(256), 0, s, ca, cb,      \
                           c->delta, oa, ob, (uint64_t)out_stride, (uint32_t)nb);                                  \
        break;
        MFHE_W_CASES(X)
#undef X
        default: return set_error(MFHE_EUNSUPPORTED, "crt words > 32");
    }
    MFHE_CHECK_LAUNCH("crt_compose_f64_pair_kernel");
    return MFHE_OK;
}
}  // namespace mfhe

extern "C" int mfhe_crt_to_f64(mfhe_ctx* c, const uint64_t* mag, const uint8_t* neg, size_t count, double* out,
                               size_t out_stride, mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (count == 0) return MFHE_OK;
    if (!mag || !neg || !out || out_stride == 0) return set_error(MFHE_EINVAL, "mfhe_crt_to_f64: bad pointer/stride");
    switch (c->W) {
#define X(w)                                                                                                     \
    case w:                                                                                                      \
        hipLaunchKernelGGL(crt_to_f64_kernel<w>, grid1d(count, 256), dim3(256), 0, (hipStream_t)s, mag, neg,     \
                           (uint64_t)count, c->delta, out, (uint64_t)out_stride);                                \
        break;
        MFHE_W_CASES(X)
#undef X
        default: return set_error(MFHE_EUNSUPPORTED, "crt words > 32");
    }
    MFHE_CHECK_LAUNCH("crt_to_f64_kernel");
    return MFHE_OK;
}

extern "C" int mfhe_crt_compose_f64_sharded(mfhe_ctx* c, const uint64_t* in, int nshards, size_t shard_stride,
                                            size_t npoly, size_t ncoeff, double* out, size_t out_stride,
                                            mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (nshards < 1 || c->L % nshards) return set_error(MFHE_EINVAL, "mfhe_crt_compose_f64_sharded: nshards must divide L");
    const uint64_t total = (uint64_t)npoly * ncoeff;
    if (total == 0) return MFHE_OK;
    if (!in || !out || out_stride == 0) return set_error(MFHE_EINVAL, "mfhe_crt_compose_f64_sharded: bad pointer/stride");
    CrtArgs a = crt_args(c, in, npoly, ncoeff);
    a.Lg = c->L / nshards;
    a.shard_stride = (uint64_t)shard_stride;
    switch (c->W) {
#define X(w)                                                                                                       \
    case w:                                                                                                        \
        hipLaunchKernelGGL(crt_compose_f64_kernel<w>, grid1d(total, 256), dim3(256), 0, (hipStream_t)s, a, c->delta, \
                           out, (uint64_t)out_stride);                                                            \
        break;
        MFHE_W_CASES(X)
#undef X
        default: return set_error(MFHE_EUNSUPPORTED, "crt words > 32");
    }
    MFHE_CHECK_LAUNCH("crt_compose_f64_kernel");
    return MFHE_OK;
}
