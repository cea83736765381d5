// ring_row.hpp -- the fused X-axis ring product of one length-n row (n = 4..64) and its 32-byte row I/O,
// shared by the encrypt / decrypt row kernels (he.hip) and the decrypt-fused inverse W-CRT digitize (gemm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ntt_arith.hpp"

#ifndef MFHE_RING_LDS
#define MFHE_RING_LDS 1   // n = 64 row products through ring_mul_row64_lds (0: the shuffle ring_mul_row, A/B only)
#endif

namespace mfhe {

// ---------------- fused X-axis ring product (n = 4..64) ----------------
// t = INTT(NTT(a) (.) s) for one length-n row, phantom convention (the ph tables of mfhe_ntt_fwd/_inv, so
// s = mfhe_ntt_fwd(secret) is in the matching order): the reference's xy_ntt_forward_phantom ->
// pointwise_mul_s_kernel -> xy_ntt_backward_phantom (HE.cu:1500-1530, 1575-1590) without the three HBM
// round trips.  T = n/4 lanes per row, lane j holds coefficients 4j..4j+3; butterflies at distance
// t >= 4 pair lane j with lane j ^ (t/4), each lane of the pair computing two of the four butterflies;
// t = 1, 2 stay in the lane.
// FP64 exact modmul (ntt_arith.hpp), q < 2^50.  Bounds (r06): a mulmod of |v| <= 4q by a centred |w| <= q/2 is
// within q (|hi - k q| <= q/2 + |hi| 2^-53 <= 0.75 q, |lo| <= ulp(hi) / 2 <= q / 4) and needs |v w / q| < 2^51, i.e.
// |v| <= 4q.  Forward: the input is canonical (< q) and each CT stage adds at most q, so the fourth stage's v is
// <= 4q; one centred reduction after stage 4 (r05: after every second stage); stages 5-6 end <= 2.5q, the input of
// the product with s.  Inverse: X is left unreduced on every other stage starting with the first (as
// ArithF64::gs_lazy: a lazy stage's inputs are <= q, so its X < 2q and the next stage's |u - v| < 4q), the last
// stage scales by n^-1 with a mulmod.  Canonical outputs are the same for every schedule.
template <int LOGN>
__device__ __forceinline__ void ring_mul_row(double (&x)[4], const double (&sv)[4], int j, const ArithF64& ar,
                                             const double* __restrict__ tw, const double* __restrict__ itw,
                                             double ninv) {
#pragma unroll
    for (int st = 0; st < LOGN; ++st) {   // forward CT: m = 2^st, t = n / 2m, W = tw[m + k / 2t]
        const int m = 1 << st, lt = LOGN - 1 - st, t = 1 << lt;
        if (t >= 4) {
            // lanes j (lower) and j ^ d (upper) pair slot by slot; the lower lane computes slots 0, 1 and the
            // upper slots 2, 3 (two shuffles in, two out, two modmuls per lane)
            const int d = t >> 2;
            const bool up = j & d;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const double recv = __shfl_xor(up ? x[k] : x[k + 2], d);
                const double u = up ? recv : x[k], v = up ? x[k + 2] : recv;
                const double mv = ar.mulmod(v, tw[m + ((4 * j + (up ? k + 2 : k)) >> (lt + 1))]);
                const double X = u + mv, Y = u - mv;
                const double back = __shfl_xor(up ? X : Y, d);
                x[k] = up ? back : X;
                x[k + 2] = up ? Y : back;
            }
        } else if (t == 2) {
            const double w = tw[m + j];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const double mv = ar.mulmod(x[a + 2], w);
                x[a + 2] = x[a] - mv;
                x[a] += mv;
            }
        } else {
#pragma unroll
            for (int a = 0; a < 4; a += 2) {
                const double mv = ar.mulmod(x[a + 1], tw[m + 2 * j + a / 2]);
                x[a + 1] = x[a] - mv;
                x[a] += mv;
            }
        }
        if (st == 3)
#pragma unroll
            for (int s = 0; s < 4; ++s) x[s] = ar.reduce(x[s]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) x[s] = ar.mulmod(x[s], sv[s]);
#pragma unroll
    for (int st = LOGN - 1; st >= 0; --st) {   // inverse GS: X = u + v, Y = (u - v) W; m = 1 scales by n^-1
        const int m = 1 << st, lt = LOGN - 1 - st, t = 1 << lt;
        const bool last = st == 0, lazy = (LOGN - 1 - st) % 2 == 0;
        auto xsum = [&](double u) { return last ? ar.mulmod(u, ninv) : (lazy ? u : ar.reduce(u)); };
        if (t >= 4) {
            const int d = t >> 2;
            const bool up = j & d;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const double recv = __shfl_xor(up ? x[k] : x[k + 2], d);
                const double u = up ? recv : x[k], v = up ? x[k + 2] : recv;
                const double X = xsum(u + v);
                const double Y = ar.mulmod(u - v, itw[m + ((4 * j + (up ? k + 2 : k)) >> (lt + 1))]);
                const double back = __shfl_xor(up ? X : Y, d);
                x[k] = up ? back : X;
                x[k + 2] = up ? Y : back;
            }
        } else if (t == 2) {
            const double w = itw[m + j];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                const double u = x[a], v = x[a + 2];
                x[a] = xsum(u + v);
                x[a + 2] = ar.mulmod(u - v, w);
            }
        } else {
#pragma unroll
            for (int a = 0; a < 4; a += 2) {
                const double u = x[a], v = x[a + 1];
                x[a] = xsum(u + v);
                x[a + 1] = ar.mulmod(u - v, itw[m + 2 * j + a / 2]);
            }
        }
    }
}

// The same product for n = 64 with every butterfly inside a lane: 16 lanes per row, three register layouts
//   A: reg m of lane j = coefficient j + 16 m      (stages t = 32, 16)
//   B: reg m of lane j = 16 (j / 4) + j % 4 + 4 m  (stages t = 8, 4)
//   C: reg m of lane j = 4 j + m                   (stages t = 2, 1, and the product with s)
// and a transpose through the row's LDS scratch `scr` (68 doubles: slot s at s + s / 16, bank-spread) between
// them.  ring_mul_row pairs lanes by shuffles instead, with a select per value moved (about 190 v_cndmask per
// row product); here the butterflies are the same operations in the same order on the same values (the reduce
// schedule too), so the canonical outputs are identical.  In and out in layout A; s in layout C.  The 16 lanes of
// a row are in one wave: the transposes need no barrier, only the wave's in-order LDS (the compiler is held by
// the memory clobbers).
// IN_C: x arrives in layout C (4 j + m, one 32-byte load per lane) and is transposed to A first.
template <bool IN_C = false>
__device__ __forceinline__ void ring_mul_row64_lds(double (&x)[4], const double (&sv)[4], int j, const ArithF64& ar,
                                                   const double* __restrict__ tw, const double* __restrict__ itw,
                                                   double ninv, double* scr) {
    const int b = j >> 2, c = j & 3;
    auto slot = [](int s) { return s + (s >> 4); };
    auto ct = [&](int i0, int i1, double w) {
        const double mv = ar.mulmod(x[i1], w);
        x[i1] = x[i0] - mv;
        x[i0] += mv;
    };
    auto gs = [&](int i0, int i1, double w, bool last, bool lazy = false) {
        const double u = x[i0], v = x[i1];
        x[i0] = last ? ar.mulmod(u + v, ninv) : (lazy ? u + v : ar.reduce(u + v));
        x[i1] = ar.mulmod(u - v, w);
    };
    auto red = [&]() {
#pragma unroll
        for (int m = 0; m < 4; ++m) x[m] = ar.reduce(x[m]);
    };
    const int sA = j, sB = 16 * b + c, sC = 4 * j;   // slot of reg 0; reg m adds 16 m / 4 m / m
    auto xchg = [&](int ws, int wstep, int rs, int rstep) {
#pragma unroll
        for (int m = 0; m < 4; ++m) scr[slot(ws + wstep * m)] = x[m];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int m = 0; m < 4; ++m) x[m] = scr[slot(rs + rstep * m)];
        asm volatile("" ::: "memory");   // the next transpose's writes stay behind these reads
    };
    if constexpr (IN_C) xchg(sC, 1, sA, 16);
    // forward (CT, W = tw[m + e / 2t])
    ct(0, 2, tw[1]);
    ct(1, 3, tw[1]);
    ct(0, 1, tw[2]);
    ct(2, 3, tw[3]);
    xchg(sA, 16, sB, 4);
    ct(0, 2, tw[4 + b]);
    ct(1, 3, tw[4 + b]);
    ct(0, 1, tw[8 + 2 * b]);
    ct(2, 3, tw[9 + 2 * b]);
    red();
    xchg(sB, 4, sC, 1);
    ct(0, 2, tw[16 + j]);
    ct(1, 3, tw[16 + j]);
    ct(0, 1, tw[32 + 2 * j]);
    ct(2, 3, tw[33 + 2 * j]);
#pragma unroll
    for (int m = 0; m < 4; ++m) x[m] = ar.mulmod(x[m], sv[m]);
    // inverse (GS, W = itw[m + e / 2t]; the last stage scales X by n^-1)
    gs(0, 1, itw[32 + 2 * j], false, true);
    gs(2, 3, itw[33 + 2 * j], false, true);
    gs(0, 2, itw[16 + j], false);
    gs(1, 3, itw[16 + j], false);
    xchg(sC, 1, sB, 4);
    gs(0, 1, itw[8 + 2 * b], false, true);
    gs(2, 3, itw[9 + 2 * b], false, true);
    gs(0, 2, itw[4 + b], false);
    gs(1, 3, itw[4 + b], false);
    xchg(sB, 4, sA, 16);
    gs(0, 1, itw[2], false, true);
    gs(2, 3, itw[3], false, true);
    gs(0, 2, itw[1], true);
    gs(1, 3, itw[1], true);
}

// 4 consecutive u64 (32-byte aligned) as two 16-byte accesses
template <bool NT = false>
__device__ __forceinline__ void ld4(const uint64_t* p, uint64_t (&v)[4]) {
    if constexpr (NT) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        const u64x2 a = __builtin_nontemporal_load((const u64x2*)p), b = __builtin_nontemporal_load((const u64x2*)(p + 2));
        v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
    } else {
        const ulonglong2 a = *(const ulonglong2*)p, b = *(const ulonglong2*)(p + 2);
        v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
    }
}
__device__ __forceinline__ void st4(uint64_t* p, const uint64_t (&v)[4]) {
    *(ulonglong2*)p = make_ulonglong2(v[0], v[1]);
    *(ulonglong2*)(p + 2) = make_ulonglong2(v[2], v[3]);
}

// lane j's four coefficients of a row starting at p: 4 j .. 4 j + 3 (ring_mul_row), or j + 16 s (ring_mul_row64_lds,
// A = true: four 8-byte accesses, each a 128-byte sweep over the row's 16 lanes)
// NT: nontemporal (streamed once, no reuse: MFHE_ENC_NT)
template <bool A, bool NT = false>
__device__ __forceinline__ void ld_row(const uint64_t* p, int j, uint64_t (&v)[4]) {
    if constexpr (A) {
#pragma unroll
        for (int s = 0; s < 4; ++s) v[s] = NT ? __builtin_nontemporal_load(p + j + 16 * s) : p[j + 16 * s];
    } else {
        ld4(p + 4 * j, v);
    }
}
template <bool A, bool NT = false>
__device__ __forceinline__ void st_row(uint64_t* p, int j, const uint64_t (&v)[4]) {
    if constexpr (A) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if constexpr (NT) __builtin_nontemporal_store(v[s], p + j + 16 * s);
            else p[j + 16 * s] = v[s];
        }
    } else {
        st4(p + 4 * j, v);
    }
}

__device__ __forceinline__ double centred_f(uint64_t v, double q) {
    const double d = ArithF64::from_u64(v);
    return d > 0.5 * q ? d - q : d;
}

}  // namespace mfhe
