// ntt_arith.hpp -- modular arithmetic policies for the CDNA4 NTT kernels.
//
// Two interchangeable policies drive the same butterfly network:
//
//  * ArithF64 -- residues held as exact integers in IEEE doubles (q < 2^50).
//    A modmul is an error-free transformation: hi = v*w, lo = fma(v,w,-hi),
//    k = rint(v*w/q), t = fma(-k,q,hi) + lo.  Every step is exact while
//    |values| < 2^53, which the reduction schedule guarantees (DESIGN.md
//    §Arithmetic).  Measured on gfx950: 2.1e12 butterflies/s vs 1.3e12 for the
//    64-bit integer Shoup butterfly (profiles/r01_microbench_modmul.txt).
//
//  * ArithU64 -- Harvey lazy butterflies with Shoup precomputation, exactly the
//    phantom fnwt/inwt arithmetic: values in [0,4q), q < 2^62.
//    Used when any modulus is >= 2^50 and for the phantom fnwt_1d/inwt_1d surface,
//    whose callers hand us u64 Shoup tables.
//
//  * ArithU60 -- the same Shoup products with lazier reduction schedules, for forward and
//    inverse transforms of contexts whose moduli are all < 2^60 (below).
//
// All produce canonical [0,q) outputs, so results are bit-identical to each
// other and to the phantom/reference transforms they restate.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>

namespace mfhe {

constexpr double kTwo52 = 4503599627370496.0;          // 2^52
constexpr uint64_t kExp52 = 0x4330000000000000ULL;      // bits of 2^52

// Per-limb constants passed to kernels.
struct LimbConst {
    uint64_t q;
    double qf, qinv;
    uint64_t pad;
};

struct ArithF64 {
    using T = double;
    using Tw = double;       // w centred in (-q/2, q/2]
    double q, qinv;

    __device__ __forceinline__ explicit ArithF64(const LimbConst& c) : q(c.qf), qinv(c.qinv) {}

    // canonical u64 (< 2^52) -> exact double
    __device__ __forceinline__ static double from_u64(uint64_t x) {
        return __longlong_as_double((long long)(x | kExp52)) - kTwo52;
    }
    // intermediate representation between passes: raw double bits
    __device__ __forceinline__ static double from_raw(uint64_t x) { return __longlong_as_double((long long)x); }
    __device__ __forceinline__ static uint64_t to_raw(double x) { return (uint64_t)__double_as_longlong(x); }

    // Round-to-integer by the 1.5*2^52 magic constant: fma(a, b, C) - C = nearest integer to a*b for
    // |a*b| < 2^51, two full-rate FP64 ops (v_rndne_f64 is not full rate on gfx950).  The quotient
    // only has to be within +-1 of v*w/q for the bounds below; canonical outputs do not depend on it.
    static constexpr double kMagic = 6755399441055744.0;   // 1.5 * 2^52
    __device__ __forceinline__ static double round_int(double a, double b) { return __fma_rn(a, b, kMagic) - kMagic; }

    // t = v*w mod q (exact integer in a double): hi + lo = v*w exactly, k = round(hi / q) (within 1 of
    // v*w/q), t = (hi - k q) + lo; needs |v w / q| < 2^51.  The quotient comes from hi, so the twiddle
    // table holds w alone (8 B per entry instead of a (w, w/q) pair).
    __device__ __forceinline__ double mulmod(double v, Tw w) const {
        double hi = v * w;
        double lo = __fma_rn(v, w, -hi);
        double k = round_int(hi, qinv);
        return __fma_rn(-k, q, hi) + lo;
    }
    // centred reduction: |result| <= q/2 (+ negligible) for |x| < 2^51 q
    __device__ __forceinline__ double reduce(double x) const {
        return __fma_rn(-round_int(x, qinv), q, x);
    }
    // Cooley-Tukey: (u, v) <- (u + wv, u - wv)
    __device__ __forceinline__ void ct(double& u, double& v, Tw w) const {
        double t = mulmod(v, w);
        double a = u;
        u = a + t;
        v = a - t;
    }
    // Gentleman-Sande: (u, v) <- (u + v, (u - v) w); X re-reduced (it doubles per stage)
    __device__ __forceinline__ void gs(double& u, double& v, Tw w) const {
        double a = u, b = v;
        u = reduce(a + b);
        v = mulmod(a - b, w);
    }
    // GS without reducing X: used on every other inverse stage.  Inputs of a lazy stage are outputs of a
    // reduced stage (|x| <= 0.83 q: centred reduce or mulmod with a +-1 quotient) or canonical (< q), so
    // its X outputs stay < 2q and the next (reducing) stage sees |u - v| < 4q: |(u - v) w / q| < 2^51
    // with centred |w| <= q/2 and q < 2^50, inside mulmod's rounding range.
    __device__ __forceinline__ void gs_lazy(double& u, double& v, Tw w) const {
        double a = u, b = v;
        u = a + b;
        v = mulmod(a - b, w);
    }
    // start-of-round reduction (keeps CT growth bounded)
    __device__ __forceinline__ double round_reduce(double x) const { return reduce(x); }
    __device__ __forceinline__ void ct_first(double& u, double& v, Tw w) const { ct(u, v, w); }
    __device__ __forceinline__ uint64_t raw_out(double x) const { return to_raw(reduce(x)); }
    // exact canonical u64 in [0, q)
    __device__ __forceinline__ uint64_t canon(double x) const {
        double r = reduce(x);          // |r| <= q/2 + eps
        r = (r < 0.0) ? r + q : r;     // [0, q)
        return (uint64_t)__double_as_longlong(r + kTwo52) & 0x000FFFFFFFFFFFFFULL;
    }
};

// hi64(a * b) with four multiplies and two glue instructions.  hi64 = ah bh + floor(S / 2^32), S = al bh + ah bl +
// hi32(al bl) < 2^65: A = al bh + hi32(al bl) cannot overflow, the second middle product is accumulated by
// v_mad_u64_u32 with its carry-out (an SGPR lane mask), and (carry, B >> 32) is the pair the last multiply adds.
// __umul64hi's lowering re-pairs each 32-bit half with a zero register instead: 3-4 v_mov per call (tools/isa_mix.py).
__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) {
    const uint32_t al = (uint32_t)a, ah = (uint32_t)(a >> 32), bl = (uint32_t)b, bh = (uint32_t)(b >> 32);
    const uint64_t A = (uint64_t)al * bh + __umulhi(al, bl);
    uint64_t B, c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(B), "=s"(c) : "v"(ah), "v"(bl), "v"(A));
    uint32_t ci;
    asm("v_cndmask_b32 %0, 0, 1, %1" : "=v"(ci) : "s"(c));
    return (uint64_t)ah * bh + (((uint64_t)ci << 32) | (uint32_t)(B >> 32));
}

struct ArithU64 {
    using T = uint64_t;
    using Tw = ulonglong2;   // (w, floor(w 2^64 / q))
    // q < 2^62.  Every 64-bit subtraction of a value is an addition of its negation (one v_lshl_add_u64, no
    // carry through VCC: a v_sub_co / v_subb_co pair reads the VCC the first one wrote, which costs wait
    // states on gfx950), and every conditional subtraction is a select on the sign of the difference
    // (v_bfi_b32 on a v_ashrrev mask, no compare).
    uint64_t q, two_q, nq, n2q;   // nq = -q, n2q = -2q (mod 2^64)

    __device__ __forceinline__ explicit ArithU64(const LimbConst& c, bool pin = true)
        : q(c.q), two_q(2 * c.q), nq(0 - c.q), n2q(0 - 2 * c.q) {
        // held as values: otherwise x + n2q is re-derived from q as a v_mad_u64_u32 by -2 (a quarter-rate
        // multiply) in every butterfly
        if (pin) {
            asm volatile("" : "+v"(nq));
            asm volatile("" : "+v"(n2q));
        }
    }

    __device__ __forceinline__ static uint64_t from_u64(uint64_t x) { return x; }
    __device__ __forceinline__ static uint64_t from_raw(uint64_t x) { return x; }
    __device__ __forceinline__ static uint64_t to_raw(uint64_t x) { return x; }

    // d = x - m (mod 2^64) with 0 <= x < 2m, m <= 2^63: x if d wrapped (top bit set), else d -- one shift for
    // the mask and a bit-field insert per half
    __device__ __forceinline__ static uint64_t sel_sub(uint64_t x, uint64_t d) {
        const uint32_t dl = (uint32_t)d, dh = (uint32_t)(d >> 32), xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
        const uint32_t msk = (uint32_t)((int32_t)dh >> 31);
        uint32_t rl, rh;
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(rl) : "v"(msk), "v"(xl), "v"(dl));
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(rh) : "v"(msk), "v"(xh), "v"(dh));
        return ((uint64_t)rh << 32) | rl;
    }
    // Shoup: v*w + hi64(v*w')*(-q) in [0,2q) for any v < 2^64
    __device__ __forceinline__ uint64_t mulmod(uint64_t v, Tw w) const {
        return v * w.x + mulhi64(v, w.y) * nq;
    }
    __device__ __forceinline__ uint64_t reduce(uint64_t x) const {   // [0,4q) -> [0,2q)
        return sel_sub(x, x + n2q);
    }
    // Harvey CT: u in [0,4q), v < 2^64 -> outputs in [0,4q)
    __device__ __forceinline__ void ct(uint64_t& u, uint64_t& v, Tw w) const {
        uint64_t t = mulmod(v, w);
        uint64_t a = reduce(u);
        u = a + t;
        v = a - t + two_q;
    }
    // Harvey GS: u, v in [0,2q) -> outputs in [0,2q)
    __device__ __forceinline__ void gs(uint64_t& u, uint64_t& v, Tw w) const {
        uint64_t a = u, b = v;
        u = reduce(a + b);
        v = mulmod(a - b + two_q, w);
    }
    __device__ __forceinline__ void gs_lazy(uint64_t& u, uint64_t& v, Tw w) const { gs(u, v, w); }
    __device__ __forceinline__ uint64_t round_reduce(uint64_t x) const { return x; }
    __device__ __forceinline__ uint64_t canon(uint64_t x) const {
        x = sel_sub(x, x + n2q);
        return sel_sub(x, x + nq);
    }
    // first CT stage of a round (executed-stage order) and the raw intermediate a pass writes: the Harvey policy
    // reduces in every butterfly, so these are its ordinary ct / reduce
    __device__ __forceinline__ void ct_first(uint64_t& u, uint64_t& v, Tw w) const { ct(u, v, w); }
    __device__ __forceinline__ uint64_t raw_out(uint64_t x) const { return reduce(x); }
};

// ArithU60 -- transforms when every modulus of the context is < 2^60 (phantom's and SEAL's range): 16q < 2^64 leaves
// room for lazier schedules than Harvey's reduce-per-butterfly.  Forward:
//  * Values enter a round (an exchange-to-exchange run of <= 4 stages) below 16q.  Only the u inputs of the round's
//    first stage are reduced, once, to [0, 8q) (one select by 8q); every CT adds at most 2q to the bound of its u
//    input (u' = u + t, v' = u + 2q - t, t = Shoup product in [0, 2q) for any v < 2^64), so after 4 stages every
//    value is below 8q + 8q = 16q again.  The v inputs never need a bound below 2^64.
//  * A pass's raw intermediate is written unreduced (< 16q; the next pass's first stage reduces it) and the final
//    canonicalisation is four selects (8q, 4q, 2q, q).
//  * The Shoup product sums lo64(v w) and lo64(Q (-q)) in one mad chain: two v_mad_u64_u32 for the low halves, the
//    four cross products into the high word by two v_add3.
// VALU instructions per thread and tile: column pass 1753 -> 1449, block pass 1631 -> 1535 (profiles/r05_u64_isa.txt);
// C3 60-bit forward 2.04 -> 2.22 M NTT/s in one rocprof run (profiles/r05_u60_kernel_stats.txt).  Constants are not
// pinned to VGPRs here (ArithU64(c, false)): pinned, the column pass spilled at its 128-VGPR bound and fell back.
struct ArithU60 : ArithU64 {
    uint64_t n8q;
    uint32_t sh;   // canon's window: x >> sh < 2^32 for x < 16q (sh = max(0, bitlen(q) - 28))
    float qs;      // 2^sh / q (1 - 2^-20), canon's quotient scale

    __device__ __forceinline__ static uint32_t window(uint64_t q) {
        const int b = 64 - __clzll((long long)q);
        return b > 28 ? (uint32_t)(b - 28) : 0u;
    }
    __device__ __forceinline__ explicit ArithU60(const LimbConst& c)
        : ArithU64(c, false), n8q(0 - 8 * c.q), sh(window(c.q)),
          qs((float)(c.qinv * (double)(1ull << window(c.q)) * (1.0 - 0x1p-20))) {}
    __device__ __forceinline__ uint64_t mulmod(uint64_t v, Tw w) const {
        const uint64_t Q = mulhi64(v, w.y);
        const uint32_t vl = (uint32_t)v, vh = (uint32_t)(v >> 32), wl = (uint32_t)w.x, wh = (uint32_t)(w.x >> 32);
        const uint32_t Ql = (uint32_t)Q, Qh = (uint32_t)(Q >> 32), ml = (uint32_t)nq, mh = (uint32_t)(nq >> 32);
        // the two low products spelled out: left to itself the compiler folds cross products into extra
        // v_mad_u64_u32 + v_mov pairs
        uint64_t p, p2, c1, c2;
        asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(c1) : "v"(vl), "v"(wl));
        asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(p2), "=s"(c2) : "v"(Ql), "v"(ml), "v"(p));
        const uint32_t hi = (uint32_t)(p2 >> 32) + vl * wh + vh * wl + Ql * mh + Qh * ml;
        return ((uint64_t)hi << 32) | (uint32_t)p2;
    }
    __device__ __forceinline__ void ct(uint64_t& u, uint64_t& v, Tw w) const {
        const uint64_t t = mulmod(v, w), a = u;
        u = a + t;
        v = a - t + two_q;
    }
    __device__ __forceinline__ void ct_first(uint64_t& u, uint64_t& v, Tw w) const {
        u = sel_sub(u, u + n8q);
        ct(u, v, w);
    }
    __device__ __forceinline__ uint64_t round_reduce(uint64_t x) const { return x; }
    __device__ __forceinline__ uint64_t raw_out(uint64_t x) const { return x; }
    // [0, 16q) -> [0, q): the quotient k = floor(x / q) - {0, 1} from a 32-bit window of x in FP32, x - k q in
    // [0, 2q) by one mad, then one select: 11 VALU instructions instead of four selects' 20.  The window
    // xs = x >> sh with sh = max(0, bitlen(q) - 28) holds all of x's significant bits down to 2^-27 q
    // (x < 16q < 2^(bitlen(q) + 4)), so with b = bitlen(q):
    //   x/q - xs 2^sh / q < 2^sh / q <= 2^-27,  three FP32 roundings <= 3 * 2^-24 relative,
    // and the scale, shaded down by 2^-20 relative (> the roundings), keeps k <= floor(x / q) while the total
    // shortfall 16 (2^-20 + 3 * 2^-24) + 2^-27 < 2e-5 keeps k >= floor(x / q) - 1, for every q < 2^60.
    // (r05 took the window as the high word for every q; for q < 2^33 the dropped low word is worth >= 0.5 of a
    // quotient step and canon returned residues >= q: tests/test_modsize_sweep_gpu.py, tests/test_u60_canon_cpu.py.)
    __device__ __forceinline__ uint64_t canon(uint64_t x) const {
        float f;
        asm("v_cvt_f32_u32 %0, %1" : "=v"(f) : "v"((uint32_t)(x >> sh)));
        uint32_t k;
        asm("v_cvt_u32_f32 %0, %1" : "=v"(k) : "v"(f * qs));
        uint64_t r, c;
        asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(c) : "v"(k), "v"((uint32_t)nq), "v"(x));
        uint32_t kh;
        asm("v_mul_lo_u32 %0, %1, %2" : "=v"(kh) : "v"(k), "v"((uint32_t)(nq >> 32)));
        const uint32_t rh = (uint32_t)(r >> 32) + kh;
        r = ((uint64_t)rh << 32) | (uint32_t)r;
        return sel_sub(r, r + nq);
    }

    // ---- the inverse (r06): Gentleman-Sande with X left unreduced ----
    // An element of bound exponent B is < 2q 2^B.  GS on a pair of equal exponents B (always the case, U60InvBounds):
    // X = u + v has exponent B + 1; Y = Shoup((u + 2q 2^B) - v, w) is in [0, 2q) (exponent 0) for any input < 2^64,
    // and (u + 2q 2^B) - v < 2q 2^(B+2) < 2^64 while B <= 2 and q < 2^60.  An exponent-3 pair (16q) is reduced
    // first.  Harvey (ArithU64::gs) instead reduces X in every butterfly: 32 selects per 4-stage round of 16
    // registers against 18 here (6 mid-round + 12 at the round's end, U60InvBounds).
    template <int B>
    __device__ __forceinline__ uint64_t red(uint64_t x) const {   // exponent B -> 0: B selects by 2q 2^(B-1), .., 2q
        if constexpr (B > 0) return red<B - 1>(sel_sub(x, x + (n2q << (B - 1))));
        else return x;
    }
    // the inverse's outputs: its last stage leaves every value in [0, 2q) (X = Shoup((u + v), n^-1), Y Shoup too)
    __device__ __forceinline__ uint64_t canon_inv(uint64_t x) const { return sel_sub(x, x + nq); }
    template <int B>
    __device__ __forceinline__ void gs_b(uint64_t& u, uint64_t& v, Tw w) const {
        static_assert(B >= 0 && B <= 2, "GS input exponent");
        const uint64_t a = u, b = v;
        u = a + b;
        v = mulmod(a + (two_q << B) - b, w);
    }
};

template <class A>
constexpr bool kIsU64 = std::is_base_of<ArithU64, A>::value;   // the 64-bit integer policies (tables, LDS layouts)
template <class A>
constexpr bool kLazyU60 = std::is_same<A, ArithU60>::value;

// Bound exponents of the lazy U60 inverse (ArithU60::gs_b) over one round: R registers, executed stages bb = 0, 1, ..
// (stage bb pairs k, k + 2^bb; X -> k, Y -> k + 2^bb).  All exponents are 0 when a round starts.  The two elements of
// a pair have the same history (they differ only in bit bb, no earlier stage's bit), hence equal exponents.  An
// exponent-3 pair is reduced before its butterfly.  R = 16: exponents after 4 stages {1,3,2,2,1,1,1,1, 0 x 8}.
template <int R>
struct U60InvBounds {
    // exponent of element k after the first n executed stages of a round
    static constexpr int after(int k, int n) {
        int B[R] = {};
        for (int bb = 0; bb < n; ++bb) {
            const int h = 1 << bb;
            for (int j = 0; j < R; ++j) {
                if (j & h) continue;
                const int e = B[j] == 3 ? 0 : B[j];
                B[j] = e + 1;
                B[j + h] = 0;
            }
        }
        return B[k];
    }
};

}  // namespace mfhe
