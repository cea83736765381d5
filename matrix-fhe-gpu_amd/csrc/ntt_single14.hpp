// ntt_single14.hpp -- N = 2^14 (BASELINE C2) in one pass at 16N bytes per transform, with the next polynomial's
// loads in flight while the current one computes.  FP64 arithmetic (every q < 2^50).
//
// Why.  A 2^14 polynomial is 128 KiB: it fits one CU's LDS, so the whole transform can run in one pass (8N read +
// 8N write) instead of the two-pass plan's 32N.  The earlier single pass (NttPass, plan 1) measured no faster than
// two passes because each CU serialised load -> compute -> store: one 1024-thread workgroup per CU (139 KiB LDS),
// and `__syncthreads()` at every LDS exchange carries a vmcnt(0) that would wait for any prefetch, as do the
// per-butterfly twiddle loads from global memory (vmcnt is in order).
//
// Here nothing in a polynomial's compute touches vector memory, so the next polynomial's 16 loads per thread stay
// in flight through the whole transform and the current one's 16 stores drain behind the next compute:
//   * twiddles come from LDS: tw[0, 2048) of the limb (16 KiB, the direct table for stages 0..10) plus
//     tw[2048 i], i = 1..7; a stage-11..13 twiddle is the product tw[k] = tw[k & 2047] * tw[k & ~2047]
//     (tw[k] = psi^brev14(k) and brev is additive over disjoint bits), one exact FP64 modmul;
//   * barriers are `s_waitcnt lgkmcnt(0); s_barrier` (lds_barrier), never __syncthreads();
//   * the loads go into raw[16] right after raw was converted into x[16]: 32 + 32 VGPRs of data.
// LDS: 128 KiB of data (no padding: an XOR swizzle makes every exchange access conflict-free) + 16 KiB of table =
// 144 KiB, so one workgroup of 1024 threads (16 waves) per CU.
//
// Layouts (element index j = b13..b0; thread t: lane = t & 63, wave = t >> 6; register k = 4 bits):
//   L0: k -> b13..b10, t -> b9..b0                                 (global loads / stores: 512 B per wave access)
//   L1: k -> b9..b6, lane -> b5..b0, wave -> b13..b10
//   L2: k -> b5..b2, lane -> b1 b0 (lane bits 0, 1), b9..b6 (lane bits 2..5), wave -> b13..b10
//   L3: k -> b3..b0, lane bits 0..3 -> b8..b5, lane bit 4 -> b4, lane bit 5 -> b9, wave -> b13..b10
// Forward (CT, stage s pairs bit 13 - s): load L0, stages 0-3 | L1 4-7 | L2 8-10 (b2 rides along) | L3 11-13 | -> L1,
// store.  Inverse (GS): load L1 -> L3 stages 13-11 | L2 10-8 | L1 7-4 | L0 3-0 (n^-1 at s = 0), store.  Only L0 is
// cross-wave: one workgroup barrier per polynomial (after the cross-wave image is written; the wait before the
// polynomial's first LDS write is the drain counter, see below), the other exchanges are wave-local.
// Arithmetic and reduction schedule as in NttPass (ntt_arith.hpp): forward, one centred reduction at the start of
// every round after the first (rounds of <= 4 stages: |x| < 3q); inverse, lazy GS on every other stage.
// Reference: phantom fnwt_1d / inwt_1d per polynomial (ntt_core.cu:443-460); same outputs, bit for bit.
#pragma once
#include "ntt_coldb.hpp"

#ifndef MFHE_S14_CPOL_OUT
#define MFHE_S14_CPOL_OUT MFHE_NTT_CPOL_OUT   // output store policy (gfx950 CPol bits: 1 sc0, 2 nt, 16 sc1)
#endif
#ifndef MFHE_S14_LATE_CVT
#define MFHE_S14_LATE_CVT 1   // +1-2% (profiles/r04_c2_late_cvt_ab.txt)
#endif
#ifndef MFHE_S14_EXP
#define MFHE_S14_EXP 0   // timing probes (wrong results), never in the product build: 1 compute only, 2 exchanges +
                         // memory, 3 memory only, 4 no stores, 5 no loads after the first
#endif

namespace mfhe {

struct S14 {
    static constexpr int LOGN = 14, N = 1 << 14, NT = 1024, R = 16;
    static constexpr int TAB = 2048;   // direct twiddles per limb in LDS (stages 0..10)
    static constexpr size_t LDS_BYTES = (size_t)N * 8 + (size_t)(TAB + 8) * 8 + 16;   // + the drain counter
};

// LDS slot of element j.  h XORs b5, b6, b7, b8 into bits 0, 2, 3, {1, 4}: every exchange access (ds_write_b64:
// 16-lane groups must hit distinct slots mod 16; ds_read_b64: 32-lane groups, distinct mod 32) is conflict-free
// in all four layouts (checked by tests/test_ntt14_layout.py).
__device__ __host__ __forceinline__ constexpr uint32_t s14_swz(uint32_t j) {
    const uint32_t h = ((j >> 5) & 1u) | (((j >> 6) & 1u) << 2) | (((j >> 7) & 1u) << 3) | (((j >> 8) & 1u) * 18u);
    return j ^ h;
}

template <int LAY>
__device__ __host__ __forceinline__ constexpr uint32_t s14_j(uint32_t t, uint32_t k) {
    const uint32_t lane = t & 63u, wave = t >> 6;
    if constexpr (LAY == 0) return (k << 10) | t;
    else if constexpr (LAY == 1) return (wave << 10) | (k << 6) | lane;
    else if constexpr (LAY == 2) return (wave << 10) | ((lane >> 2) << 6) | (k << 2) | (lane & 3u);
    else return (wave << 10) | ((lane >> 5) << 9) | ((lane & 15u) << 5) | (((lane >> 4) & 1u) << 4) | k;
}
// j bit held by register bit 0 of each layout
template <int LAY>
constexpr int s14_kbase() { return LAY == 0 ? 10 : LAY == 1 ? 6 : LAY == 2 ? 2 : 0; }

// A thread index the compiler cannot see through: every address derived from it is computed where it is used.
// Without this, LICM hoists the ~130 loop-invariant LDS addresses of the four exchanges and the twiddle reads out
// of the polynomial loop and keeps them live (VGPRs 128 + 102 spilled).
__device__ __forceinline__ uint32_t s14_opaque(uint32_t t) {
    asm volatile("" : "+v"(t));
    return t;
}

// Exchange addressing.  j(t, k) = jt(t) | jk(k) with disjoint bits and the swizzle is XOR-linear, so
// swz(j) = S(t) ^ C(k), S(t) = swz(jt(t)), C(k) = swz(jk(k)) a compile-time constant.  The bits of C outside those S
// can occupy (TB: jt's bits and the swizzle's target bits 0..4) are added, which the ds_read / ds_write immediate
// offset absorbs; only C & TB needs a v_xor (none in L0, 7 distinct in L1, 15 in L2 and L3).  One S per access group
// instead of a full address computation per element (r04: ~500 -> ~110 VALU address instructions per polynomial).
template <int LAY>
__device__ __host__ constexpr uint32_t s14_tbits() {
    uint32_t m = 0x1Fu;
    for (uint32_t t = 0; t < 1024; ++t) m |= s14_j<LAY>(t, 0);
    return m;
}
// In bytes, on the LDS address space: S8 = lds + 8 S once per access group, then one v_xor per element (the buffer is
// 256-B aligned, so the XOR of bits 3..7 commutes with the base) and the added part in the instruction's offset.
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __forceinline__ uint32_t s14_lds_addr(const double* p) { return (uint32_t)(size_t)(const lds_f64*)p; }
template <int LAY, int K>
__device__ __forceinline__ lds_f64* s14_slot(uint32_t S8) {
    constexpr uint32_t c = s14_swz(s14_j<LAY>(0, (uint32_t)K)), tb = s14_tbits<LAY>();
    static_assert(((c & tb) << 3) < 256, "XOR part stays inside the buffer's 256-B alignment");
    return (lds_f64*)(size_t)((S8 ^ ((c & tb) << 3)) + ((c & ~tb) << 3));
}
template <int LAY>
__device__ __forceinline__ uint32_t s14_s8(const double* lds, uint32_t t_) {
    return s14_lds_addr(lds) + (s14_swz(s14_j<LAY>(s14_opaque(t_), 0)) << 3);
}
template <int LAY>
__device__ __forceinline__ void s14_write(const double (&x)[16], double* lds, uint32_t t) {
    const uint32_t S8 = s14_s8<LAY>(lds, t);
    static_for<0, 16>([&](auto kc) { *s14_slot<LAY, decltype(kc)::value>(S8) = x[decltype(kc)::value]; });
}
template <int LAY>
__device__ __forceinline__ void s14_read(double (&x)[16], double* lds, uint32_t t) {
    const uint32_t S8 = s14_s8<LAY>(lds, t);
    static_for<0, 16>([&](auto kc) { x[decltype(kc)::value] = *s14_slot<LAY, decltype(kc)::value>(S8); });
}

// Exchange FROM -> TO.  L1, L2 and L3 keep each wave on its own 1024-element block (j >> 10 = wave), so an exchange
// between two of them is wave-local: the wave reads only slots it wrote, LDS operations of one wave are performed in
// order -- a wait for this wave's own writes suffices, no s_barrier.  L0 spreads every thread over all 16 blocks:
// reading it needs every wave's writes (barrier after the writes).  BAR: a barrier before the writes, needed by the
// first exchange of a polynomial -- its writes land in blocks another wave may still be reading (the previous
// polynomial's last exchange); inside a polynomial only the wave itself touches its block between the cross-wave
// exchanges.
// Drain counter (r04): instead of a workgroup barrier before a polynomial's first LDS write, each wave adds 1 to an
// LDS counter after its last read of the previous polynomial's image (a wave's LDS operations are performed in order,
// so the add lands after those reads), and the first write waits until all 16 waves have added.  A barrier would also
// wait for everything the other waves issued after their reads -- the output stores (inverse) or a whole round of
// butterflies (forward).
// Both in inline asm: the compiler's lowering of an LDS atomic or a volatile LDS load also waits for vmcnt(0), i.e.
// for the next polynomial's loads in flight.
__device__ __forceinline__ void s14_drained(uint32_t* cnt) {
    const uint32_t a = (uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t*)cnt;
    if ((threadIdx.x & 63) == 0) asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(1u) : "memory");   // after this wave's reads
}
__device__ __forceinline__ void s14_wait_drained(const uint32_t* cnt, uint32_t target) {
    const uint32_t a = (uint32_t)(size_t)(const __attribute__((address_space(3))) uint32_t*)cnt;
    while (true) {
        uint32_t v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
        if (__builtin_amdgcn_readfirstlane(v) >= target) break;
        __builtin_amdgcn_s_sleep(1);
    }
}
template <int FROM, int TO, bool BAR>
__device__ __forceinline__ void s14_exchange(double (&x)[16], double* lds, uint32_t t, const uint32_t* cnt = nullptr,
                                             uint32_t target = 0) {
    if constexpr (BAR) s14_wait_drained(cnt, target);   // every wave is done reading the buffer's previous image
    s14_write<FROM>(x, lds, t);
    if constexpr (FROM == 0 || TO == 0) lds_barrier();
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    s14_read<TO>(x, lds, t);
}

// Twiddle of stage S for the butterfly group whose lower element is j = jt | JK (thread part, compile-time register
// part; disjoint bits): index 2^S + (j >> (14 - S)), from the LDS tables -- direct below 2048, else the product of
// tab[idx & 2047] and btab[idx >> 11] = tw[idx & ~2047].  The shifted parts stay disjoint, so the register part is an
// added constant (the ds_read offset) and the thread part one VGPR per stage.
template <int S, uint32_t JK>
__device__ __forceinline__ double s14_tw(const ArithF64& ar, const double* tab, const double* btab, uint32_t jt) {
    constexpr int sh = 14 - S;
    constexpr uint32_t ck = (1u << S) | (JK >> sh);
    const uint32_t vt = jt >> sh;
    if constexpr (S <= 10) return tab[vt + ck];
    else return ar.mulmod(tab[(vt & 2047u) + (ck & 2047u)], btab[(vt >> 11) + (ck >> 11)]);
}

// CT stages on register bits BB_HI .. BB_LO (descending) of layout LAY
template <int LAY, int BB_HI, int BB_LO>
__device__ __forceinline__ void s14_ct_round(double (&x)[16], const ArithF64& ar, const double* tab,
                                             const double* btab, uint32_t t_) {
    const uint32_t t = s14_opaque(t_);
    static_for<0, BB_HI - BB_LO + 1>([&](auto ic) {
        constexpr int bb = BB_HI - decltype(ic)::value;
        constexpr int b = s14_kbase<LAY>() + bb, s = 13 - b, half = 1 << bb;
        // one twiddle per group of butterflies sharing the register bits above bb
        double w[16 >> (bb + 1)];
        const uint32_t jt = s14_j<LAY>(t, 0);
        static_for<0, (16 >> (bb + 1))>([&](auto gc) {
            constexpr int g = decltype(gc)::value;
            w[g] = s14_tw<s, s14_j<LAY>(0, (uint32_t)(g << (bb + 1)))>(ar, tab, btab, jt);
        });
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k & half) continue;
            ar.ct(x[k], x[k + half], w[k >> (bb + 1)]);
        }
    });
}

// GS stages on register bits BB_LO .. BB_HI (ascending) of layout LAY; lazy on odd s, reducing on even s, and the
// s = 0 stage: X = (u + v) n^-1, Y = (u - v) itw[1] (itw[1] carries n^-1)
template <int LAY, int BB_LO, int BB_HI>
__device__ __forceinline__ void s14_gs_round(double (&x)[16], const ArithF64& ar, const double* tab,
                                             const double* btab, double w1, double ninv, uint32_t t_) {
    const uint32_t t = s14_opaque(t_);
    static_for<0, BB_HI - BB_LO + 1>([&](auto ic) {
        constexpr int bb = BB_LO + decltype(ic)::value;
        constexpr int b = s14_kbase<LAY>() + bb, s = 13 - b, half = 1 << bb;
        if constexpr (s == 0) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k & half) continue;
                double u = x[k], v = x[k + half];
                ar.gs_lazy(u, v, w1);
                x[k] = ar.mulmod(u, ninv);
                x[k + half] = v;
            }
        } else {
            double w[16 >> (bb + 1)];
            const uint32_t jt = s14_j<LAY>(t, 0);
            static_for<0, (16 >> (bb + 1))>([&](auto gc) {
                constexpr int g = decltype(gc)::value;
                w[g] = s14_tw<s, s14_j<LAY>(0, (uint32_t)(g << (bb + 1)))>(ar, tab, btab, jt);
            });
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                if (k & half) continue;
                if constexpr (s % 2 == 1) ar.gs_lazy(x[k], x[k + half], w[k >> (bb + 1)]);
                else ar.gs(x[k], x[k + half], w[k >> (bb + 1)]);
            }
        }
    });
}

template <bool INV>
__global__ __launch_bounds__(S14::NT, 1) void ntt14_kernel(PassArgs<TwSrcF> a) {
    extern __shared__ __attribute__((aligned(256))) uint64_t lds_raw[];   // 256: s14_slot's XOR
    double* lds = (double*)lds_raw;
    double* tab = lds + S14::N;          // [2048]: tw[0, 2048) of the limb (inverse: itw, entry 1 without n^-1)
    double* btab = tab + S14::TAB;       // [8]: tw[2048 i]
    uint32_t* drain = (uint32_t*)(btab + 8);   // waves done with the current polynomial's LDS image (s14_drained)
    const uint32_t t = threadIdx.x;
    const uint32_t nb = a.nblocks;       // polynomials (batch * nl)
    uint32_t lt = blockIdx.x;
    if (lt >= nb) return;
    const uint32_t bt = (uint32_t)a.batch;
    auto poly = [&](uint32_t l, int* mod) {
        const uint32_t v = xcd_remap(l, nb);   // limb-major: v = limb * batch + b
        const uint32_t li = v / bt, b = v - li * bt;
        *mod = a.start_limb + (int)li;
        const uint64_t* p = a.data + (((uint64_t)b * (uint64_t)a.nl + li) << S14::LOGN);
        // workgroup-uniform: say so, so the accesses are SGPR base + lane offset
        const uint64_t pu = (uint64_t)p;
        return (uint64_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(pu >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)pu));
    };
    // global layouts: the forward loads L0 (its first round pairs b13..b10) and stores L1, the inverse loads L1 and
    // stores L0; in both, each register's 64 lanes cover 512 contiguous bytes
    constexpr int LIN = INV ? 1 : 0, LOUT = INV ? 0 : 1;
    auto load = [&](const uint64_t* base, uint64_t (&raw)[16]) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 0x7FFFFFFF, 0x00020000);
        const int vo = (int)(s14_j<LIN>(t, 0) * 8u);   // thread part in the VGPR offset, register part in soffset
#pragma unroll
        for (int k = 0; k < 16; ++k)
            raw[k] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                                      rs, vo, (int)(s14_j<LIN>(0, (uint32_t)k) * 8u), 0));
    };
    int mod = 0, tmod = -1;
    uint32_t done = 0;   // polynomials this workgroup has finished: the drain counter's target is 16 done
    if (t == 0) *drain = 0u;   // published by the first limb's table barriers below
    uint64_t* base = poly(lt, &mod);
    uint64_t raw[16];
    load(base, raw);
    // the polynomial's words are converted at the END of the previous iteration, after its stores: the loop then
    // carries the converted doubles, so the compiler's loop-carried register copies no longer wait (vmcnt) for the
    // prefetch in the middle of the store sequence (r04, MFHE_S14_LATE_CVT)
    double x[16];
    if constexpr (MFHE_S14_LATE_CVT) {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = ArithF64::from_u64(raw[k]);
    }
    ArithF64 ar(LimbConst{});
    double w1 = 0.0, ninv = 0.0;
    while (true) {
        const uint32_t nlt = lt + gridDim.x;
        const bool more = nlt < nb;   // workgroup-uniform
        if (mod != tmod) {
            // the limb's constants by scalar loads; its twiddle table into LDS (a vector load + wait, once per limb)
            tmod = mod;
            const __attribute__((address_space(4))) LimbConst* cl =
                (const __attribute__((address_space(4))) LimbConst*)a.limbs + mod;
            LimbConst lc;
            lc.q = cl->q;
            lc.qf = cl->qf;
            lc.qinv = cl->qinv;
            ar = ArithF64(lc);
            typedef const __attribute__((address_space(4))) double* cd_t;
            const double* tw = a.tw.p + ((size_t)mod << S14::LOGN);
            if constexpr (INV) {
                w1 = ((cd_t)tw)[1];
                ninv = ((cd_t)a.ninv.p)[mod];
            }
            lds_barrier();   // every thread is done with the previous limb's table
            const double2 v = ((const double2*)tw)[t];   // tw[2t], tw[2t + 1]
            ((double2*)tab)[t] = v;
            if (t < 8) btab[t] = t ? tw[t << 11] : 1.0;
            if constexpr (INV) {
                // itw[1] carries n^-1 (ctx.cpp build_ct_tables): the table needs the plain power psi^-brev(1)
                if (t == 0) tab[1] = ar.reduce(ar.mulmod(v.y, (double)S14::N));
            }
            lds_barrier();
        }
        if constexpr (!MFHE_S14_LATE_CVT) {
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = ArithF64::from_u64(raw[k]);
        }
        uint64_t* nbase = base;
        int nmod = mod;
        if (more) {
            nbase = poly(nlt, &nmod);
#if MFHE_S14_EXP != 1 && MFHE_S14_EXP != 5
            load(nbase, raw);   // in flight through the whole transform below
#endif
        }
#if MFHE_S14_EXP == 2 || MFHE_S14_EXP == 3   // timing probes only (wrong results): 2 = no butterflies, 3 = no butterflies, no exchanges
        if (true) {
#if MFHE_S14_EXP == 2
            if constexpr (!INV) {
                s14_exchange<0, 1, true>(x, lds, t, drain, 16u * done);
                s14_exchange<1, 2, false>(x, lds, t);
                s14_exchange<2, 3, false>(x, lds, t);
                s14_exchange<3, 1, false>(x, lds, t);
            } else {
                s14_exchange<1, 3, true>(x, lds, t, drain, 16u * done);
                s14_exchange<3, 2, false>(x, lds, t);
                s14_exchange<2, 1, false>(x, lds, t);
                s14_exchange<1, 0, false>(x, lds, t);
            }
            s14_drained(drain);
#endif
        } else
#endif
        if constexpr (!INV) {
            s14_ct_round<0, 3, 0>(x, ar, tab, btab, t);
            s14_exchange<0, 1, true>(x, lds, t, drain, 16u * done);
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = ar.round_reduce(x[k]);
            s14_ct_round<1, 3, 0>(x, ar, tab, btab, t);
            s14_exchange<1, 2, false>(x, lds, t);
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = ar.round_reduce(x[k]);
            s14_ct_round<2, 3, 1>(x, ar, tab, btab, t);
            s14_exchange<2, 3, false>(x, lds, t);
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = ar.round_reduce(x[k]);
            s14_ct_round<3, 2, 0>(x, ar, tab, btab, t);
            s14_exchange<3, 1, false>(x, lds, t);   // wave-local: each wave stores its block when it is done
            s14_drained(drain);
        } else {
            s14_exchange<1, 3, true>(x, lds, t, drain, 16u * done);
            s14_gs_round<3, 0, 2>(x, ar, tab, btab, w1, ninv, t);
            s14_exchange<3, 2, false>(x, lds, t);
            s14_gs_round<2, 1, 3>(x, ar, tab, btab, w1, ninv, t);
            s14_exchange<2, 1, false>(x, lds, t);
            s14_gs_round<1, 0, 3>(x, ar, tab, btab, w1, ninv, t);
            s14_exchange<1, 0, false>(x, lds, t);
            s14_drained(drain);
            s14_gs_round<0, 0, 3>(x, ar, tab, btab, w1, ninv, t);
        }
        ++done;
#if MFHE_S14_EXP == 1 || MFHE_S14_EXP == 4   // timing probes only: no stores
        if (lt == 0xFFFFFFFFu)
#endif
        {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFFF, 0x00020000);
            const int vo = (int)(s14_j<LOUT>(s14_opaque(t), 0) * 8u);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                __builtin_amdgcn_raw_buffer_store_b64(
                    __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, ar.canon(x[k])), rs, vo,
                    (int)(s14_j<LOUT>(0, (uint32_t)k) * 8u), MFHE_S14_CPOL_OUT);
        }
        if (!more) break;
        if constexpr (MFHE_S14_LATE_CVT) {
#pragma unroll
            for (int k = 0; k < 16; ++k) x[k] = ArithF64::from_u64(raw[k]);
        }
        lt = nlt;
        base = nbase;
        mod = nmod;
    }
}

}  // namespace mfhe
