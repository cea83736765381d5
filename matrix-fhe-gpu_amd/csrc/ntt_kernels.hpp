// ntt_kernels.hpp -- batched NTT pass kernels for gfx950 (CDNA4).
//
// Transform: the phantom-fhe negacyclic NTT (SEAL convention) restated in
// SURVEY.md Appendix A -- Cooley-Tukey forward with tw[m+i] = psi^brev(m+i),
// bit-reversed output; Gentleman-Sande inverse with itw[m+i] = psi^-brev(m+i),
// n^-1 folded into the last stage.  Reference call sites: ntt_core.cu:443-460
// (xy_ntt_forward/backward_phantom -> fnwt_1d/inwt_1d).
//
// Decomposition.  Stage s (0..logN-1) pairs elements j, j + N/2^(s+1).  A
// *pass* runs stages [s0, s0+LOG_G) on independent *groups* of G = 2^LOG_G
// elements: for fixed (hi, lo) the group is j = hi<<(logN-s0) | g<<logS | lo,
// g in [0,G), S = 2^logS = N / 2^(s0+LOG_G).  Inside a pass each thread holds
// R = 2^LOG_R elements in registers and runs up to LOG_R stages per *round*;
// rounds exchange data through padded LDS.  N <= 2^14 runs as one pass (whole
// polynomial per workgroup); N = 2^15..2^17 as two passes (column pass with
// coalesced strided groups, then contiguous-block pass).
//
// Lane maps.  COLS (strided groups, S >= NG): lane -> group first, so every
// wave instruction touches NG consecutive columns; any g-layout is coalesced.
// Block mode (contiguous groups): lane -> tau first; only the round-0 layout
// (g = tau + TG*k) is coalesced, so loads/stores go through that layout.
//
// Workgroup -> data mapping is XCD aware: hardware deals blocks round-robin
// over the 8 XCDs, we remap so each XCD walks a contiguous range of a
// limb-major ordering, keeping one limb's twiddle table hot in that XCD's L2.
#pragma once
#include <type_traits>

#include "ntt_arith.hpp"

#ifndef MFHE_NTT_CPOL_IN
#define MFHE_NTT_CPOL_IN 0
#endif
#ifndef MFHE_NTT_CPOL_OUT
#define MFHE_NTT_CPOL_OUT 18   // sc1 nt: final outputs leave the L2 at once (+2-3% two-pass, profiles/r02_cpol.txt)
#endif
#ifndef MFHE_NTT_CPOL_MID_LD
#define MFHE_NTT_CPOL_MID_LD 0
#endif
#ifndef MFHE_NTT_CPOL_MID_ST
#define MFHE_NTT_CPOL_MID_ST 0
#endif
#ifndef MFHE_NTT_U64_INV_TWPRE
#define MFHE_NTT_U64_INV_TWPRE 1   // +4% U64 inverse (profiles/r04_u64_block_variants.txt)
#endif
#ifndef MFHE_NTT_COL_DMA
#define MFHE_NTT_COL_DMA 1   // forward column pass: tile -> LDS by LDS-DMA (16 B per lane), no VGPR staging
#endif

namespace mfhe {

struct TwSrcF {
    const double* p;
    __device__ __forceinline__ double get(size_t i) const { return p[i]; }
};
struct TwSrcU {
    const uint64_t* w;
    const uint64_t* ws;
    __device__ __forceinline__ ulonglong2 get(size_t i) const {
#ifdef MFHE_EXP_TWCONST   // timing probe only (wrong results): twiddles computed from the index, no loads
        return make_ulonglong2((uint64_t)i * 0x9E3779B97F4A7C15ull >> 6, (uint64_t)i * 0xC2B2AE3D27D4EB4Full);
#endif
        return make_ulonglong2(w[i], ws[i]);
    }
};

template <class TS>
struct PassArgs {
    uint64_t* data;          // [batch][nl][N]
    TS tw;                   // [mod][N]  (forward or inverse table)
    TS twist;                // [mod][N]  pre-twist (fwd) / post-twist (inv), TWIST only
    TS ninv;                 // [mod]     inverse last-stage X scale (n^-1)
    const LimbConst* limbs;  // [mod]; null -> q read from qraw[mod * qstride] (phantom DModulus)
    const uint64_t* qraw;
    int qstride;
    uint64_t batch;
    int nl, start_limb;
    int logN, s0;
    uint32_t nblocks;
};

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
    const uint32_t q = nb >> 3, r = nb & 7, x = b & 7, s = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
}

template <int LOG_G, int LOG_R>
struct Geo {
    static constexpr int G = 1 << LOG_G;
    static constexpr int R = 1 << LOG_R;
    static constexpr int TG = G / R;
    static constexpr int NR = (LOG_G + LOG_R - 1) / LOG_R;
    static constexpr int GS = G + G / 16 + 1;   // odd padded group stride (doubles)
    __host__ __device__ static constexpr int HB(int r) { return LOG_G - 1 - r * LOG_R; }
    __host__ __device__ static constexpr int WL(int r) { return (HB(r) - LOG_R + 1) > 0 ? (HB(r) - LOG_R + 1) : 0; }
    __device__ __forceinline__ static uint32_t g_of(int r, uint32_t tau, uint32_t k) {
        const int wl = WL(r);
        return ((tau >> wl) << (wl + LOG_R)) | (k << wl) | (tau & ((1u << wl) - 1));
    }
    __device__ __forceinline__ static uint32_t pad(uint32_t g) { return g + (g >> 4); }
};

__device__ __forceinline__ uint32_t brev_bits(uint32_t x, int bits) { return __brev(x) >> (32 - bits); }

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// One lazy U60 inverse butterfly stage on registers x[0..R): executed stage bb of its round, twiddle of pair k from
// tw(k), X scaled by wn instead when LAST (the s = 0 stage: X = (u + v) n^-1 in [0, 2q), Y = (u - v) itw[1]).
template <int R, int BB, bool LAST, class A, class T, class TWF>
__device__ __forceinline__ void u60_inv_stage(const A& ar, T (&x)[R], TWF&& tw, typename A::Tw wn) {
    constexpr int half = 1 << BB;
    static_for<0, R>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if constexpr (!(k & half)) {
            constexpr int e0 = U60InvBounds<R>::after(k, BB);
            constexpr int e = e0 == 3 ? 0 : e0;
            if constexpr (e0 == 3) {
                x[k] = ar.template red<3>(x[k]);
                x[k + half] = ar.template red<3>(x[k + half]);
            }
            const auto w = tw(k);
            ar.template gs_b<e>(x[k], x[k + half], w);
            if constexpr (LAST) x[k] = ar.mulmod(x[k], wn);
        }
    });
}

// canonical output of an inverse pass that ran the transform's last stage (s = 0): < 2q under the lazy U60 inverse
template <class A>
__device__ __forceinline__ uint64_t inv_out(const A& ar, typename A::T x) {
    if constexpr (kLazyU60<A>) return ar.canon_inv(x);
    else return ar.canon(x);
}

// the end of a lazy U60 inverse round of n executed stages: every element back to exponent 0 (< 2q)
template <int R, int N, class A, class T>
__device__ __forceinline__ void u60_inv_round_end(const A& ar, T (&x)[R]) {
    static_for<0, R>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        x[k] = ar.template red<U60InvBounds<R>::after(k, N)>(x[k]);
    });
}

// Where one tile (NG groups) of a pass lives: limb/batch, base pointer, twiddle offset, (hi, lo).
// UNI: every group of the tile lies in one polynomial (two-pass plans; single pass with NG = 1), so the
// base pointer is workgroup-uniform and each element address is an SGPR base + 32-bit lane offset.
struct TileLoc {
    uint64_t* base;
    size_t twoff;
    uint32_t off0;    // jhi | lo  (element offset inside the polynomial, without the group index)
    uint64_t hi;
    int mod;
    bool active;
};

template <int LOG_G, int NG, bool COLS, bool UNI>
__device__ __forceinline__ TileLoc tile_loc(uint64_t* data, uint64_t batch, int nl, int start_limb, int logN, int s0,
                                            uint32_t lb, uint32_t gl) {
    const int logS = logN - s0 - LOG_G;
    const int log_gpp = logS + s0;  // log2(groups per polynomial-limb)
    const uint32_t npl = (uint32_t)(batch * (uint64_t)nl);   // launcher guarantees < 2^32
    uint32_t v;
    uint64_t hi, lo;
    if constexpr (COLS) {
        // tiles of NG consecutive columns; tiles per poly = 2^log_gpp / NG
        constexpr int LOG_NG = __builtin_ctz(NG);
        const int log_tpp = log_gpp - LOG_NG, log_ct = logS - LOG_NG;
        v = lb >> log_tpp;
        const uint32_t tile = lb & ((1u << log_tpp) - 1);
        hi = tile >> log_ct;
        lo = ((uint64_t)(tile & ((1u << log_ct) - 1)) << LOG_NG) + gl;
    } else if constexpr (UNI) {
        const uint64_t g0 = (uint64_t)lb * NG;   // NG divides groups-per-poly: v is workgroup-uniform
        v = (uint32_t)(g0 >> log_gpp);
        const uint64_t rem = (g0 & ((1ull << log_gpp) - 1)) + gl;
        hi = rem >> logS;
        lo = rem & ((1ull << logS) - 1);
    } else {
        const uint64_t gid = (uint64_t)lb * NG + gl;
        v = (uint32_t)(gid >> log_gpp);
        const uint64_t rem = gid & ((1ull << log_gpp) - 1);
        hi = rem >> logS;
        lo = rem & ((1ull << logS) - 1);
    }
    TileLoc t;
    t.active = v < npl;
    if (!t.active) v = 0;   // inactive tail lanes read a valid polynomial and store nothing
    // virtual poly index is limb-major: v = l * batch + b
    const uint32_t bt = (uint32_t)batch;
    const int l = (int)(v / bt);
    const uint64_t b = v - (uint32_t)l * bt;
    t.mod = start_limb + l;
    t.base = data + ((b * (uint64_t)nl + (uint64_t)l) << logN);
    t.twoff = (size_t)t.mod << logN;
    t.hi = hi;
    t.off0 = (uint32_t)((hi << (logN - s0)) | lo);
    return t;
}

// One pass of the transform: LOG_G stages on groups of G = 2^LOG_G elements, one tile (NG groups) per
// workgroup at a time.  Split into locate / load / compute+store so the persistent pass kernel can
// prefetch.
// PACK (N = 2^16 two-pass plan, FP64 arithmetic, forward): the intermediate between the passes is stored as
// 50-bit canonical residues instead of 64-bit words.  Unit (rb, t) = the 16 x 16 block of rows 16 rb.. and
// columns 16 t.., column-major: LO[c][i] u32 (1024 B), MID[c][i] u16 (512 B), TOP[c] 16 x 2 bits (64 B),
// padded to 13 cache lines (1664 B).  Unit (rb, t) lives in rows 16 rb .. 16 rb + 12 of column tile t: lines
// the column pass of tile t read itself (it stages its 16 units in LDS and writes them, full lines only), and
// that only the block pass of row block rb reads and then overwrites with its outputs, so no workgroup's
// unread input is overwritten in either pass.  The block pass reads its 16 units with whole-line loads into
// LDS, takes unit column (t, c) per thread from there and exchanges into its round-0 layout.  Intermediate traffic: 208 instead of 256 lines each way
// (r02: the passes are fabric-bound, 25% fewer intermediate lines measured +11%, profiles/r02_pack.txt).
constexpr int kPackUnitBytes = 1664;   // 13 lines
constexpr int kPackRowBytes = 2048;    // one row of the 256 x 256 view of an N = 2^16 polynomial

template <class A, class TS, int LOG_G, int LOG_R, int NG, bool COLS, bool INV, bool IN_RAW, bool OUT_RAW,
          bool TWIST, bool BREV, bool UNI, bool PACK = false>
struct NttPass {
    static_assert(!PACK || (LOG_G == 8 && LOG_R == 4 && NG == 16 && UNI && !INV && !TWIST && !BREV &&
                            (COLS ? (OUT_RAW && !IN_RAW) : (IN_RAW && !OUT_RAW))),
                  "PACK: forward N = 2^16 two-pass plan only");
    // forward column pass reading the transform input: the 32 KiB tile goes global -> LDS by LDS-DMA
    // (global_load_lds_dwordx4: 16 B per lane, each wave instruction 1 KiB), then round 0 reads it from LDS
    static constexpr bool COL_DMA = MFHE_NTT_COL_DMA && COLS && !INV && !IN_RAW && UNI && !TWIST &&
                                    (1 << LOG_G) * NG * 8 == 32768 && NG % 2 == 0;
    static constexpr bool PACK_OUT = PACK && COLS;   // column pass writes packed units
    static constexpr bool PACK_IN = PACK && !COLS;   // block pass reads them
    using Gm = Geo<LOG_G, LOG_R>;
    using T = typename A::T;
    using Tw = typename A::Tw;
    static constexpr int R = Gm::R, TG = Gm::TG, NR = Gm::NR, GS = Gm::GS;
    static constexpr int NT = NG * TG;
    static constexpr size_t LDS_BYTES = (NR > 1 || BREV) ? (size_t)NG * GS * sizeof(uint64_t) : 0;
    static constexpr int r_load = (INV && COLS) ? (NR - 1) : 0;
    static constexpr int r_store = (!INV && COLS) ? (NR - 1) : 0;

    const PassArgs<TS>& a;
    uint32_t gl, tau;
    int s0, logS;   // a column pass is always the first LOG_G stages, a block pass the last LOG_G

    __device__ __forceinline__ explicit NttPass(const PassArgs<TS>& args) : a(args) {
        const uint32_t t = threadIdx.x;
        gl = COLS ? (t % NG) : (t / TG);
        tau = COLS ? (t / NG) : (t % TG);
        s0 = COLS ? 0 : a.logN - LOG_G;
        logS = a.logN - s0 - LOG_G;
    }
    __device__ __forceinline__ uint32_t jidx(const TileLoc& L, uint32_t g) const { return L.off0 | (g << logS); }
    __device__ __forceinline__ TileLoc locate(uint32_t lb) const {
        return tile_loc<LOG_G, NG, COLS, UNI>(a.data, a.batch, a.nl, a.start_limb, a.logN, s0, lb, gl);
    }
    // cache policy (gfx950 CPol bits: 1 sc0, 2 nt, 16 sc1) of the global loads / stores of a pass:
    // input of a transform, intermediate between the passes, output of a transform
    static constexpr int kCpolLd = IN_RAW ? MFHE_NTT_CPOL_MID_LD : MFHE_NTT_CPOL_IN;
    static constexpr int kCpolSt = OUT_RAW ? MFHE_NTT_CPOL_MID_ST : MFHE_NTT_CPOL_OUT;

    __device__ __forceinline__ void load(const TileLoc& L, uint64_t (&raw)[R]) const {
        if constexpr (COL_DMA) return;   // compute_store issues the DMA once the LDS is free
        if constexpr (PACK_IN) {
            // the 16 units of this row block, 16 B chunks q = tid + NT s (1664 of them): every wave instruction
            // reads 8 whole lines; compute_store sorts them out through LDS
            const uint32_t rb = (uint32_t)(L.hi >> 4);
            const char* base = (const char*)L.base + (size_t)(16 * rb) * kPackRowBytes;
#pragma unroll
            for (int s = 0; s < 7; ++s) {
                const uint32_t q = threadIdx.x + NT * s;
                ulonglong2 v = make_ulonglong2(0, 0);
                if (s < 6 || q < 16 * kPackUnitBytes / 16) {
                    const uint32_t t = q / 104, w = q - 104 * t;   // unit, chunk in the unit (8 per line)
                    v = *(const ulonglong2*)(base + (w >> 3) * kPackRowBytes + t * 128 + (w & 7) * 16);
                }
                raw[2 * s] = v.x;
                raw[2 * s + 1] = v.y;
            }
            return;
        }
        if constexpr (UNI && kCpolLd != 0) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(L.base, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
            for (int k = 0; k < R; ++k)
                raw[k] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                                          rs, (int)(jidx(L, Gm::g_of(r_load, tau, k)) * 8u), 0, kCpolLd));
        } else {
#pragma unroll
            for (int k = 0; k < R; ++k) {
#ifdef MFHE_EXP_SKIP
                if (IN_RAW && k >= 12) { raw[k] = 0; continue; }   // traffic experiment only (wrong results)
#endif
                raw[k] = L.base[jidx(L, Gm::g_of(r_load, tau, k))];
            }
        }
    }

    __device__ __forceinline__ void compute_store(const TileLoc& L, const uint64_t (&raw)[R], uint64_t* lds) const {
        uint64_t* my_lds = lds + (size_t)gl * GS;
        LimbConst lc;
        if (a.limbs) {
            lc = a.limbs[L.mod];
        } else {
            lc.q = a.qraw[(size_t)L.mod * a.qstride];
            lc.qf = (double)lc.q;
            lc.qinv = 1.0 / lc.qf;
        }
        const A ar(lc);
        const size_t twoff = L.twoff;
        const uint32_t tau_ = tau;

        T x[R];
        if constexpr (COL_DMA) {
            typedef __attribute__((address_space(3))) void* lds_vp;
            constexpr int CPR = NG / 2;                      // 16-B chunks per row of the tile
            const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
            const char* tile = (const char*)(L.base + (L.off0 - gl));   // row 0, first column of the tile
            __syncthreads();   // the previous tile's readers of this LDS are done
#pragma unroll
            for (int i = 0; i < 32768 / (NT * 16); ++i) {
                const uint32_t q = (i * (NT / 64) + w) * 64 + lane;   // chunk: row q / CPR, part q % CPR
                const char* src = tile + (size_t)(q / CPR) * ((size_t)8 << (a.logN - LOG_G)) + (q % CPR) * 16;
                __builtin_amdgcn_global_load_lds((const void*)src,
                                                 (lds_vp)((char*)lds + (size_t)(i * (NT / 64) + w) * 1024), 16, 0,
                                                 kCpolLd);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
#pragma unroll
            for (int k = 0; k < R; ++k) x[k] = A::from_u64(lds[(size_t)Gm::g_of(r_load, tau_, k) * NG + gl]);
        } else if constexpr (PACK_IN) {
            // staging image of the 16 units -> this thread's unit column (t, c) = rows 16 rb + i of column 16 t + c
            __syncthreads();   // the previous tile's readers of this LDS are done
            ulonglong2* img = (ulonglong2*)lds;
#pragma unroll
            for (int s = 0; s < 7; ++s) {
                const uint32_t q = threadIdx.x + NT * s;
                if (s < 6 || q < 16 * kPackUnitBytes / 16) img[q] = make_ulonglong2(raw[2 * s], raw[2 * s + 1]);
            }
            __syncthreads();
            const uint32_t C = threadIdx.x, t = C >> 4, c = C & 15;
            const char* ub = (const char*)lds + t * kPackUnitBytes;
            uint64_t w[13];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const ulonglong2 v = *(const ulonglong2*)(ub + c * 64 + 16 * s);
                w[2 * s] = v.x;
                w[2 * s + 1] = v.y;
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const ulonglong2 v = *(const ulonglong2*)(ub + 1024 + c * 32 + 16 * s);
                w[8 + 2 * s] = v.x;
                w[9 + 2 * s] = v.y;
            }
            w[12] = *(const uint32_t*)(ub + 1536 + c * 4);
            __syncthreads();   // staging image consumed: the exchange may overwrite it
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint64_t lo = (w[i >> 1] >> (32 * (i & 1))) & 0xFFFFFFFFull;
                const uint64_t mid = (w[8 + (i >> 2)] >> (16 * (i & 3))) & 0xFFFFull;
                const uint64_t top = (w[12] >> (2 * i)) & 3ull;
                lds[(size_t)i * GS + Gm::pad(C)] = lo | (mid << 32) | (top << 48);
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < R; ++k) x[k] = A::from_u64(my_lds[Gm::pad(Gm::g_of(0, tau_, k))]);
        } else {
#pragma unroll
            for (int k = 0; k < R; ++k) {
                x[k] = IN_RAW ? A::from_raw(raw[k]) : A::from_u64(raw[k]);
                if constexpr (TWIST && !INV) x[k] = ar.mulmod(x[k], a.twist.get(twoff + jidx(L, Gm::g_of(r_load, tau_, k))));
            }
        }

        auto exchange = [&](auto rf, auto rt, bool brev_pos) {
            constexpr int r_from = decltype(rf)::value, r_to = decltype(rt)::value;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < R; ++k) {
                uint32_t g = Gm::g_of(r_from, tau_, k);
                if (brev_pos) g = brev_bits(g, LOG_G);
                my_lds[Gm::pad(g)] = A::to_raw(x[k]);
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < R; ++k) x[k] = A::from_raw(my_lds[Gm::pad(Gm::g_of(r_to, tau_, k))]);
        };

        // U64 inverse block pass (MFHE_NTT_U64_INV_TWPRE, default on): the first executed stage's (w, w') pairs are loaded
        // before the entry exchange, so their latency overlaps it instead of following it (profiles/
        // r04_u64_twiddle_probe.txt: the inverse's first pass waits on these loads, the forward's passes do not)
        constexpr bool kTwPre = INV && !COLS && kIsU64<A> && MFHE_NTT_U64_INV_TWPRE;
        Tw wpre[kTwPre ? R / 2 : 1];
        if constexpr (kTwPre) {
            constexpr int r = NR - 1, wl = Gm::WL(r), bit = wl;   // bb = 0
            const int s = s0 + (LOG_G - 1 - bit);
            const uint64_t twb = twoff + (1ull << s) + (L.hi << (LOG_G - 1 - bit)) + ((uint64_t)(tau_ >> wl) << (LOG_R - 1));
#pragma unroll
            for (int m = 0; m < R / 2; ++m) wpre[m] = a.tw.get(twb + (uint64_t)m);
        }
        if constexpr (INV && !COLS && (NR > 1 || BREV))
            exchange(std::integral_constant<int, 0>{}, std::integral_constant<int, NR - 1>{}, BREV);

        // ---- one stage on register bit bb of round r ----
        auto stage = [&](auto rc, auto bc) {
            constexpr int r = decltype(rc)::value, bb = decltype(bc)::value;
            constexpr int hb = Gm::HB(r), wl = Gm::WL(r);
            constexpr int bit = wl + bb;
            if constexpr (bit <= hb) {
                const int s = s0 + (LOG_G - 1 - bit);
                constexpr int half = 1 << bb;
                const uint64_t tau_hi = tau_ >> wl;
                const uint64_t twb =
                    twoff + (1ull << s) + (L.hi << (LOG_G - 1 - bit)) + (tau_hi << (LOG_R - 1 - bb));
                if constexpr (!INV) {
                    // first executed stage of the round: the lazy U60 policy reduces its u inputs there (a pass's
                    // first round needs it only when the input is a raw intermediate)
                    constexpr int fb = (LOG_R - 1 < hb - wl) ? LOG_R - 1 : hb - wl;
                    constexpr bool first = bb == fb && (r > 0 || IN_RAW);
                    static_assert(!kLazyU60<A> || LOG_R <= 4, "U60 bound: at most 4 stages between reductions");
#pragma unroll
                    for (int k = 0; k < R; ++k) {
                        if (k & half) continue;
                        const Tw w = a.tw.get(twb + (uint64_t)(k >> (bb + 1)));
                        if constexpr (first) ar.ct_first(x[k], x[k + half], w);
                        else ar.ct(x[k], x[k + half], w);
                    }
                } else {
                    // executed-stage index inside this pass (inverse rounds run r = NR-1 .. 0; only the first
                    // round can skip stages, at its top bits): even -> lazy GS, odd -> reducing GS
                    constexpr int ri = NR - 1 - r;
                    constexpr int first = (Gm::HB(NR - 1) < LOG_R - 1 ? Gm::HB(NR - 1) : LOG_R - 1) + 1;
                    constexpr int e = ri == 0 ? bb : first + (ri - 1) * LOG_R + bb;
                    if constexpr (kLazyU60<A>) {
                        // lazy U60 inverse: X unreduced, per-register bound exponents (U60InvBounds; bb is the
                        // executed-stage index of this round: a round's executed stages are bb = 0, 1, ..)
                        if (s == 0) {
                            const Tw wn = a.ninv.get((size_t)L.mod);
                            const Tw w1 = a.tw.get(twoff + 1);
                            u60_inv_stage<R, bb, true>(ar, x, [&](int) { return w1; }, wn);
                        } else {
                            u60_inv_stage<R, bb, false>(ar, x, [&](int k) {
                                if constexpr (kTwPre && r == NR - 1 && bb == 0) return wpre[k >> 1];
                                else return a.tw.get(twb + (uint64_t)(k >> (bb + 1)));
                            }, Tw{});
                        }
                    } else if (s == 0) {
                        const Tw wn = a.ninv.get((size_t)L.mod);
                        const Tw w1 = a.tw.get(twoff + 1);
#pragma unroll
                        for (int k = 0; k < R; ++k) {
                            if (k & half) continue;
                            T u = x[k], vv = x[k + half];
                            ar.gs_lazy(u, vv, w1);     // u = u+v, vv = (u-v) * itw[1]
                            x[k] = ar.mulmod(u, wn);   // X * n^-1
                            x[k + half] = vv;
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < R; ++k) {
                            if (k & half) continue;
                            Tw w;
                            if constexpr (kTwPre && r == NR - 1 && bb == 0) w = wpre[k >> 1];
                            else w = a.tw.get(twb + (uint64_t)(k >> (bb + 1)));
                            if constexpr (e % 2 == 0) ar.gs_lazy(x[k], x[k + half], w);
                            else ar.gs(x[k], x[k + half], w);
                        }
                    }
                }
            }
        };

        if constexpr (!INV) {
            static_for<0, NR>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                if constexpr (r > 0) {
                    exchange(std::integral_constant<int, r - 1>{}, rc, false);
#pragma unroll
                    for (int k = 0; k < R; ++k) x[k] = ar.round_reduce(x[k]);
                }
                static_for<0, LOG_R>([&](auto bi) {
                    stage(rc, std::integral_constant<int, LOG_R - 1 - decltype(bi)::value>{});
                });
            });
        } else {
            static_for<0, NR>([&](auto ri) {
                constexpr int r = NR - 1 - decltype(ri)::value;
                if constexpr (r < NR - 1)
                    exchange(std::integral_constant<int, r + 1>{}, std::integral_constant<int, r>{}, false);
                static_for<0, LOG_R>([&](auto bi) { stage(std::integral_constant<int, r>{}, bi); });
                if constexpr (kLazyU60<A>) {
                    // back to < 2q before an exchange or a raw intermediate store (the next round / pass starts
                    // at exponent 0); a canonical store takes up to 16q (ArithU60::canon) as it is
                    constexpr int hb = Gm::HB(r), wl = Gm::WL(r);
                    constexpr int nexec = (hb - wl + 1) < LOG_R ? (hb - wl + 1) : LOG_R;
                    if constexpr (r > 0 || OUT_RAW) u60_inv_round_end<R, nexec>(ar, x);
                }
            });
        }

        // ---- store ----
        if constexpr (!INV && !COLS && (NR > 1 || BREV))
            exchange(std::integral_constant<int, NR - 1>{}, std::integral_constant<int, 0>{}, BREV);
        if constexpr (PACK_OUT) {
            // x[k]: row 16 tau + k of column off0 -> unit (rb = tau, t) column c = gl, staged in LDS
            uint32_t lo[16], mid[8] = {}, top = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint64_t u = ar.canon(x[k]);   // < q < 2^50
                lo[k] = (uint32_t)u;
                const uint32_t hi = (uint32_t)(u >> 32);
                mid[k >> 1] |= (hi & 0xFFFFu) << (16 * (k & 1));
                top |= (hi >> 16) << (2 * k);
            }
            __syncthreads();   // last exchange's readers are done with the LDS
            char* ub = (char*)lds + tau_ * kPackUnitBytes;
            uint4* plo = (uint4*)(ub + gl * 64);
            uint4* pmid = (uint4*)(ub + 1024 + gl * 32);
#pragma unroll
            for (int s = 0; s < 4; ++s) plo[s] = make_uint4(lo[4 * s], lo[4 * s + 1], lo[4 * s + 2], lo[4 * s + 3]);
#pragma unroll
            for (int s = 0; s < 2; ++s) pmid[s] = make_uint4(mid[4 * s], mid[4 * s + 1], mid[4 * s + 2], mid[4 * s + 3]);
            *(uint32_t*)(ub + 1536 + gl * 4) = top;
            __syncthreads();
            if (L.active) {
                // line j of unit rb -> row 16 rb + j of this column tile (its own, already read lines)
                const uint4* src = (const uint4*)lds;
                char* dst = (char*)L.base + (size_t)(L.off0 & ~15u) * 8;
                for (uint32_t q = threadIdx.x; q < 16 * kPackUnitBytes / 16; q += NT) {
                    const uint32_t m = q >> 3, rb = m / 13, j = m - 13 * rb;
                    *(uint4*)(dst + (size_t)(16 * rb + j) * kPackRowBytes + (q & 7) * 16) = src[q];
                }
            }
            return;
        }
        if (L.active) {
            if constexpr (UNI && kCpolSt != 0) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(L.base, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const uint32_t g = Gm::g_of(r_store, tau_, k);
                    T y = x[k];
                    if constexpr (TWIST && INV) y = ar.mulmod(y, a.twist.get(twoff + jidx(L, g)));
                    const uint64_t o = OUT_RAW ? ar.raw_out(y) : INV ? inv_out(ar, y) : ar.canon(y);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o),
                                                          rs, (int)(jidx(L, g) * 8u), 0, kCpolSt);
                }
            } else {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    const uint32_t g = Gm::g_of(r_store, tau_, k);
                    T y = x[k];
                    if constexpr (TWIST && INV) y = ar.mulmod(y, a.twist.get(twoff + jidx(L, g)));
#ifdef MFHE_EXP_SKIP
                    if (OUT_RAW && k >= 12) continue;   // traffic experiment only (wrong results)
#endif
                    L.base[jidx(L, g)] = OUT_RAW ? ar.raw_out(y) : INV ? inv_out(ar, y) : ar.canon(y);
                }
            }
        }
    }
};

// One launch runs one pass over the whole batch.  Workgroups are persistent: each walks tiles
// blockIdx.x, blockIdx.x + gridDim.x, ... (gridDim.x a multiple of 8, so a workgroup's tiles all fall
// in its XCD group's contiguous range of xcd_remap).  PF: the raw loads of the next tile are issued
// before the butterflies of the current one.
template <class P, bool PF, class TS>
__device__ __forceinline__ void pass_loop(const PassArgs<TS>& a, uint64_t* lds) {
    const P p(a);
    const uint32_t nb = a.nblocks;
    uint32_t lt = blockIdx.x;
    if (lt >= nb) return;
    TileLoc L = p.locate(xcd_remap(lt, nb));
    uint64_t raw[P::R];
    p.load(L, raw);
    while (true) {
        const uint32_t nlt = lt + gridDim.x;
        const bool more = nlt < nb;   // workgroup-uniform
        TileLoc Ln;
        uint64_t nraw[PF ? P::R : 1];
        if constexpr (PF) {
            if (more) {
                Ln = p.locate(xcd_remap(nlt, nb));
                p.load(Ln, nraw);
            }
        }
        p.compute_store(L, raw, lds);
        if (!more) break;
        lt = nlt;
        if constexpr (PF) {
            L = Ln;
            for (int k = 0; k < P::R; ++k) raw[k] = nraw[k];   // register renaming, no code
        } else {
            L = p.locate(xcd_remap(lt, nb));
            p.load(L, raw);
        }
        // the next tile's first LDS exchange starts with a barrier, so LDS rows are not overwritten early
    }
}

// Minimum resident workgroups per CU the register allocation must allow (launch-bounds waves/SIMD).
#ifndef MFHE_NTT_MIN_WG_CU
#define MFHE_NTT_MIN_WG_CU 1
#endif
constexpr int min_waves_per_simd(int nt) {
    return (MFHE_NTT_MIN_WG_CU * nt / 256) < 1 ? 1 : (MFHE_NTT_MIN_WG_CU * nt / 256);
}

// U64 block passes (A/B, MFHE_NTT_U64_BLOCK_W4): registers held to 4 waves per SIMD (128 VGPRs); the inverse's first
// pass otherwise compiles to 129 and runs 3
#ifndef MFHE_NTT_U64_BLOCK_W4
#define MFHE_NTT_U64_BLOCK_W4 0
#endif
template <class A, bool COLS>
constexpr int pass_min_waves(int nt) {
    return (MFHE_NTT_U64_BLOCK_W4 && kIsU64<A> && !COLS && nt <= 256) ? 4 : min_waves_per_simd(nt);
}

template <class A, class TS, int LOG_G, int LOG_R, int NG, bool COLS, bool INV, bool IN_RAW, bool OUT_RAW,
          bool TWIST, bool BREV, bool UNI, bool PF, bool PACK = false>
__global__ __launch_bounds__(NG * (1 << (LOG_G - LOG_R)), (pass_min_waves<A, COLS>(NG * (1 << (LOG_G - LOG_R)))))
void ntt_pass_kernel(PassArgs<TS> a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    pass_loop<NttPass<A, TS, LOG_G, LOG_R, NG, COLS, INV, IN_RAW, OUT_RAW, TWIST, BREV, UNI, PACK>, PF>(a, lds);
}

}  // namespace mfhe
