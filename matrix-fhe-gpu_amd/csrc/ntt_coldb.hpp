// ntt_coldb.hpp -- forward column pass of the two-pass NTT (first 8 stages, 16-column tiles, N = 2^15..2^17)
// with the next tile's LDS-DMA in flight while the current tile's butterflies run.
//
// Why: the column pass reads the transform input from HBM and is the slower of the two passes (98 vs 82 us
// per 240 MiB chunk at C3, profiles/r02_kernel_stats.csv).  In the plain pass a workgroup loads a tile,
// waits, computes and stores, so only the workgroups that happen to be in their load phase have bytes in
// flight.  Here every workgroup keeps one 32 KiB tile landing in LDS at all times: two tile buffers,
// tile t + 1 is DMA'd into one while tile t is transformed in the other.
//
// Counted waits.  vmcnt is in order on gfx950, so "tile t has landed" is s_waitcnt vmcnt(n) with n = the
// vector-memory operations issued after tile t's DMA: the previous tile's 16 stores and the next tile's
// 8 DMA instructions.  Nothing else in the loop touches vector memory: the twiddles of a limb (15 shared
// by the workgroup, 15 per thread) are loaded into registers when the limb changes, followed by
// vmcnt(0).  The DMA is issued by the builtin; the ISA is checked to carry no compiler wait that would
// cover the prefetch.
//
// Same transform, same reduction schedule and same intermediate as NttPass<..., COLS, !INV, OUT_RAW>:
// the block pass that follows is unchanged, and the output is bit-identical (tests/test_ntt_gpu.py).
#pragma once
#include "ntt_kernels.hpp"

namespace mfhe {

#ifndef MFHE_NTT_CPOL_INV_COL_OUT
#define MFHE_NTT_CPOL_INV_COL_OUT MFHE_NTT_CPOL_OUT   // the inverse's last (column) pass output stores
#endif

#ifndef MFHE_NTT_U64_COLDB_WAVES
#define MFHE_NTT_U64_COLDB_WAVES 4   // single-buffer (U64) column pass: waves per SIMD the registers must allow (4: 128 VGPRs)
#endif

#ifndef MFHE_NTT_COLDB_NG
#define MFHE_NTT_COLDB_NG 16   // columns per tile: 16 (128-B row segments, 2 workgroups/CU) or 32 (256 B, 1/CU)
#endif

struct ColDb {
    static constexpr int LOG_G = 8, LOG_R = 4, NG = MFHE_NTT_COLDB_NG;
    static constexpr int LOG_NG = NG == 32 ? 5 : 4;
    static constexpr int CPR = NG / 2;                 // 16-B chunks per tile row
    using Gm = Geo<LOG_G, LOG_R>;
    static constexpr int R = Gm::R, TG = Gm::TG, GS = Gm::GS;
    static constexpr int NT = NG * TG;                 // 256 threads
    static constexpr int BUF = NG * GS;                // u64 words per tile buffer (exchange layout, 34,944 B)
    static constexpr size_t LDS_BYTES = 2 * (size_t)BUF * sizeof(uint64_t);
    static constexpr size_t LDS_BYTES_U64 = LDS_BYTES + 512 * sizeof(uint64_t);   // + the U64 twiddle table
    static constexpr size_t LDS_BYTES_SB_U64 = (size_t)BUF * sizeof(uint64_t) + 512 * sizeof(uint64_t);   // one buffer
    static constexpr int kDmaOps = 256 * NG * 8 / (NT * 16);  // 16-B DMA instructions per thread per tile (8)
    static_assert(Gm::NR == 2 && TG == 16, "two rounds of four stages");
    static_assert(NG == 16 || NG == 32, "16 or 32 columns per tile");
};

// tile (row-major [256 rows][NG columns] image, 8 NG bytes per row) -> buf by LDS-DMA, 16 B per lane
__device__ __forceinline__ void coldb_dma(const char* tile, size_t row_bytes, uint64_t* buf, uint32_t w, uint32_t lane) {
    typedef __attribute__((address_space(3))) void* lds_vp;
#pragma unroll
    for (int i = 0; i < ColDb::kDmaOps; ++i) {
        const uint32_t q = (i * (ColDb::NT / 64) + w) * 64 + lane;   // chunk: row q / CPR, part q % CPR
        const char* src = tile + (size_t)(q / ColDb::CPR) * row_bytes + (q % ColDb::CPR) * 16;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (lds_vp)((char*)buf + (size_t)(i * (ColDb::NT / 64) + w) * 1024), 16, 0,
                                         MFHE_NTT_CPOL_IN);
    }
}

template <int N>
__device__ __forceinline__ void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt immediate");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// LDS-only workgroup barrier: __syncthreads() also carries a workgroup release fence, i.e. a vmcnt(0) that
// would wait for the prefetch in flight.  Every cross-thread hand-off in this kernel goes through LDS
// (exchanges) or is ordered by an explicit vm_wait (DMA'd tiles), so lgkmcnt(0) + s_barrier suffices.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One column tile whose DMA has landed in buf ([256 rows][NG] row-major): stages 0..7, the exchange in buf itself,
// then the raw intermediate (F64: centred doubles; U64: [0, 2q)) stored to base (plain stores, R per thread).
// tw0: tw[1..15] of the limb (shared), tw1: this thread's round-1 twiddles ((16 + tau) << e) + j.  TW0 / TW1:
// anything indexable by [0, 15) giving A::Tw -- register arrays (F64), LDS table views (U64).
template <class A, bool STORE = true, class TW0, class TW1, class HOOK>
__device__ __forceinline__ void coldb_tile(uint64_t* buf, uint32_t gl, uint32_t tau, const LimbConst& lc,
                                           const TW0& tw0, const TW1& tw1, uint64_t* base, uint32_t off0, int logS,
                                           HOOK&& after_reads) {
    using C = ColDb;
    using Gm = C::Gm;
    uint64_t* my = buf + (size_t)gl * C::GS;
    const A ar(lc);
    typename A::T x[C::R];
#pragma unroll
    for (int k = 0; k < C::R; ++k) x[k] = A::from_u64(buf[(size_t)Gm::g_of(0, tau, k) * C::NG + gl]);
    // round 0: stages 0..3 (register bits 3..0), twiddles shared by the workgroup
    static_for<0, 4>([&](auto bi) {
        constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
        for (int k = 0; k < C::R; ++k) {
            if (k & half) continue;
            ar.ct(x[k], x[k + half], tw0[(1 << e) - 1 + (k >> (bb + 1))]);
        }
    });
    lds_barrier();
#pragma unroll
    for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(0, tau, k))] = A::to_raw(x[k]);
    lds_barrier();
#pragma unroll
    for (int k = 0; k < C::R; ++k) x[k] = ar.round_reduce(A::from_raw(my[Gm::pad(Gm::g_of(1, tau, k))]));
    after_reads();   // single-buffer kernel: every thread's reads are done -> the next tile's DMA may land here
    // round 1: stages 4..7, twiddles per thread
    static_for<0, 4>([&](auto bi) {
        constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
        for (int k = 0; k < C::R; ++k) {
            if (k & half) continue;
            if constexpr (bb == 3) ar.ct_first(x[k], x[k + half], tw1[(1 << e) - 1 + (k >> (bb + 1))]);
            else ar.ct(x[k], x[k + half], tw1[(1 << e) - 1 + (k >> (bb + 1))]);
        }
    });
    // intermediate, the same words NttPass<COLS, OUT_RAW> writes
#pragma unroll
    for (int k = 0; k < C::R; ++k) {
        const uint64_t o = ar.raw_out(x[k]);
        if constexpr (STORE) base[off0 | ((uint32_t)Gm::g_of(1, tau, k) << logS)] = o;
        else asm volatile("" ::"v"(o));   // timing probe (no store)
    }
}

// U64 twiddle views of a limb's table T = tw[0, 256) (value and Shoup companion) held in LDS
struct Tw0U {
    const uint64_t* w;
    const uint64_t* ws;
    __device__ __forceinline__ ulonglong2 operator[](int j) const { return make_ulonglong2(w[1 + j], ws[1 + j]); }
};
struct Tw1U {
    const uint64_t* w;
    const uint64_t* ws;
    uint32_t tau;
    __device__ __forceinline__ ulonglong2 operator[](int i) const {   // i = 2^e - 1 + j, folded at compile time
        const int e = i >= 7 ? 3 : i >= 3 ? 2 : i >= 1 ? 1 : 0;
        const uint32_t t = ((16 + tau) << e) + (uint32_t)(i + 1 - (1 << e));
        return make_ulonglong2(w[t], ws[t]);
    }
};

// The inverse column pass (the last 8 GS stages, s = 7..0, of the inverse) on a DMA'd tile of the raw centred
// intermediate the inverse block pass wrote: NttPass<ArithF64, ..., COLS, INV, IN_RAW, !OUT_RAW>'s schedule --
// round 1 first (register bits 0..3, per-thread twiddles, even executed stage lazy), the exchange, round 0 (shared
// twiddles; the s = 0 stage folds n^-1 into X), canonical output stored sc1 nt (R buffer stores per thread).
// The inverse table has the forward one's shape, so tw0 / tw1 are coldb_twiddles of itw: round-1 stage bb uses
// itw[2^(7-bb) + (tau << (3-bb)) + m] = tw1[2^e - 1 + m], round-0 stage bb uses itw[2^(3-bb) + m] = tw0[2^e - 2 + m + 1]
// with e = 3 - bb.
template <class A, class TW0, class TW1, class HOOK>
__device__ __forceinline__ void coldb_tile_inv(uint64_t* buf, uint32_t gl, uint32_t tau, const LimbConst& lc,
                                               typename A::Tw ninv, const TW0& tw0, const TW1& tw1, uint64_t* base,
                                               uint32_t off0, int logS, HOOK&& after_reads) {
    using C = ColDb;
    using Gm = C::Gm;
    uint64_t* my = buf + (size_t)gl * C::GS;
    const A ar(lc);
    typename A::T x[C::R];
#pragma unroll
    for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(buf[(size_t)Gm::g_of(1, tau, k) * C::NG + gl]);
    if constexpr (kLazyU60<A>) {
        // the lazy U60 inverse (ntt_arith.hpp ArithU60::gs_b, U60InvBounds): the same two rounds with X unreduced
        static_for<0, 4>([&](auto bi) {
            constexpr int bb = decltype(bi)::value, e = 3 - bb;
            u60_inv_stage<C::R, bb, false>(ar, x, [&](int k) { return tw1[(1 << e) - 1 + (k >> (bb + 1))]; },
                                           typename A::Tw{});
        });
        u60_inv_round_end<C::R, 4>(ar, x);
        lds_barrier();
#pragma unroll
        for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(1, tau, k))] = A::to_raw(x[k]);
        lds_barrier();
#pragma unroll
        for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(0, tau, k))]);
        after_reads();
        static_for<0, 4>([&](auto bi) {
            constexpr int bb = decltype(bi)::value, e = 3 - bb;
            if constexpr (bb == 3) {
                const auto w1 = tw0[0];
                u60_inv_stage<C::R, bb, true>(ar, x, [&](int) { return w1; }, ninv);
            } else {
                u60_inv_stage<C::R, bb, false>(ar, x, [&](int k) { return tw0[(1 << e) - 1 + (k >> (bb + 1))]; },
                                               typename A::Tw{});
            }
        });
    } else {
    // round 1: stages 7..4 (register bits 0..3); executed stages 0..3 of the pass: even -> lazy GS
    static_for<0, 4>([&](auto bi) {
        constexpr int bb = decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
        for (int k = 0; k < C::R; ++k) {
            if (k & half) continue;
            const auto w = tw1[(1 << e) - 1 + (k >> (bb + 1))];
            if constexpr (bb % 2 == 0) ar.gs_lazy(x[k], x[k + half], w);
            else ar.gs(x[k], x[k + half], w);
        }
    });
    lds_barrier();
#pragma unroll
    for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(1, tau, k))] = A::to_raw(x[k]);
    lds_barrier();
#pragma unroll
    for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(0, tau, k))]);
    after_reads();
    // round 0: stages 3..0 (register bits 0..3); executed stages 4..7 of the pass: 4, 6 lazy, 5 reducing, and the
    // s = 0 stage: X = (u + v) n^-1, Y = (u - v) itw[1] (itw[1] carries n^-1)
    static_for<0, 4>([&](auto bi) {
        constexpr int bb = decltype(bi)::value, e = 3 - bb, half = 1 << bb;
        if constexpr (bb == 3) {
            const auto w1 = tw0[0];
#pragma unroll
            for (int k = 0; k < C::R; ++k) {
                if (k & half) continue;
                typename A::T u = x[k], v = x[k + half];
                ar.gs_lazy(u, v, w1);
                x[k] = ar.mulmod(u, ninv);
                x[k + half] = v;
            }
        } else {
#pragma unroll
            for (int k = 0; k < C::R; ++k) {
                if (k & half) continue;
                const auto w = tw0[(1 << e) - 1 + (k >> (bb + 1))];
                if constexpr (bb % 2 == 0) ar.gs_lazy(x[k], x[k + half], w);
                else ar.gs(x[k], x[k + half], w);
            }
        }
    });
    }
    // base is workgroup-uniform; say so (the U64 kernel otherwise wraps every store in a readfirstlane loop)
    const uint64_t bu = (uint64_t)base;
    uint64_t* const ubase = (uint64_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bu >> 32)) << 32) |
                                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bu));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ubase, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int k = 0; k < C::R; ++k)
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, inv_out(ar, x[k])), rs,
            (int)((off0 | ((uint32_t)Gm::g_of(0, tau, k) << logS)) * 8u), 0, MFHE_NTT_CPOL_INV_COL_OUT);
}

// a limb's column-pass twiddles into registers (tw0 shared, tw1 per thread), see coldb_tile.  tw0 is the same
// for every thread: read through the constant address space it is fetched by scalar loads into SGPRs, which
// count in lgkmcnt, not in the vmcnt the tile waits are counted against, and cost no VGPRs.
__device__ __forceinline__ void coldb_twiddles(const double* tw, uint32_t tau, double (&tw0)[15], double (&tw1)[15]) {
    typedef const __attribute__((address_space(4))) double* ctw_t;
    const ctw_t ctw = (ctw_t)tw;
#pragma unroll
    for (int j = 0; j < 15; ++j) tw0[j] = ctw[1 + j];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < (1 << e); ++j) tw1[(1 << e) - 1 + j] = tw[((16 + tau) << e) + j];
}

// INV: the inverse's last pass (the column stages), reading the raw intermediate of the inverse block pass from
// the Infinity Cache; otherwise the forward's first pass reading the transform input.
// A = ArithF64: the limb's twiddles in registers (tw0 by scalar loads); A = ArithU64: the limb's table tw[0, 256)
// and its Shoup companions DMA'd into LDS (4 KiB after the two tile buffers) -- 30 (w, w') pairs per thread do
// not fit beside the U64 butterflies' registers, and per-butterfly global loads were the r02 U64 pass's stall.
// SB (single buffer, the U64 default): one tile buffer; the next tile's DMA is issued once every thread has read the
// current tile's last LDS image (after the exchange), so it lands during the second round and the stores.  39 KiB of
// LDS and <= 128 VGPRs (MFHE_NTT_U64_COLDB_WAVES): 4 workgroups per CU instead of 2 -- the U64 pass is VALU-bound (busy
// 0.70 at 1.5 waves/SIMD, profiles/r03_ntt_sq_pmc.txt) and needs the waves more than the longer DMA lead.
template <class A, class TS, bool INV = false, bool SB = false>
__global__ __launch_bounds__(ColDb::NT, SB ? MFHE_NTT_U64_COLDB_WAVES : 1) void ntt_col_db_kernel(PassArgs<TS> a) {
    using C = ColDb;
    constexpr bool U = kIsU64<A>;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t t = threadIdx.x, gl = t % C::NG, tau = t / C::NG, w = t >> 6, lane = t & 63;
    const uint32_t nb = a.nblocks;
    uint32_t lt = blockIdx.x;
    if (lt >= nb) return;
    const int logS = a.logN - C::LOG_G;
    const size_t row_bytes = (size_t)8 << logS;
    auto locate = [&](uint32_t l) {
        return tile_loc<C::LOG_G, C::NG, true, true>(a.data, a.batch, a.nl, a.start_limb, a.logN, 0, xcd_remap(l, nb), gl);
    };
    auto tile_ptr = [&](const TileLoc& L) { return (const char*)(L.base + (L.off0 - gl)); };
    uint64_t* tabw = lds + (SB ? 1 : 2) * C::BUF;   // U64: [0, 256) values, [256, 512) Shoup companions
    typedef __attribute__((address_space(3))) void* lds_vp;

    TileLoc L0 = locate(lt);
    uint64_t* base = L0.base;   // current tile: polynomial base, element offset of its first row, limb
    uint32_t off0 = L0.off0;
    int lmod = L0.mod;
    coldb_dma(tile_ptr(L0), row_bytes, lds, w, lane);
    int cur = 0, mod = -1;
    bool first = true;
    LimbConst lc{};
    typename A::Tw ninv{};
    double tw0[15], tw1[15];   // F64 round 0: tw[1..15] (shared); round 1: ((16 + tau) << e) + j, e = 3 - bb
    while (true) {
        const uint32_t nlt = lt + gridDim.x;
        const bool more = nlt < nb;   // workgroup-uniform
        if (lmod != mod) {
            mod = lmod;
            // per-limb constants by scalar loads (constant address space): a vector load here would make the
            // compiler put a vmcnt(0) before their first use in the butterflies, which waits for the prefetch
            {
                const __attribute__((address_space(4))) LimbConst* cl =
                    (const __attribute__((address_space(4))) LimbConst*)a.limbs + mod;
                lc.q = cl->q;
                lc.qf = cl->qf;
                lc.qinv = cl->qinv;
            }
            if constexpr (!U) {
                if constexpr (INV) ninv = ((const __attribute__((address_space(4))) double*)a.ninv.p)[mod];
                coldb_twiddles(a.tw.p + ((size_t)mod << a.logN), tau, tw0, tw1);
                vm_wait<0>();   // twiddles in registers (also drains tile t's DMA and the previous stores)
                // re-define the twiddle registers by an (empty) asm after the wait: the compiler's own wait tracking
                // would otherwise keep these loads pending into the butterflies and put a vmcnt(0) there, which
                // also waits for the next tile's DMA
#pragma unroll
                for (int j = 0; j < 15; ++j) asm volatile("" : "+v"(tw1[j]));
            } else {
                typedef const __attribute__((address_space(4))) uint64_t* cu64_t;
                if constexpr (INV) ninv = make_ulonglong2(((cu64_t)a.ninv.w)[mod], ((cu64_t)a.ninv.ws)[mod]);
                lds_barrier();   // every thread is done with the previous limb's table
                // waves 0, 1: tw[0, 256); waves 2, 3: the Shoup companions (1 KiB per DMA instruction)
                const uint64_t* src = (w < 2 ? a.tw.w : a.tw.ws) + ((size_t)mod << a.logN) + (w & 1) * 128 + lane * 2;
                __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)(tabw + (w >> 1) * 256 + (w & 1) * 128), 16,
                                                 0, 0);
                vm_wait<0>();   // table landed for this wave (published by the barrier below)
            }
        }
        uint64_t* nbase = base;
        uint32_t noff0 = off0;
        int nmod = lmod;
        const char* ntile = nullptr;   // the next tile's first row (DMA source)
        if (more) {
            const TileLoc Ln = locate(nlt);
            nbase = Ln.base;
            noff0 = Ln.off0;
            nmod = Ln.mod;
            ntile = tile_ptr(Ln);
        }
        if constexpr (!SB) {
            lds_barrier();   // every thread is done with the other buffer (previous tile's exchange reads)
            if (more) coldb_dma(ntile, row_bytes, lds + (cur ^ 1) * C::BUF, w, lane);
            // this thread's part of tile t has landed: newer than its DMA are the previous tile's R stores and the
            // next tile's DMA instructions
            if (first) {
                if (more) vm_wait<C::kDmaOps>();
                else vm_wait<0>();
            } else {
                if (more) vm_wait<C::R + C::kDmaOps>();
                else vm_wait<C::R>();
            }
        } else {
            // single buffer: tile t's DMA was issued during tile t - 1, before that tile's R stores
            if (first) vm_wait<0>();
            else vm_wait<C::R>();
        }
        lds_barrier();   // ... and every other thread's part
        first = false;

        uint64_t* buf = lds + (size_t)(SB ? 0 : cur) * C::BUF;
        auto hook = [&]() {
            if constexpr (SB) {
                if (more) {
                    lds_barrier();   // every thread has read the buffer's last image of tile t
                    coldb_dma(ntile, row_bytes, lds, w, lane);
                }
            }
        };
        if constexpr (U) {
            const Tw0U t0{tabw, tabw + 256};
            const Tw1U t1{tabw, tabw + 256, tau};
            if constexpr (INV) coldb_tile_inv<A>(buf, gl, tau, lc, ninv, t0, t1, base, off0, logS, hook);
            else coldb_tile<A>(buf, gl, tau, lc, t0, t1, base, off0, logS, hook);
        } else {
            if constexpr (INV) coldb_tile_inv<A>(buf, gl, tau, lc, ninv, tw0, tw1, base, off0, logS, hook);
            else coldb_tile<A>(buf, gl, tau, lc, tw0, tw1, base, off0, logS, hook);
        }
        if (!more) break;
        lt = nlt;
        base = nbase;
        off0 = noff0;
        lmod = nmod;
        cur ^= 1;
    }
}

}  // namespace mfhe
