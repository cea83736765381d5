// ntt_plans.hpp -- NTT launch plans (single pass / two-pass) shared by the per-arithmetic,
// per-direction translation units ntt_{f64,u64}_{fwd,inv}.hip (split so they compile in parallel).
//
// Plans (one launch per pass over the whole batch; the reference launches
// fnwt_1d once per polynomial, ntt_core.cu:445-449):
//   logN <= 14 : single pass, whole polynomial per workgroup group-set
//   logN 15-17 : pass A = first 8/9 stages on strided columns (COLS lanes),
//                pass B = remaining 7/8 stages on contiguous blocks
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mfhe_ctx.hpp"
#include "ntt_coldb.hpp"
#include "ntt_single14.hpp"

// Groups (contiguous rows) per block-pass workgroup.  N = 2^16: 4 rows (64 threads, 8.7 KiB LDS) rather than 16
// (256 threads, 34.9 KiB): the block pass gains from residency and 16-row tiles are LDS-bound at 4 per CU;
// C3 +0.9% forward / +1.4% inverse (profiles/r02_block_ng.txt).
#ifndef MFHE_NTT_NGB16
#define MFHE_NTT_NGB16 4
#endif
#ifndef MFHE_NTT_NGA14
#define MFHE_NTT_NGA14 16   // N = 2^14 two-pass plan: columns per column-pass workgroup (16: 128-B row segments, +5% C2 fwd over 32)
#endif
#ifndef MFHE_NTT_NGB14
#define MFHE_NTT_NGB14 8    // N = 2^14 two-pass plan: 128-element rows per block-pass workgroup (32 -> 8)
#endif
#ifndef MFHE_NTT_NGA17I
#define MFHE_NTT_NGA17I 8   // N = 2^17 inverse: columns per column-pass workgroup (second pass, 9 stages)
#endif
#ifndef MFHE_NTT_NGB17I
#define MFHE_NTT_NGB17I 4   // N = 2^17 inverse: 256-element rows per block-pass workgroup (first pass, reads the input)
#endif
#ifndef MFHE_NTT_NGB17
#define MFHE_NTT_NGB17 4    // N = 2^17 forward: 512-element rows per block-pass workgroup (8 -> 4: +0.9% C5 shard)
#endif
#ifndef MFHE_NTT_INV17_SPLIT
#define MFHE_NTT_INV17_SPLIT 0      // N = 2^17 inverse: 0 = 8 block + 9 column stages; 1 = 9 block + 8 column (DMA pass)
#endif
#ifndef MFHE_NTT_U64_COLDB_SB
#define MFHE_NTT_U64_COLDB_SB 1     // U64 column pass: 1 = single tile buffer, 3 workgroups per CU; 0 = double buffer, 2
#endif
#ifndef MFHE_NTT_INV16_PLAIN_NG
#define MFHE_NTT_INV16_PLAIN_NG 0   // N = 2^16 inverse last pass: 0 = DMA column pass; 16 / 32 = plain column pass (A/B)
#endif

namespace mfhe {

enum class Kind { Phantom, GL, Cyclic };

template <class TS>
struct NttJob {
    uint64_t* data;
    uint64_t batch;
    int nl, start_limb, logN;
    TS tw, twist, ninv;
    const LimbConst* limbs;
    const uint64_t* qraw;
    int qstride;
    int64_t chunk_bytes;  // two-pass batch chunking (0 = whole batch per pass)
    int plan;             // MFHE_OPT_NTT_PLAN
    int wg_per_cu;        // MFHE_OPT_NTT_WG_PER_CU (0 = occupancy limit)
    int prefetch;         // MFHE_OPT_NTT_PREFETCH
    int pack = 0;         // MFHE_OPT_NTT_PACK: 50-bit packed intermediate (N = 2^16, F64)
    int num_cus;
    mfhe_ctx* ctx;        // owning context (null: raw phantom entry)
};

#ifndef MFHE_NTT_U64_BLOCK_PF
#define MFHE_NTT_U64_BLOCK_PF 0   // A/B: the U64 block passes with the next tile's loads issued before the butterflies
#endif
template <class A, class TS, int LOG_G, int LOG_R, int NG, bool COLS, bool INV, bool IN_RAW, bool OUT_RAW, bool TWIST,
          bool BREV, bool UNI, bool PACK = false>
static int launch_pass(const NttJob<TS>& j, int s0, hipStream_t st) {
    using Gm = Geo<LOG_G, LOG_R>;
    constexpr int TG = Gm::TG;
    constexpr int NT = NG * TG;
    const uint64_t npl = j.batch * (uint64_t)j.nl;
    const int logS = j.logN - s0 - LOG_G;
    const uint64_t gpp = (1ull << logS) << s0;
    const uint64_t groups = npl * gpp;
    const uint64_t nb = (groups + NG - 1) / NG;
    if (nb == 0) return MFHE_OK;
    if (nb > 0xFFFFFFFFull || npl >= 0xFFFFFFFFull)
        return set_error(MFHE_EINVAL, "NTT batch too large for one launch (batch * nlimbs must be < 2^32)");
    PassArgs<TS> a;
    a.data = j.data;
    a.tw = j.tw;
    a.twist = j.twist;
    a.ninv = j.ninv;
    a.limbs = j.limbs;
    a.qraw = j.qraw;
    a.qstride = j.qstride;
    a.batch = j.batch;
    a.nl = j.nl;
    a.start_limb = j.start_limb;
    a.logN = j.logN;
    a.s0 = s0;
    a.nblocks = (uint32_t)nb;
    const bool need_lds = (Gm::NR > 1) || BREV;
    const size_t lds = need_lds ? (size_t)NG * Gm::GS * sizeof(uint64_t) : 0;
    const bool pf = j.prefetch == 1 || (MFHE_NTT_U64_BLOCK_PF && kIsU64<A> && !COLS);
    auto kern = pf ? ntt_pass_kernel<A, TS, LOG_G, LOG_R, NG, COLS, INV, IN_RAW, OUT_RAW, TWIST, BREV, UNI, true, PACK>
                   : ntt_pass_kernel<A, TS, LOG_G, LOG_R, NG, COLS, INV, IN_RAW, OUT_RAW, TWIST, BREV, UNI, false, PACK>;
    // persistent grid: resident workgroups only (occupancy query cached per instantiation), a multiple of 8
    static int occ_cache[2] = {0, 0};
    int& occ = occ_cache[pf ? 1 : 0];
    if (occ == 0) {
        int o = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, kern, NT, lds) != hipSuccess || o < 1) o = 1;
        occ = o;
    }
    const int per_cu = j.wg_per_cu > 0 ? std::min(j.wg_per_cu, occ) : occ;
    uint64_t cap = std::max<uint64_t>(8, ((uint64_t)per_cu * j.num_cus) & ~7ull);
    if (j.wg_per_cu >= 16) cap = nb;   // non-persistent: one tile per workgroup
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nb, cap);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, st, a);
    MFHE_CHECK_LAUNCH("ntt_pass_kernel launch");
    return MFHE_OK;
}

// The column pass's counted vmcnt waits assume its loop issues exactly R stores + kDmaOps DMAs per tile: a build
// whose kernel spills (scratch loads/stores are vector-memory ops too) would make them too loose.  Checked once
// per process from the code object's metadata; such a build runs the plain column pass instead
// (tests/test_isa.py checks the instruction counts of the shipped library).
template <class A, class TS, bool INV, bool SB>
static bool col_db_usable() {
    static int ok = -1;
    if (ok < 0) {
        hipFuncAttributes fa{};
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(ntt_col_db_kernel<A, TS, INV, SB>)) == hipSuccess &&
             fa.localSizeBytes == 0;
    }
    return ok == 1;
}
// U64 runs the single-buffer column pass (3 workgroups per CU; ntt_coldb.hpp SB), FP64 the double buffer
template <class A>
constexpr bool col_db_single() { return kIsU64<A> && MFHE_NTT_U64_COLDB_SB; }

// column pass with the next tile's DMA in flight (ntt_coldb.hpp), MFHE_OPT_NTT_PREFETCH = 2: the forward's first
// pass, or (INV) the inverse's last pass
template <class A, class TS, bool INV>
static int launch_col_db(const NttJob<TS>& j, hipStream_t st) {
    using C = ColDb;
    constexpr bool SB = col_db_single<A>();
    constexpr size_t lds = SB ? C::LDS_BYTES_SB_U64 : kIsU64<A> ? C::LDS_BYTES_U64 : C::LDS_BYTES;
    const uint64_t npl = j.batch * (uint64_t)j.nl;
    const uint64_t nb = npl << (j.logN - C::LOG_G - C::LOG_NG);   // NG-column tiles: 2^(logN - 8) / NG per polynomial
    if (nb == 0) return MFHE_OK;
    if (nb > 0xFFFFFFFFull || npl >= 0xFFFFFFFFull)
        return set_error(MFHE_EINVAL, "NTT batch too large for one launch (batch * nlimbs must be < 2^32)");
    PassArgs<TS> a{};
    a.data = j.data;
    a.tw = j.tw;
    a.ninv = j.ninv;
    a.limbs = j.limbs;
    a.batch = j.batch;
    a.nl = j.nl;
    a.start_limb = j.start_limb;
    a.logN = j.logN;
    a.s0 = 0;
    a.nblocks = (uint32_t)nb;
    static int occ = 0;
    if (occ == 0) {
        int o = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, ntt_col_db_kernel<A, TS, INV, SB>, C::NT, lds) != hipSuccess ||
            o < 1)
            o = 1;
        occ = o;
    }
    const int per_cu = j.wg_per_cu > 0 ? std::min(j.wg_per_cu, occ) : occ;
    const uint64_t cap = std::max<uint64_t>(8, ((uint64_t)per_cu * j.num_cus) & ~7ull);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nb, cap);
    hipLaunchKernelGGL((ntt_col_db_kernel<A, TS, INV, SB>), dim3(grid), dim3(C::NT), lds, st, a);
    MFHE_CHECK_LAUNCH("ntt_col_db_kernel launch");
    return MFHE_OK;
}

// N = 2^14, FP64: one pass, one polynomial per workgroup at a time with the next one's loads in flight
// (ntt_single14.hpp).  Persistent grid of one workgroup per CU (144 KiB of LDS).
template <bool INV>
static int launch_s14(const NttJob<TwSrcF>& j, hipStream_t st) {
    const uint64_t npl = j.batch * (uint64_t)j.nl;
    if (npl == 0) return MFHE_OK;
    if (npl >= 0xFFFFFFFFull) return set_error(MFHE_EINVAL, "NTT batch too large for one launch (batch * nlimbs must be < 2^32)");
    PassArgs<TwSrcF> a{};
    a.data = j.data;
    a.tw = j.tw;
    a.ninv = j.ninv;
    a.limbs = j.limbs;
    a.batch = j.batch;
    a.nl = j.nl;
    a.start_limb = j.start_limb;
    a.logN = 14;
    a.nblocks = (uint32_t)npl;
    static int occ = 0;
    if (occ == 0) {
        int o = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, ntt14_kernel<INV>, S14::NT, S14::LDS_BYTES) != hipSuccess ||
            o < 1)
            o = 1;
        occ = o;
    }
    const uint32_t grid = (uint32_t)std::min<uint64_t>(npl, (uint64_t)occ * j.num_cus);
    hipLaunchKernelGGL((ntt14_kernel<INV>), dim3(grid), dim3(S14::NT), S14::LDS_BYTES, st, a);
    MFHE_CHECK_LAUNCH("ntt14_kernel launch");
    return MFHE_OK;
}

template <int LOGN>
struct SinglePlan {
    // 16 elements per thread (N = 2^14: 1024 threads, 128 VGPRs, 16 waves per CU).  The earlier 32 per
    // thread at 2^14 (512 threads) needed 234-256 VGPRs with spills and measured 1-10% slower.
    static constexpr int LOG_R = LOGN < 4 ? LOGN : 4;
    static constexpr int TG = 1 << (LOGN - LOG_R);
    static constexpr int NG = TG >= 256 ? 1 : 256 / TG;
};

template <class A, class TS, int LOGN, bool INV, bool TW>
static int single(const NttJob<TS>& j, hipStream_t st) {
    using P = SinglePlan<LOGN>;
    return launch_pass<A, TS, LOGN, P::LOG_R, P::NG, false, INV, false, false, TW, TW, P::NG == 1>(j, 0, st);
}

template <class A, class TS, bool INV, bool TW>
static int run_single(const NttJob<TS>& j, hipStream_t st) {
    switch (j.logN) {
        case 1: return single<A, TS, 1, INV, TW>(j, st);
        case 2: return single<A, TS, 2, INV, TW>(j, st);
        case 3: return single<A, TS, 3, INV, TW>(j, st);
        case 4: return single<A, TS, 4, INV, TW>(j, st);
        case 5: return single<A, TS, 5, INV, TW>(j, st);
        case 6: return single<A, TS, 6, INV, TW>(j, st);
        case 7: return single<A, TS, 7, INV, TW>(j, st);
        case 8: return single<A, TS, 8, INV, TW>(j, st);
        case 9: return single<A, TS, 9, INV, TW>(j, st);
        case 10: return single<A, TS, 10, INV, TW>(j, st);
        case 11: return single<A, TS, 11, INV, TW>(j, st);
        case 12: return single<A, TS, 12, INV, TW>(j, st);
        case 13: return single<A, TS, 13, INV, TW>(j, st);
        case 14: return single<A, TS, 14, INV, TW>(j, st);
        default: return set_error(MFHE_EUNSUPPORTED, "single-pass NTT supports log_n <= 14");
    }
}

// two-pass plans: pass A (COLS, s0 = 0, LOG_GA stages), pass B (block, s0 = LOG_GA).
// The batch is processed in chunks of about chunk_bytes so the raw intermediate written by pass A
// is still resident in the Infinity Cache (256 MiB) when pass B reads and overwrites it: HBM then
// sees ~one read and one write per element instead of two of each.
// register bits per round of the U64 block passes (the FP64 ones keep 4): 16 values per thread at 4
#ifndef MFHE_NTT_U64_BLOCK_LOGR
#define MFHE_NTT_U64_BLOCK_LOGR 4
#endif
#ifndef MFHE_NTT_U64_BLOCK_NG
#define MFHE_NTT_U64_BLOCK_NG 0   // 0: the plan's NGB
#endif

template <class A, class TS, int LOG_GA, int NGA, int LOG_GB, int NGB_, bool INV>
static int two_pass_chunk(const NttJob<TS>& c, int pass, hipStream_t st) {
    constexpr int RB = kIsU64<A> ? MFHE_NTT_U64_BLOCK_LOGR : 4;
    constexpr int NGB = (kIsU64<A> && MFHE_NTT_U64_BLOCK_NG > 0) ? MFHE_NTT_U64_BLOCK_NG : NGB_;
    // pass 0 = first pass of the direction (forward: column, inverse: block), 1 = second
    constexpr bool kPackable = std::is_same<A, ArithF64>::value && LOG_GA == 8 && NGA == 16 && LOG_GB == 8 && NGB == 16;
    if constexpr (!INV && kPackable) {
        if (c.pack) {
            if (pass == 0) return launch_pass<A, TS, LOG_GA, 4, NGA, true, false, false, true, false, false, true, true>(c, 0, st);
            return launch_pass<A, TS, LOG_GB, 4, NGB, false, false, true, false, false, false, true, true>(c, LOG_GA, st);
        }
    }
    if constexpr (LOG_GA == 8 && NGA == 16) {
        // the column pass with the next tile's DMA in flight: the forward's first pass, the inverse's second
        if (pass == (INV ? 1 : 0) && c.prefetch >= 2 && c.limbs && col_db_usable<A, TS, INV, col_db_single<A>()>())
            return launch_col_db<A, TS, INV>(c, st);
    }
    if (!INV) {
        if (pass == 0) return launch_pass<A, TS, LOG_GA, 4, NGA, true, false, false, true, false, false, true>(c, 0, st);
        return launch_pass<A, TS, LOG_GB, RB, NGB, false, false, true, false, false, false, true>(c, LOG_GA, st);
    }
    if (pass == 0) return launch_pass<A, TS, LOG_GB, RB, NGB, false, true, false, true, false, false, true>(c, LOG_GA, st);
    return launch_pass<A, TS, LOG_GA, 4, NGA, true, true, true, false, false, false, true>(c, 0, st);
}

// two-pass plans: pass A (COLS, s0 = 0, LOG_GA stages), pass B (block, s0 = LOG_GA).
// The batch is processed in chunks of about chunk_bytes so the raw intermediate written by pass A
// is still resident in the Infinity Cache (256 MiB) when pass B reads and overwrites it: HBM then
// sees ~one read and one write per element instead of two of each.
// (Running chunk c + 1's first pass on a second stream beside chunk c's second pass measured 13-23% slower
// at 64-128 MiB chunks, r02 with sc1 nt output stores as in r01 without: DESIGN.md §3.1.)
template <class A, class TS, int LOG_GA, int NGA, int LOG_GB, int NGB, bool INV>
static int two_pass(const NttJob<TS>& j, hipStream_t st) {
    const uint64_t poly_bytes = (uint64_t)j.nl << (j.logN + 3);
    uint64_t cb = j.batch;
    if (j.chunk_bytes > 0) cb = std::max<uint64_t>(1, (uint64_t)j.chunk_bytes / poly_bytes);
    const uint64_t nch = (j.batch + cb - 1) / cb;
    cb = (j.batch + nch - 1) / nch;   // equal chunks (no small tail chunk paying two launches for little work)
    auto chunk = [&](uint64_t k) {
        NttJob<TS> c = j;
        const uint64_t b0 = k * cb;
        c.batch = std::min<uint64_t>(cb, j.batch - b0);
        c.data = j.data + b0 * ((uint64_t)j.nl << j.logN);
        return c;
    };
    for (uint64_t k = 0; k < nch; ++k) {
        int rc;
        if ((rc = two_pass_chunk<A, TS, LOG_GA, NGA, LOG_GB, NGB, INV>(chunk(k), 0, st))) return rc;
        if ((rc = two_pass_chunk<A, TS, LOG_GA, NGA, LOG_GB, NGB, INV>(chunk(k), 1, st))) return rc;
    }
    return MFHE_OK;
}

template <class A, class TS, bool INV>
static int run_phantom(const NttJob<TS>& j, hipStream_t st) {
    // auto (plan 0, or 3): N = 2^14 with FP64 arithmetic and the context's limb table runs the pipelined single pass
    // (ntt_single14.hpp, one polynomial per CU with the next one's loads in flight, 16N bytes); otherwise (U64, or
    // the raw phantom entry points without a limb table) two passes (7 + 7): the plain single pass holds one 2^14
    // polynomial per CU and cannot overlap loads with butterflies (profiles/r02_c2_plans2.txt).  Plan 1 / 2 keep
    // the plain single pass / two passes for A/B.
    int kind = ntt_phantom_plan(std::is_same<A, ArithF64>::value, j.logN, j.plan, j.limbs != nullptr);
    if constexpr (std::is_same<A, ArithF64>::value) {
        if (kind == 4) return launch_s14<INV>(j, st);
    }
    const bool two = kind == 2;
    if (!two) return run_single<A, TS, INV, false>(j, st);
    switch (j.logN) {
        case 12: return two_pass<A, TS, 6, 64, 6, 64, INV>(j, st);
        case 13: return two_pass<A, TS, 7, 32, 6, 64, INV>(j, st);
        case 14: return two_pass<A, TS, 7, MFHE_NTT_NGA14, 7, MFHE_NTT_NGB14, INV>(j, st);
        case 15: return two_pass<A, TS, 8, 16, 7, 32, INV>(j, st);
        case 16:
            // the packed intermediate's units are laid out for 16-row block tiles
            if (!INV && j.pack) return two_pass<A, TS, 8, 16, 8, 16, INV>(j, st);
            if constexpr (INV && MFHE_NTT_INV16_PLAIN_NG > 0)
                return two_pass<A, TS, 8, MFHE_NTT_INV16_PLAIN_NG, 8, MFHE_NTT_NGB16, INV>(j, st);
            return two_pass<A, TS, 8, 16, 8, MFHE_NTT_NGB16, INV>(j, st);
        // N = 2^17: the forward column pass takes 8 stages on 16-column tiles (128-B row segments) and the block
        // pass 9; the inverse keeps 9 column + 8 block stages.  Measured per direction (profiles/r02_n17_split.txt):
        // forward +5%, inverse -2.5% with the other split.
        case 17:
            if constexpr (INV && MFHE_NTT_INV17_SPLIT == 1) return two_pass<A, TS, 8, 16, 9, MFHE_NTT_NGB17, INV>(j, st);
            else if constexpr (INV) return two_pass<A, TS, 9, MFHE_NTT_NGA17I, 8, MFHE_NTT_NGB17I, INV>(j, st);
            else return two_pass<A, TS, 8, 16, 9, MFHE_NTT_NGB17, INV>(j, st);
        default: return set_error(MFHE_EUNSUPPORTED, "NTT supports log_n <= 17");
    }
}

// Entry used by ntt.hip: phantom transforms run the plan for j.logN; GL / cyclic (TW) run the single-pass
// plan with the fused twist.  Instantiated once per (arith, direction) in ntt_{f64,u64}_{fwd,inv}.hip.
template <class A, class TS, bool INV>
int run_kind(const NttJob<TS>& j, Kind kind, hipStream_t st);

template <class A, class TS, bool INV>
int run_kind(const NttJob<TS>& j, Kind kind, hipStream_t st) {
    if (kind == Kind::Phantom) return run_phantom<A, TS, INV>(j, st);
    return run_single<A, TS, INV, true>(j, st);
}

extern template int run_kind<ArithF64, TwSrcF, false>(const NttJob<TwSrcF>&, Kind, hipStream_t);
extern template int run_kind<ArithF64, TwSrcF, true>(const NttJob<TwSrcF>&, Kind, hipStream_t);
extern template int run_kind<ArithU64, TwSrcU, false>(const NttJob<TwSrcU>&, Kind, hipStream_t);
extern template int run_kind<ArithU64, TwSrcU, true>(const NttJob<TwSrcU>&, Kind, hipStream_t);
extern template int run_kind<ArithU60, TwSrcU, false>(const NttJob<TwSrcU>&, Kind, hipStream_t);
extern template int run_kind<ArithU60, TwSrcU, true>(const NttJob<TwSrcU>&, Kind, hipStream_t);

}  // namespace mfhe
