// ntt_blkdb.hpp -- block pass of the N = 2^16 two-pass NTT (FP64) with the next tile's LDS-DMA in flight, as
// ntt_coldb.hpp does for the column pass: the forward's second pass (raw intermediate from the Infinity Cache ->
// canonical output) and the inverse's first pass (canonical input from HBM -> raw intermediate).
// MFHE_OPT_NTT_PREFETCH = 3.
//
// Tile: 16 consecutive rows of the 256 x 256 view of one polynomial, i.e. 32 KiB of contiguous memory, moved
// global -> LDS by 8 LDS-DMA instructions per thread.  Thread (gl = t / 16, tau = t % 16) owns row gl, elements
// k * 16 + tau -- NttPass<..., !COLS, ...>'s block layout -- and reads them out of the DMA'd image before the
// first exchange overwrites the buffer with the padded exchange layout (ColDb's buffer size).
//
// Twiddles: 15 per row (round 0, shared by the row's 16 threads) and 15 per thread (round 1), L2-resident
// global loads.  hipcc puts a vmcnt(0) before the first use of an ordinary load's result while an LDS-DMA is in
// flight, so a tile's twiddles are loaded and consumed (re-defined by empty asm statements) at the top of its
// iteration, before the next tile's DMA is issued: one vmcnt(0) per tile there -- which also covers this tile's
// DMA, issued one iteration earlier -- and none inside the butterflies, where the next tile's DMA is in flight.
#pragma once
#include "ntt_coldb.hpp"

namespace mfhe {

struct BlkDb {
    static constexpr int LOG_G = 8, NG = 16, R = 16, NT = 256;
    using Gm = Geo<8, 4>;
    static constexpr int GS = Gm::GS;
    static constexpr int BUF = NG * GS;                                // u64 words per buffer (34,944 B)
    static constexpr size_t LDS_BYTES = 2 * (size_t)BUF * sizeof(uint64_t);
    static constexpr int kDmaOps = 8;                                  // 32 KiB / (256 threads x 16 B)
    static_assert(BUF == ColDb::BUF && ColDb::kDmaOps == kDmaOps, "same buffers and DMA as the column pass");
};

// the tile's twiddles for rows hi (this thread's row): round 0 tw[(256 << e) + (hi << e) + j], round 1
// tw[(4096 << e) + ((16 hi + tau) << e) + j], e = 0..3 (index (1 << e) - 1 + j) -- NttPass::stage at s0 = 8
__device__ __forceinline__ void blkdb_twiddles(const double* tw, uint32_t hi, uint32_t tau, double (&twa)[15],
                                               double (&twb)[15]) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < (1 << e); ++j) {
            twa[(1 << e) - 1 + j] = tw[(256u << e) + (hi << e) + j];
            twb[(1 << e) - 1 + j] = tw[(4096u << e) + ((hi * 16 + tau) << e) + j];
        }
}

template <bool INV>
__global__ __launch_bounds__(BlkDb::NT, 2) void ntt_blk_db_kernel(PassArgs<TwSrcF> a) {
    using A = ArithF64;
    using C = BlkDb;
    using Gm = C::Gm;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    const uint32_t t = threadIdx.x, gl = t / 16, tau = t % 16, w = t >> 6, lane = t & 63;
    const uint32_t nb = a.nblocks;
    uint32_t lt = blockIdx.x;
    if (lt >= nb) return;
    auto locate = [&](uint32_t l) {
        return tile_loc<C::LOG_G, C::NG, false, true>(a.data, a.batch, a.nl, a.start_limb, a.logN, a.logN - C::LOG_G,
                                                      xcd_remap(l, nb), gl);
    };
    // row 0 of the tile: 16 rows x 2 KiB contiguous, copied as one 32 KiB image (coldb_dma with 128-B "rows")
    auto tile_ptr = [&](const TileLoc& L) { return (const char*)(L.base + (L.off0 - gl * 256u)); };
    typedef const __attribute__((address_space(4))) LimbConst* climb_t;

    TileLoc L = locate(lt);
    coldb_dma(tile_ptr(L), 128, lds, w, lane);
    int cur = 0;
    while (true) {
        const uint32_t nlt = lt + gridDim.x;
        const bool more = nlt < nb;   // workgroup-uniform
        double twa[15], twb[15];
        blkdb_twiddles(a.tw.p + L.twoff, (uint32_t)L.hi, tau, twa, twb);
        vm_wait<0>();   // the twiddles, this tile's DMA (issued last iteration), the previous tile's stores
#pragma unroll
        for (int k = 0; k < 15; ++k) {
            asm volatile("" : "+v"(twa[k]));
            asm volatile("" : "+v"(twb[k]));
        }
        lds_barrier();   // every thread's part of this tile landed; everyone is done with the other buffer
        TileLoc Ln = L;
        if (more) {
            Ln = locate(nlt);
            coldb_dma(tile_ptr(Ln), 128, lds + (cur ^ 1) * C::BUF, w, lane);
        }

        uint64_t* buf = lds + (size_t)cur * C::BUF;
        uint64_t* my = buf + (size_t)gl * C::GS;
        const climb_t cl = (climb_t)a.limbs + L.mod;
        const A ar(LimbConst{0, cl->qf, cl->qinv, 0});
        double x[C::R];
#pragma unroll
        for (int k = 0; k < C::R; ++k) {
            const uint64_t v = buf[gl * 256u + k * 16 + tau];
            x[k] = INV ? A::from_u64(v) : A::from_raw(v);
        }
        lds_barrier();   // the image is read: the exchanges may overwrite it
        if constexpr (!INV) {
            // round 0 (stages 8..11, shared twiddles), exchange, round 1 (stages 12..15, per-thread twiddles)
            static_for<0, 4>([&](auto bi) {
                constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
                for (int k = 0; k < C::R; ++k) {
                    if (k & half) continue;
                    ar.ct(x[k], x[k + half], twa[(1 << e) - 1 + (k >> (bb + 1))]);
                }
            });
#pragma unroll
            for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(0, tau, k))] = A::to_raw(x[k]);
            lds_barrier();
#pragma unroll
            for (int k = 0; k < C::R; ++k) x[k] = ar.round_reduce(A::from_raw(my[Gm::pad(Gm::g_of(1, tau, k))]));
            static_for<0, 4>([&](auto bi) {
                constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
                for (int k = 0; k < C::R; ++k) {
                    if (k & half) continue;
                    ar.ct(x[k], x[k + half], twb[(1 << e) - 1 + (k >> (bb + 1))]);
                }
            });
            lds_barrier();
#pragma unroll
            for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(1, tau, k))] = A::to_raw(x[k]);
            lds_barrier();
#pragma unroll
            for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(0, tau, k))]);
        } else {
            // exchange into round 1's layout, round 1 (stages 15..12: executed 0..3, even lazy), exchange,
            // round 0 (stages 11..8: executed 4..7)
#pragma unroll
            for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(0, tau, k))] = A::to_raw(x[k]);
            lds_barrier();
#pragma unroll
            for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(1, tau, k))]);
            static_for<0, 4>([&](auto bi) {
                constexpr int bb = decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
                for (int k = 0; k < C::R; ++k) {
                    if (k & half) continue;
                    const double tw = twb[(1 << e) - 1 + (k >> (bb + 1))];
                    if constexpr (bb % 2 == 0) ar.gs_lazy(x[k], x[k + half], tw);
                    else ar.gs(x[k], x[k + half], tw);
                }
            });
            lds_barrier();
#pragma unroll
            for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(1, tau, k))] = A::to_raw(x[k]);
            lds_barrier();
#pragma unroll
            for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(0, tau, k))]);
            static_for<0, 4>([&](auto bi) {
                constexpr int bb = decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
                for (int k = 0; k < C::R; ++k) {
                    if (k & half) continue;
                    const double tw = twa[(1 << e) - 1 + (k >> (bb + 1))];
                    if constexpr (bb % 2 == 0) ar.gs_lazy(x[k], x[k + half], tw);
                    else ar.gs(x[k], x[k + half], tw);
                }
            });
        }
        // row gl, elements k * 16 + tau: 16 lanes store 128 contiguous bytes
        const uint64_t bu = (uint64_t)L.base;
        uint64_t* const ubase = (uint64_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bu >> 32)) << 32) |
                                            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bu));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ubase, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (int k = 0; k < C::R; ++k) {
            const uint64_t v = INV ? A::to_raw(x[k]) : ar.canon(x[k]);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), rs,
                                                  (int)((L.off0 + k * 16 + tau) * 8u), 0,
                                                  INV ? MFHE_NTT_CPOL_MID_ST : MFHE_NTT_CPOL_OUT);
        }
        if (!more) break;
        lt = nlt;
        L = Ln;
        cur ^= 1;
    }
}

}  // namespace mfhe
