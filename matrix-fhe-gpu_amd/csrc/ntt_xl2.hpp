// ntt_xl2.hpp -- N = 2^16 forward NTT (FP64) in ONE persistent launch whose column -> block hand-off stays inside
// one XCD's L2 (MFHE_OPT_NTT_PLAN = 5).
//
// Why.  The two-pass plan moves 32N bytes across the L2 <-> fabric boundary per transform (the intermediate goes
// out to the Infinity Cache and back) and runs at the speed of two plain in-place copies (frac 0.37,
// profiles/r03_twopass_floor.txt).  Here a polynomial's 16 column tiles (stages 0..7) and 16 block tiles (stages
// 8..15) are processed by workgroups of ONE XCD, a few polynomials at a time, so the intermediate is written to and
// read back from that XCD's 4 MiB L2: 16N across the fabric.  The memory schedule alone was measured first
// (tools/microbench/l2_handoff_floor.hip, profiles/r05_l2_handoff_floor.txt).
//
// Queues.  A workgroup reads its XCD from HW_REG_XCC_ID and only takes tasks of that XCD, so producer and consumer
// of every intermediate tile run on the same XCD by construction -- placement is read at run time, never assumed.
// At the start every workgroup registers its XCD (the returned count is its rank inside the XCD) and waits (bounded)
// until the whole grid has (one grid-wide arrival, a few µs per 2.5 ms launch): the NX XCDs present get dense ranks,
// XCD rank r owns the global mini-chunks g = c NX + r, c = 0, 1, ... (M = MFHE_XL2_M polynomials each, limb-major),
// whatever the device's XCD count and ids, and inside an XCD the tasks are dealt round-robin over its workgroups.  An XCD's task sequence is blocks of 16 M
// tasks: A(0..lam), B(0), A(lam + 1), B(1), ..., then the remaining B blocks, where A(c) are the column tiles and
// B(c) the block tiles of its chunk c; its length is known, so a workgroup stops at the first task id past it.
//
// Hand-off.  An A task stores its intermediate with plain stores (the lines stay in this XCD's L2), every storing
// wave's stores are complete (counted vmcnt, below) before a workgroup barrier, then one lane adds 1 to done[x][c]
// (an agent-scope atomic, performed at the L2).  A B task's DMA waits until done[x][c] reads 16 M (sc1 loads); EVERY
// load of the tile is an LDS-DMA with sc1 (bypasses the CU's vector L1, served by the XCD's L2, the point of
// coherence for both workgroups).  No agent-scope release is needed because no byte crosses an L2: that release
// (buffer_wbl2) would write the intermediate back to memory, the 8N this plan exists to save.
//
// Pipeline.  Per iteration every thread issues the next tile's LDS-DMA (its data, and for a B tile its 32 KiB of
// stage-8..15 twiddles; one tile always landing while another is transformed, two 66 KiB slots), then transforms and
// stores the current tile.  The top of the
// next iteration waits with a counted vmcnt(16): the DMA and twiddles are complete, the 16 stores just issued may
// stay in flight -- they are known complete one iteration later, which is when an A task is signalled.  The
// B-readiness poll (lane 0) is issued one iteration ahead as a one-dword LDS-DMA, so it holds no register and its
// result is covered by that same counted wait.  A next B tile whose chunk is not yet
// complete is not prefetched: the workgroup drains, signals everything it stored, then polls (bounded) -- so no
// workgroup ever waits while it holds an unsignalled A task, and every wait is for tasks earlier in its XCD's
// sequence: the earliest waited-on task is always runnable (no deadlock for any residency after the start).  Every
// spin is bounded; a timeout sets a sticky word and ends the spins (results are then wrong, never a hang;
// MFHE_OPT_NTT_XL2_TIMEOUT reads it).
//
// Arithmetic.  A tasks run stages 0..7 on a 16-column tile, B tasks stages 8..15 on 16 rows: NttPass's schedule and
// reductions (xl2_tile), so the intermediate and the outputs are bit-identical to the two-pass plan's.
#pragma once
#include "ntt_coldb.hpp"

#ifndef MFHE_XL2_M
#define MFHE_XL2_M 2       // polynomials per mini-chunk
#endif
#ifndef MFHE_XL2_LAM
#define MFHE_XL2_LAM 2     // A blocks the sequence runs ahead of its B blocks
#endif
#ifndef MFHE_XL2_OUT_CPOL
#define MFHE_XL2_OUT_CPOL 0   // final output stores: plain (write-back; measured best on this schedule)
#endif
#ifndef MFHE_XL2_PROBE
#define MFHE_XL2_PROBE 0   // timing probes (wrong results): 1 = no output / intermediate stores, 2 = also no DMA
#endif
#ifndef MFHE_XL2_LOG_R
#define MFHE_XL2_LOG_R 4   // elements per thread 2^LOG_R: 4 = 256-thread workgroups, 3 = 512 (two waves per SIMD)
#endif
#ifndef MFHE_XL2_WPC
#define MFHE_XL2_WPC 1     // workgroups per CU
#endif

namespace mfhe {

struct Xl2Args {
    uint64_t* data;          // [batch][nl][2^16]
    const double* tw;        // forward phantom table [mod][2^16] (centred doubles)
    const LimbConst* limbs;  // [mod]
    uint32_t* st;            // state words (zeroed before every launch)
    uint32_t batch, nl, start_limb;
    uint32_t npoly;          // batch * nl
    uint32_t nchunk;         // ceil(npoly / M)
    uint32_t cmax;           // per-XCD chunk slots (>= chunks of any XCD)
};

// state layout (u32 words): scratch words (510, 511); the grid arrival counter; the timeout word; the XCD
// registration counts reg[16] (one line); then done[16][cmax]
constexpr uint32_t kXl2Arr = 512, kXl2Tmo = 513, kXl2Reg = 544, kXl2Done = 1024;
inline size_t xl2_state_words(uint32_t cmax) { return kXl2Done + 16ull * cmax; }

__device__ __forceinline__ uint32_t xl2_xcc() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 15u;
}
__device__ __forceinline__ uint32_t xl2_ld(uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t xl2_add(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A task id of an XCD with nc chunks -> block type / XCD-local chunk / tile inside the chunk.  Blocks: A(0..na-1),
// then B(0), A(na), B(1), A(na + 1), ... while A chunks remain, then the remaining B blocks (na = min(lam + 1, nc)).
struct Xl2Task {
    bool a;
    uint32_t c, tile;
};
template <uint32_t M, uint32_t LAM>
__device__ __forceinline__ Xl2Task xl2_decode(uint32_t id, uint32_t nc) {
    constexpr uint32_t TPB = 16 * M;
    const uint32_t b = id / TPB;
    const uint32_t na = nc < LAM + 1 ? nc : LAM + 1, mid = 2 * (nc - na);
    Xl2Task k;
    k.tile = id - b * TPB;
    if (b < na) {
        k.a = true;
        k.c = b;
    } else if (b < na + mid) {
        const uint32_t j = b - na;
        k.a = (j & 1) != 0;
        k.c = k.a ? na + (j >> 1) : (j >> 1);
    } else {
        k.a = false;
        k.c = b - nc;
    }
    return k;
}

// ---- generic tile code for NT = 16 * 2^(8 - LOG_R) threads (LOG_R = 4: 256 threads, 16 elements each; LOG_R = 3:
// 512 threads, 8 elements each, three rounds) ----
// A tile (COLS): 16 columns x 256 rows DMA'd as [256][16]: stages 0..7, stored in the last round's layout (each
// wave instruction covers whole 128-B row segments).  B tile: 16 rows x 256 DMA'd as [16][256]: stages 8..15,
// exchanged back to the round-0 layout for contiguous row stores.  NttPass's schedule (same rounds, same
// reductions: bit-identical outputs), with LDS-only barriers and twiddles from registers:
// tw[r][(1 << (LOG_R - 1 - bb)) - 1 + m] for round r, register bit bb, m < 2^(LOG_R - 1 - bb).
template <int LOG_R>
struct Xl2G {
    using Gm = Geo<8, LOG_R>;
    static constexpr int R = Gm::R, TG = Gm::TG, NR = Gm::NR, NT = 16 * TG, GS = Gm::GS;
    static constexpr int TWR = R - 1;   // twiddle slots per round
};

// the twiddles a thread needs for one tile from the table: COLS (A, per limb: hi = 0) or block (B, per row hi)
template <int LOG_R, bool COLS>
__device__ __forceinline__ void xl2_twiddles(const double* tw, uint32_t hi, uint32_t tau,
                                             double (&w)[Xl2G<LOG_R>::NR][Xl2G<LOG_R>::TWR]) {
    using G = Xl2G<LOG_R>;
    using Gm = typename G::Gm;
    const int s0 = COLS ? 0 : 8;
    static_for<0, G::NR>([&](auto rc) {
        constexpr int r = decltype(rc)::value, hb = Gm::HB(r), wl = Gm::WL(r);
        const uint32_t tau_hi = tau >> wl;
        static_for<0, LOG_R>([&](auto bi) {
            constexpr int bb = decltype(bi)::value, bit = wl + bb;
            if constexpr (bit <= hb) {
                const int s = s0 + (8 - 1 - bit);
                const uint32_t twb = (1u << s) + (hi << (8 - 1 - bit)) + (tau_hi << (LOG_R - 1 - bb));
#pragma unroll
                for (int m = 0; m < (1 << (LOG_R - 1 - bb)); ++m) {
                    w[r][(1 << (LOG_R - 1 - bb)) - 1 + m] = tw[twb + m];
                }
            }
        });
    });
}

// B tiles: the tile's stage-8..15 twiddles are DMA'd next to its data ([stage e][16 rows][2^e], offset 16 (2^e - 1)
// doubles for stage 8 + e, 4080 doubles, see xl2_twdma); this thread's share into registers (ds_reads)
template <int LOG_R>
__device__ __forceinline__ void xl2_btw_lds(const double* tl, uint32_t gl, uint32_t tau,
                                            double (&w)[Xl2G<LOG_R>::NR][Xl2G<LOG_R>::TWR]) {
    using G = Xl2G<LOG_R>;
    using Gm = typename G::Gm;
    static_for<0, G::NR>([&](auto rc) {
        constexpr int r = decltype(rc)::value, hb = Gm::HB(r), wl = Gm::WL(r);
        const uint32_t tau_hi = tau >> wl;
        static_for<0, LOG_R>([&](auto bi) {
            constexpr int bb = decltype(bi)::value, bit = wl + bb;
            if constexpr (bit <= hb) {
                constexpr int e = 7 - bit;   // stage 8 + e
                const uint32_t base = 16u * ((1u << e) - 1) + (gl << e) + (tau_hi << (LOG_R - 1 - bb));
#pragma unroll
                for (int m = 0; m < (1 << (LOG_R - 1 - bb)); ++m) w[r][(1 << (LOG_R - 1 - bb)) - 1 + m] = tl[base + m];
            }
        });
    });
}

template <int LOG_R, bool COLS, bool STORE = true>
__device__ __forceinline__ void xl2_tile(uint64_t* buf, uint32_t gl, uint32_t tau, const LimbConst& lc,
                                         const double (&w)[Xl2G<LOG_R>::NR][Xl2G<LOG_R>::TWR], uint64_t* base) {
    using G = Xl2G<LOG_R>;
    using Gm = typename G::Gm;
    using A = ArithF64;
    constexpr int R = G::R, NR = G::NR;
    const A ar(lc);
    double x[R];
    // round-0 layout reads of the DMA'd tile (raw canonical inputs for A, raw intermediate doubles for B)
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t g = Gm::g_of(0, tau, k);
        x[k] = COLS ? A::from_u64(buf[g * 16 + gl]) : A::from_raw(buf[gl * 256 + g]);
    }
    uint64_t* my = buf + (size_t)gl * G::GS;
    auto exchange = [&](auto rf, auto rt) {
        constexpr int r_from = decltype(rf)::value, r_to = decltype(rt)::value;
        lds_barrier();
#pragma unroll
        for (int k = 0; k < R; ++k) my[Gm::pad(Gm::g_of(r_from, tau, k))] = A::to_raw(x[k]);
        lds_barrier();
#pragma unroll
        for (int k = 0; k < R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(r_to, tau, k))]);
    };
    static_for<0, NR>([&](auto rc) {
        constexpr int r = decltype(rc)::value, hb = Gm::HB(r), wl = Gm::WL(r);
        if constexpr (r > 0) {
            exchange(std::integral_constant<int, r - 1>{}, rc);
#pragma unroll
            for (int k = 0; k < R; ++k) x[k] = ar.round_reduce(x[k]);
        }
        static_for<0, LOG_R>([&](auto bi) {
            constexpr int bb = LOG_R - 1 - decltype(bi)::value, bit = wl + bb, half = 1 << bb;
            if constexpr (bit <= hb) {
#pragma unroll
                for (int k = 0; k < R; ++k) {
                    if (k & half) continue;
                    ar.ct(x[k], x[k + half], w[r][(1 << (LOG_R - 1 - bb)) - 1 + (k >> (bb + 1))]);
                }
            }
        });
    });
    constexpr int r_store = COLS ? NR - 1 : 0;
    if constexpr (!COLS) exchange(std::integral_constant<int, NR - 1>{}, std::integral_constant<int, 0>{});
    const uint64_t bu = (uint64_t)base;
    uint64_t* const ub = (uint64_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bu >> 32)) << 32) |
                                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bu));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const uint32_t g = Gm::g_of(r_store, tau, k);
        // A: raw centred intermediate (plain stores: the lines stay in this XCD's L2); B: canonical outputs
        const uint64_t o = COLS ? A::to_raw(ar.reduce(x[k])) : ar.canon(x[k]);
        const uint32_t e = COLS ? (g << 8) | gl : gl * 256 + g;   // element offset from base
        if constexpr (!STORE) asm volatile("" ::"v"(o));        // timing probe
        else if constexpr (COLS)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o), rs,
                                                  (int)(e * 8u), 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o), rs,
                                                  (int)(e * 8u), 0, MFHE_XL2_OUT_CPOL);
    }
}

template <uint32_t M, uint32_t LAM, int LOG_R>
__global__ __launch_bounds__(Xl2G<LOG_R>::NT, MFHE_XL2_WPC * Xl2G<LOG_R>::NT / 256) void ntt16_xl2_kernel(Xl2Args a) {
    using C = ColDb;
    using G = Xl2G<LOG_R>;
    constexpr int NT = G::NT, NW = NT / 64, R = G::R, NR = G::NR, TWR = G::TWR, NDMA = 2048 / NT;
    constexpr uint32_t TPB = 16 * M;
    constexpr uint32_t kSpin = 1u << 20;   // ~1-2 s of polling (a poll is an L2/fabric round trip, 1-2 us)
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];   // two tile buffers of C::BUF words
    __shared__ uint32_t s_ctl[8];
    __shared__ uint32_t s_poll[2];   // LDS-DMA target of the asynchronous readiness poll (lane 0)
    typedef __attribute__((address_space(3))) void* lds_vp;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t x = xl2_xcc();
    uint32_t* const done = a.st + kXl2Done + x * a.cmax;
    uint32_t* const tmo = a.st + kXl2Tmo;

    // lane 0: bounded spin (a timeout is sticky and ends every spin)
    auto spin_until = [&](auto&& cond) {
        for (uint32_t n = 0; !cond(); ++n) {
            __builtin_amdgcn_s_sleep(1);
            if (n > kSpin || xl2_ld(tmo)) {
                __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        }
    };
    // lane 0, asynchronous: done[c] -> s_poll[slot] by a one-dword LDS-DMA (sc1), so no VGPR holds an in-flight
    // result (a register the compiler believes valid could be copied before the load returns); read after a counted
    // wait that covers it
    auto async_poll = [&](uint32_t c, int slot) {
        __builtin_amdgcn_global_load_lds((const void*)(done + c), (lds_vp)(s_poll + slot), 4, 0, 16);
    };

    // ---- start: register this XCD, wait for the grid; dense XCD ranks; this workgroup's rank inside its XCD ----
    // Tasks are dealt round-robin inside an XCD: the workgroup of rank rho among the XCD's nwg workgroups takes task
    // ids rho, rho + nwg, rho + 2 nwg, ... (no dequeue atomics; every workgroup is resident after the start)
    if (t == 0) {
        const uint32_t r = xl2_add(a.st + kXl2Reg + x, 1u);
        asm volatile("" ::"v"(r));   // the registration is performed before the arrival is counted
        xl2_add(a.st + kXl2Arr, 1u);
        spin_until([&] { return xl2_ld(a.st + kXl2Arr) >= gridDim.x; });
        uint32_t nx = 0, rank = 0;
        for (uint32_t y = 0; y < 16; ++y) {
            const bool here = xl2_ld(a.st + kXl2Reg + y) != 0;
            nx += here;
            rank += here && y < x;
        }
        const uint32_t nc = a.nchunk > rank ? (a.nchunk - rank + nx - 1) / nx : 0;   // chunks g = c nx + rank
        s_ctl[0] = nx;
        s_ctl[1] = rank;
        s_ctl[2] = nc;
        s_ctl[3] = r;                                   // this workgroup's rank in its XCD
        s_ctl[4] = xl2_ld(a.st + kXl2Reg + x);          // workgroups of its XCD
    }
    __syncthreads();
    const uint32_t nx = s_ctl[0], xrank = s_ctl[1], nc = s_ctl[2], nwg = s_ctl[4];
    const uint32_t ntask = 2 * nc * TPB;
    uint32_t cur = s_ctl[3], nxt = cur + nwg;
    if (cur >= ntask || nc > a.cmax) return;

    struct Loc {
        uint64_t* pb;   // polynomial base
        int mod;
        bool live;      // the polynomial exists
    };
    auto locate = [&](const Xl2Task& k) {
        Loc L{nullptr, 0, false};
        const uint64_t v = ((uint64_t)k.c * nx + xrank) * M + k.tile / 16;   // limb-major virtual polynomial index
        if (v < a.npoly) {
            const uint32_t l = (uint32_t)(v / a.batch), b = (uint32_t)(v - (uint64_t)l * a.batch);
            L.pb = a.data + (((uint64_t)b * a.nl + l) << 16);
            L.mod = (int)(a.start_limb + l);
            L.live = true;
        }
        return L;
    };
    // One tile -> buf by LDS-DMA: exactly NDMA global_load_lds_dwordx4 per thread whatever the task, so the compiler's
    // vmcnt bookkeeping stays exact on every path.  A: 16 columns x 256 rows -> [256][16] (the column pass's DMA);
    // B: 16 contiguous rows of 256 -> [16][256]; none: 1 KiB of the table's start (16 B per lane) into buf, which the
    // next real DMA overwrites.  All with sc1: for the B tiles it is the hand-off's consumer load (bypasses
    // this CU's L1); for A tiles it costs nothing measurable (HBM reads).
    auto dma = [&](const Xl2Task& k, const Loc& L, bool real, uint64_t* buf) {
        // branch-free source selection (a select per address, no exec-masked branches around the DMAs)
        const uint32_t sub = k.tile % 16;
        const uint64_t ma = 0 - (uint64_t)(real && k.a), mb = 0 - (uint64_t)(real && !k.a);
        const uint64_t pbase = (uint64_t)L.pb & (ma | mb);
        // dummy source: 1 KiB at the table's start, 16 B per lane (spread over 8 lines: every lane reading one word
        // would make all CUs hammer one L2 line)
        const uint64_t dummy = ((uint64_t)a.tw + lane * 16) & ~(ma | mb);
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
            const uint32_t q = (i * NW + w) * 64 + lane;   // 16-B chunk of the tile
            const uint64_t offa = (uint64_t)sub * 128 + (uint64_t)(q >> 3) * 2048 + (q & 7) * 16;
            const uint64_t offb = (uint64_t)sub * 32768 + (uint64_t)q * 16;
            const uint64_t src = pbase + (offa & ma) + (offb & mb) + dummy;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)((char*)buf + (size_t)(i * NW + w) * 1024), 16,
                                             0, 16);
        }
    };
    // The next tile's twiddles (B: its 16 rows' stage-8..15 segments of the table, 4080 doubles, DMA'd next to its
    // data; A / none: a dummy source, so the per-thread DMA count never depends on the task) -- by LDS-DMA like the
    // data: no VGPR ever holds an in-flight load result.  (Twiddles loaded by inline asm into registers were copied
    // to AGPRs by the compiler before they had landed.)
    constexpr int kTwChunks = 2048;   // 16-B chunks of the twiddle area (4096 doubles, 4080 used)
    auto twdma = [&](const Xl2Task& k, const Loc& L, bool real, uint64_t* twbuf) {
        const bool bt = real && !k.a;
        const uint64_t mb = 0 - (uint64_t)bt;
        const double* tt = a.tw + ((size_t)(bt ? L.mod : 0) << 16);
        const uint32_t r0 = (k.tile % 16) * 16;
        const uint64_t dummy = ((uint64_t)a.tw + lane * 16) & ~mb;   // (spread, as in dma())
#pragma unroll
        for (int i = 0; i < kTwChunks / NT; ++i) {
            const uint32_t q0 = (i * NW + w) * 64 + lane, q = q0 < 2040 ? q0 : 2039;
            const uint32_t e = 31 - __builtin_clz(q / 8 + 1);       // stage 8 + e: doubles [16 (2^e - 1), 16 (2^(e+1) - 1))
            const uint32_t d = 2 * q - 16 * ((1u << e) - 1);        // offset inside the stage's segment
            const uint64_t src = ((uint64_t)(tt + (256u << e) + (r0 << e) + d) & mb) + dummy;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)((char*)twbuf + (size_t)(i * NW + w) * 1024), 16,
                                             0, 0);
        }
    };
    auto issue = [&](const Xl2Task& k, const Loc& L, bool real, uint64_t* slot) {
        twdma(k, L, real, slot + C::BUF);
        dma(k, L, real, slot);
    };
    const uint32_t glb = t / G::TG, taub = t % G::TG;   // block lanes: row, position
    constexpr size_t SLOT = (size_t)C::BUF + 2 * kTwChunks;   // u64 words per slot: tile buffer + twiddle area

    // ---- first task (lane 0 may wait here: this workgroup holds nothing yet) ----
    Xl2Task kc = xl2_decode<M, LAM>(cur, nc);
    if (t == 0 && !kc.a) spin_until([&] { return xl2_ld(done + kc.c) >= TPB; });
    lds_barrier();
    Loc Lc = locate(kc);
    issue(kc, Lc, Lc.live, lds);
    uint32_t cb = 0;

    // lane 0's control state
    int64_t sig_a = -1, sig_b = -1;   // chunks of the A tasks stored one and two iterations ago (unsignalled)
    int ps = 0;                       // s_poll slot of nxt's readiness poll
    if (t == 0) {
        const Xl2Task k1 = xl2_decode<M, LAM>(nxt, nc);
        async_poll(nxt < ntask && !k1.a ? k1.c : 0, ps);
    }

    int tmod = -1;
    LimbConst lc{};
    double twa[NR][TWR];                           // the limb's column-stage twiddles (A tiles)
    const uint32_t gla = t % 16, taua = t / 16;   // column lanes: column, position

    bool first = true;
    while (true) {
        // this tile's DMA and twiddles, lane 0's async results, and the stores of two iterations ago are complete;
        // the R stores of the previous iteration may still be in flight
        if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R) : "memory");
        first = false;
        lds_barrier();   // ... for every wave: the A task stored two iterations ago is complete everywhere
        // ---- control (lane 0): signal, decide on nxt from the async poll, issue the next async ops ----
        if (t == 0) {
            if (sig_b >= 0) xl2_add(done + sig_b, 1u);
            sig_b = sig_a;
            sig_a = -1;
            const Xl2Task k1 = xl2_decode<M, LAM>(nxt, nc);
            const uint32_t poll = s_poll[ps];   // (landed: covered by the counted wait above)
            const uint32_t ready = nxt >= ntask ? 2u : (k1.a || poll >= TPB) ? 1u : 0u;   // 2: no next task
            s_ctl[5] = ready;
            const uint32_t nn = nxt + nwg;   // the task after nxt: its readiness poll, landing by the next top
            const Xl2Task k2 = xl2_decode<M, LAM>(nn, nc);
            ps ^= 1;
            async_poll(nn < ntask && !k2.a ? k2.c : 0, ps);
        }
        lds_barrier();
        const uint32_t ready = s_ctl[5];
        const uint32_t nn_id = nxt + nwg;
        const Xl2Task kn = xl2_decode<M, LAM>(nxt < ntask ? nxt : 0, nc);
        const Loc Ln = nxt < ntask ? locate(kn) : Loc{nullptr, 0, false};
        uint64_t* const nbuf = lds + (size_t)(cb ^ 1) * SLOT;
        uint64_t* const buf = lds + (size_t)cb * SLOT;

        if (Lc.live && Lc.mod != tmod) {   // limb constants and the column twiddles (rare: limb-major order)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            tmod = __builtin_amdgcn_readfirstlane(Lc.mod);   // uniform: scalar loads for the constants
            const __attribute__((address_space(4))) LimbConst* cl =
                (const __attribute__((address_space(4))) LimbConst*)a.limbs + tmod;
            lc.q = cl->q;
            lc.qf = cl->qf;
            lc.qinv = cl->qinv;
            xl2_twiddles<LOG_R, true>(a.tw + ((size_t)tmod << 16), 0, taua, twa);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int j = 0; j < TWR; ++j) asm volatile("" : "+v"(twa[r][j]));   // no load left pending in them
        }
        issue(kn, Ln, ready == 1 && Ln.live && MFHE_XL2_PROBE < 2, nbuf);
        if (Lc.live) {
            constexpr bool ST = MFHE_XL2_PROBE == 0;
            const uint32_t sub = kc.tile % 16;
            if (kc.a) xl2_tile<LOG_R, true, ST>(buf, gla, taua, lc, twa, Lc.pb + sub * 16);
            else {
                double wc[NR][TWR];
                xl2_btw_lds<LOG_R>((const double*)(buf + C::BUF), glb, taub, wc);
                xl2_tile<LOG_R, false, ST>(buf, glb, taub, lc, wc, Lc.pb + (size_t)sub * 4096);
            }
        } else {   // a tile past the batch: keep the per-iteration store count (R) with stores to the state's
                   // scratch line, so the counted waits stay exact
            uint32_t* const scratch = a.st + kXl2Tmo - 2 - (t & 1);
#pragma unroll
            for (int k = 0; k < R; ++k) asm volatile("global_store_dword %0, %1, off" ::"v"(scratch), "v"(0u) : "memory");
        }
        if (t == 0 && kc.a) sig_a = kc.c;   // also for a tile past the batch: its chunk's count must complete
        if (ready == 2) break;
        if (ready == 0) {   // nxt's chunk is not complete: drain, signal everything stored, then wait for it
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();
            if (t == 0) {
                if (sig_b >= 0) xl2_add(done + sig_b, 1u);
                if (sig_a >= 0) xl2_add(done + sig_a, 1u);
                sig_a = sig_b = -1;
                spin_until([&] { return xl2_ld(done + kn.c) >= TPB; });
            }
            lds_barrier();
            issue(kn, Ln, Ln.live && MFHE_XL2_PROBE < 2, nbuf);
            first = true;   // no stores after this DMA: the next top wait is vmcnt(0)
        }
        cur = nxt;
        nxt = nn_id;
        kc = kn;
        Lc = Ln;
        cb ^= 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (t == 0) {
        if (sig_b >= 0) xl2_add(done + sig_b, 1u);
        if (sig_a >= 0) xl2_add(done + sig_a, 1u);
    }
}

}  // namespace mfhe
