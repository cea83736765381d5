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
// Queues.  A workgroup reads its XCD from HW_REG_XCC_ID and only takes tasks from that XCD's queue (one returning
// atomic per task on the XCD's head word), so producer and consumer of every intermediate tile run on the same XCD
// by construction -- placement is read at run time, never assumed.  At the start every workgroup registers its XCD
// and waits (bounded) until the whole grid has (one grid-wide arrival, a few µs per 2.5 ms launch): the NX XCDs
// present get dense ranks, and XCD rank r owns the global mini-chunks g = c NX + r, c = 0, 1, ... (M = MFHE_XL2_M
// polynomials each, limb-major), whatever the device's XCD count and ids.  An XCD's task sequence is blocks of 16 M
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
// Pipeline.  Per iteration every thread issues the next tile's B twiddles and LDS-DMA (one tile always landing
// while another is transformed, two 34.9 KiB buffers), then transforms and stores the current tile.  The top of the
// next iteration waits with a counted vmcnt(16): the DMA and twiddles are complete, the 16 stores just issued may
// stay in flight -- they are known complete one iteration later, which is when an A task is signalled.  The
// control (lane 0: dequeue, the B-readiness poll) is issued by inline asm one iteration ahead, so the compiler adds
// no wait for it and its results are covered by that same counted wait.  A next B tile whose chunk is not yet
// complete is not prefetched: the workgroup drains, signals everything it stored, then polls (bounded) -- so no
// workgroup ever waits while it holds an unsignalled A task, and every wait is for tasks earlier in its XCD's
// sequence: the earliest waited-on task is always runnable (no deadlock for any residency after the start).  Every
// spin is bounded; a timeout sets a sticky word and ends the spins (results are then wrong, never a hang;
// MFHE_OPT_NTT_XL2_TIMEOUT reads it).
//
// Arithmetic.  A tasks run coldb_tile (the column pass's tile code, bit-identical intermediate); B tasks the block
// pass's stages 8..15 on 16 rows (NttPass's schedule and reductions: same outputs, bit for bit).
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

// state layout (u32 words): head of XCC x at 32 x (x < 16); the grid arrival counter; the timeout word; the XCD
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

// one B tile (16 rows of 256) whose raw intermediate has landed in buf ([16][256] row-major): stages 8..15 (the
// block pass: round 0 = stages 8..11, exchange, round 1 = 12..15, exchange back), canonical outputs stored with
// MFHE_XL2_OUT_CPOL.  Exchanges in buf itself (padded groups of GS words), LDS-only barriers.  tw: the limb's
// table; the 30 twiddles this thread needs are loaded first (before the caller issues the next DMA).
struct Xl2B {
    static constexpr int R = 16, TG = 16, GS = ColDb::GS;
    using Gm = Geo<8, 4>;
};
// By inline asm: the compiler sees no load, so it never waits for these registers itself (a compiler wait here would
// be a vmcnt(0): it cannot count through the kernel's loop, and that would also wait for the stores and the DMA in
// flight).  Valid after a counted s_waitcnt that covers them (ntt16_xl2_kernel's loop top).
__device__ __forceinline__ void xl2_ld_f64(double& v, const double* p) {
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
}
__device__ __forceinline__ void xl2_btwiddles(const double* tw, uint32_t row, uint32_t tau, double (&w0)[15],
                                              double (&w1)[15]) {
    // round 0: bit = 4 + bb (bb = 3..0), s = 15 - bit, index 2^s + (row << (7 - bit)) + (k >> (bb + 1))
#pragma unroll
    for (int e = 0; e < 4; ++e) {   // e = 3 - bb: stage s = 8 + e, 2^e twiddles
#pragma unroll
        for (int m = 0; m < (1 << e); ++m) xl2_ld_f64(w0[(1 << e) - 1 + m], tw + (256u << e) + (row << e) + m);
    }
    // round 1: bit = bb, s = 15 - bb, index 2^s + (row << (7 - bb)) + (tau << (3 - bb)) + (k >> (bb + 1))
#pragma unroll
    for (int e = 0; e < 4; ++e) {   // e = 3 - bb: stage s = 12 + e
#pragma unroll
        for (int m = 0; m < (1 << e); ++m)
            xl2_ld_f64(w1[(1 << e) - 1 + m], tw + (4096u << e) + (row << (4 + e)) + (tau << e) + m);
    }
}

template <bool STORE = true>
__device__ __forceinline__ void xl2_btile(uint64_t* buf, uint32_t gl, uint32_t tau, const LimbConst& lc,
                                          const double (&w0)[15], const double (&w1)[15], uint64_t* rowbase) {
    using Gm = Xl2B::Gm;
    using A = ArithF64;
    const A ar(lc);
    double x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = A::from_raw(buf[gl * 256 + k * 16 + tau]);   // g_of(0, tau, k) = 16 k + tau
    // round 0: stages 8..11 on register bits 3..0 (element bits 7..4)
    static_for<0, 4>([&](auto bi) {
        constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k & half) continue;
            ar.ct(x[k], x[k + half], w0[(1 << e) - 1 + (k >> (bb + 1))]);
        }
    });
    uint64_t* my = buf + (size_t)gl * Xl2B::GS;
    lds_barrier();   // every thread has read its raw words out of buf
#pragma unroll
    for (int k = 0; k < 16; ++k) my[Gm::pad(k * 16 + tau)] = A::to_raw(x[k]);
    lds_barrier();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = ar.round_reduce(A::from_raw(my[Gm::pad(tau * 16 + k)]));   // g_of(1, tau, k)
    // round 1: stages 12..15 on register bits 3..0 (element bits 3..0)
    static_for<0, 4>([&](auto bi) {
        constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (k & half) continue;
            ar.ct(x[k], x[k + half], w1[(1 << e) - 1 + (k >> (bb + 1))]);
        }
    });
    // back to the round-0 layout for coalesced stores (the block pass's final exchange)
    lds_barrier();
#pragma unroll
    for (int k = 0; k < 16; ++k) my[Gm::pad(tau * 16 + k)] = A::to_raw(x[k]);
    lds_barrier();
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = A::from_raw(my[Gm::pad(k * 16 + tau)]);
    const uint64_t bu = (uint64_t)rowbase;
    uint64_t* const ub = (uint64_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bu >> 32)) << 32) |
                                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bu));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ub, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t o = ar.canon(x[k]);
        if constexpr (STORE)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, o), rs,
                                                  (int)((gl * 256 + k * 16 + tau) * 8u), 0, MFHE_XL2_OUT_CPOL);
        else   // timing probe: keep the result live without a store
            asm volatile("" ::"v"(o));
    }
}

template <uint32_t M, uint32_t LAM>
__global__ __launch_bounds__(256, MFHE_XL2_WPC) void ntt16_xl2_kernel(Xl2Args a) {
    using C = ColDb;
    constexpr uint32_t TPB = 16 * M;
    constexpr uint32_t kSpin = 1u << 24;   // ~1 s of polling at ~60 ns per poll
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];   // two tile buffers of C::BUF words
    __shared__ uint32_t s_ctl[8];
    typedef __attribute__((address_space(3))) void* lds_vp;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t x = xl2_xcc();
    uint32_t* const head = a.st + x * 32;
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
    // lane 0, asynchronous (the compiler sees no memory operation, so it inserts no wait for them): the result
    // register is valid after the next counted wait that covers the instruction
    auto async_add = [&](uint32_t* p) {
        uint32_t r;
        asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(r) : "v"(p), "v"(1u) : "memory");
        return r;
    };
    auto async_ld = [&](uint32_t* p) {
        uint32_t r;
        asm volatile("global_load_dword %0, %1, off sc1" : "=v"(r) : "v"(p) : "memory");
        return r;
    };

    // ---- start: register this XCD, wait for the grid, dense XCD rank ----
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
        s_ctl[3] = xl2_add(head, 1u);
        s_ctl[4] = xl2_add(head, 1u);
    }
    __syncthreads();
    const uint32_t nx = s_ctl[0], xrank = s_ctl[1], nc = s_ctl[2];
    const uint32_t ntask = 2 * nc * TPB;
    uint32_t cur = s_ctl[3], nxt = s_ctl[4];
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
    // One tile -> buf by LDS-DMA: exactly 8 global_load_lds_dwordx4 per thread whatever the task, so the compiler's
    // vmcnt bookkeeping stays exact on every path.  A: 16 columns x 256 rows -> [256][16] (the column pass's DMA);
    // B: 16 contiguous rows of 256 -> [16][256]; none: every lane re-reads one 16-B state word (one line) into buf,
    // which the next real DMA overwrites.  All with sc1: for the B tiles it is the hand-off's consumer load (bypasses
    // this CU's L1); for A tiles it costs nothing measurable (HBM reads).
    auto dma = [&](const Xl2Task& k, const Loc& L, bool real, uint64_t* buf) {
        // branch-free source selection (a select per address, no exec-masked branches around the DMAs)
        const uint32_t sub = k.tile % 16;
        const uint64_t ma = 0 - (uint64_t)(real && k.a), mb = 0 - (uint64_t)(real && !k.a);
        const uint64_t pbase = (uint64_t)L.pb & (ma | mb);
        const uint64_t dummy = (uint64_t)(a.st + kXl2Tmo - 1) & ~(ma | mb);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t q = (i * 4 + w) * 64 + lane;   // 16-B chunk of the tile
            const uint64_t offa = (uint64_t)sub * 128 + (uint64_t)(q >> 3) * 2048 + (q & 7) * 16;
            const uint64_t offb = (uint64_t)sub * 32768 + (uint64_t)q * 16;
            const uint64_t src = pbase + (offa & ma) + (offb & mb) + dummy;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_vp)((char*)buf + (size_t)(i * 4 + w) * 1024), 16,
                                             0, 16);
        }
    };
    // The next tile's loads: its 30 B-stage twiddles into wn0 / wn1 (loop-carried registers, loaded by inline asm;
    // an A or absent tile loads 30 copies of the table's first line instead, so the count never depends on the task)
    // and its DMA.  The counted wait at the top of the next iteration covers them.
    const uint32_t glb = t / 16, taub = t % 16;   // block lanes
    double wn0[15], wn1[15];
    auto issue = [&](const Xl2Task& k, const Loc& L, bool real, uint64_t* buf) {
        const bool bt = real && !k.a;
        const double* tt = a.tw + ((size_t)(bt ? L.mod : 0) << 16);
        const uint32_t row = bt ? (k.tile % 16) * 16 + glb : 0, tau = bt ? taub : 0;
        xl2_btwiddles(tt, row, tau, wn0, wn1);
        dma(k, L, real, buf);
    };

    // ---- first task (lane 0 may wait here: this workgroup holds nothing yet) ----
    Xl2Task kc = xl2_decode<M, LAM>(cur, nc);
    if (t == 0 && !kc.a) spin_until([&] { return xl2_ld(done + kc.c) >= TPB; });
    lds_barrier();
    Loc Lc = locate(kc);
    issue(kc, Lc, Lc.live, lds);
    uint32_t cb = 0;

    // lane 0's control state
    uint32_t nn = 0, poll = 0;   // async results: the task after nxt; done[] of nxt's chunk (B)
    int64_t sig_a = -1, sig_b = -1;   // chunks of the A tasks stored one and two iterations ago (unsignalled)
    if (t == 0) {
        nn = async_add(head);
        const Xl2Task k1 = xl2_decode<M, LAM>(nxt, nc);
        poll = async_ld(done + (nxt < ntask && !k1.a ? k1.c : 0));
    }

    int tmod = -1;
    LimbConst lc{};
    double tw0[15], tw1[15];
    const uint32_t gla = t % 16, taua = t / 16;   // column lanes
    double wc0[15], wc1[15];                       // the current B tile's twiddles

    bool first = true;
    while (true) {
        // this tile's DMA and twiddles, lane 0's async results, and the stores of two iterations ago are complete;
        // the 16 stores of the previous iteration may still be in flight
        if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        first = false;
#pragma unroll
        for (int j = 0; j < 15; ++j) {   // (asm-loaded: no compiler wait)
            wc0[j] = wn0[j];
            wc1[j] = wn1[j];
        }
        lds_barrier();   // ... for every wave: the A task stored two iterations ago is complete everywhere
        // ---- control (lane 0): signal, decide on nxt from the async poll, issue the next async ops ----
        if (t == 0) {
            asm volatile("" : "+v"(nn), "+v"(poll));   // (valid: covered by the counted wait above)
            if (sig_b >= 0) xl2_add(done + sig_b, 1u);
            sig_b = sig_a;
            sig_a = -1;
            const Xl2Task k1 = xl2_decode<M, LAM>(nxt, nc);
            const uint32_t ready = nxt >= ntask ? 2u : (k1.a || poll >= TPB) ? 1u : 0u;   // 2: no next task
            s_ctl[5] = ready;
            s_ctl[6] = nn;
            const uint32_t nn2 = nn;
            nn = async_add(head);   // the task after nn
            const Xl2Task k2 = xl2_decode<M, LAM>(nn2, nc);
            poll = async_ld(done + (nn2 < ntask && !k2.a ? k2.c : 0));
        }
        lds_barrier();
        const uint32_t ready = s_ctl[5];
        const uint32_t nn_id = s_ctl[6];
        const Xl2Task kn = xl2_decode<M, LAM>(nxt < ntask ? nxt : 0, nc);
        const Loc Ln = nxt < ntask ? locate(kn) : Loc{nullptr, 0, false};
        uint64_t* const nbuf = lds + (size_t)(cb ^ 1) * C::BUF;
        uint64_t* const buf = lds + (size_t)cb * C::BUF;

        if (Lc.live && Lc.mod != tmod) {   // limb constants and the column twiddles (rare: limb-major order)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            tmod = __builtin_amdgcn_readfirstlane(Lc.mod);   // uniform: scalar loads for tw0 and the constants
            const __attribute__((address_space(4))) LimbConst* cl =
                (const __attribute__((address_space(4))) LimbConst*)a.limbs + tmod;
            lc.q = cl->q;
            lc.qf = cl->qf;
            lc.qinv = cl->qinv;
            coldb_twiddles(a.tw + ((size_t)tmod << 16), taua, tw0, tw1);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 0; j < 15; ++j) {   // no load left pending in them
                asm volatile("" : "+v"(tw1[j]));
                asm volatile("" : "+v"(tw0[j]));
            }
        }
        issue(kn, Ln, ready == 1 && Ln.live && MFHE_XL2_PROBE < 2, nbuf);
        if (Lc.live) {
            constexpr bool ST = MFHE_XL2_PROBE == 0;
            if (kc.a) coldb_tile<ArithF64, ST>(buf, gla, taua, lc, tw0, tw1, Lc.pb, (kc.tile % 16) * 16 + gla, 8, [] {});
            else xl2_btile<ST>(buf, glb, taub, lc, wc0, wc1, Lc.pb + (size_t)(kc.tile % 16) * 4096);
        } else {   // a tile past the batch: keep the per-iteration store count (16) with stores to the state's
                   // scratch line, so the counted waits stay exact
            uint32_t* const scratch = a.st + kXl2Tmo - 2 - (t & 1);
#pragma unroll
            for (int k = 0; k < 16; ++k) asm volatile("global_store_dword %0, %1, off" ::"v"(scratch), "v"(0u) : "memory");
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
