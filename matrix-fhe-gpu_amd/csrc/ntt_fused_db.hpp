// ntt_fused_db.hpp -- forward N = 2^16 NTT, both passes in one launch with the intermediate handed over in the
// XCD's L2 (ntt_fused.hpp's task queues), and the next pass-1 tile's LDS-DMA in flight while the current task
// computes (ntt_coldb.hpp's double buffer).  MFHE_OPT_NTT_FUSED = 2.
//
// Why: the two-pass plan crosses the L2 <-> fabric boundary 32N bytes per transform; the r02 fused kernel cut
// that to 24.6N but ran latency-bound at 2 workgroups per CU (each task: load -> compute -> store, nothing in
// flight while it computes; profiles/r02_pmc_fused_vs_twopass.json).  Here every workgroup has two 32 KiB LDS
// tile buffers: while task c computes in one, the next task's pass-1 tile (the HBM reads, the long-latency
// ones) lands in the other.
//
// Tasks (per XCD queue, as ntt_fused.hpp): block k = t / 2K, u = t % 2K; u < K: column tile u of local poly k
// (16 columns x 256 rows, DMA'd from the input); u >= K: block tile u - K of local poly k - D (16 rows x 256
// contiguous, read from the intermediate with sc1 loads into registers, after its K arrivals).  A workgroup
// holds its current task c and the next task n, and dequeues the one after n during c.
//
// One wait per task.  An iteration issues, in this order: the dequeue atomic (wave 0), the current task's loads
// (pass 2: data + twiddles into registers; pass 1 on a new limb: its 2 KiB twiddle table by LDS-DMA), then
// exactly 8 LDS-DMA instructions -- the next task's pass-1 tile, or, when the next task is not a pass-1 task, a
// dummy copy of 32 KiB of the (L2-resident) twiddle table into the idle buffer -- then s_waitcnt vmcnt(8): all but
// those 8 have completed (vmcnt is in order), i.e. the current tile, its loads, the dequeue and the previous
// task's stores.  Keeping the 8 on every path makes the count the compiler's own as well, so it inserts no
// vmcnt(0) of its own that would wait for the prefetch.  The previous pass-1 tile's arrival is signalled right
// after that wait (its stores are complete); before an arrival spin the workgroup signals after vmcnt(0).  It
// never spins while holding an unsignalled tile, and spins only for tiles of smaller task numbers than its
// current one, so the progress argument of ntt_fused.hpp holds (the task after n is only dequeued, never
// started, while c waits).
//
// Visibility, placement and the drain of queues without workgroups: as ntt_fused.hpp (plain intermediate
// stores stay in the producer XCD's L2; pass-2 loads are sc1; outputs stored sc1 nt).  A workgroup whose XCC id
// the context's census did not see sets err bit 4 and takes no task (it can neither produce nor consume a
// hand-off in a queue's L2).
#pragma once
#include "ntt_coldb.hpp"
#include "ntt_fused.hpp"

namespace mfhe {

struct FusedDb {
    static constexpr int LOG_G = 8, LOG_R = 4, NG = 16, R = 16, TG = 16, NT = 256;
    using Gm = Geo<8, 4>;
    static constexpr int GS = Gm::GS;
    static constexpr int BUF = NG * GS;                                 // words per tile buffer (34,944 B)
    static constexpr int TWL = 256;   // pass-1 twiddle table: tw[0, 256) of the limb
    static constexpr size_t LDS_BYTES = 2 * (size_t)BUF * 8 + (size_t)TWL * 8 + 64;   // buffers, twiddles, words
    static constexpr uint32_t K = 16;                                   // tiles per polynomial and pass
    static_assert(ColDb::NG == 16 && ColDb::kDmaOps == 8, "pass-1 tiles are ColDb's 16-column tiles");
};

template <int kVariant>   // a template: instantiated only by the F64 forward translation unit
__global__ __launch_bounds__(FusedDb::NT, 2) void ntt_fused_db_kernel(FusedArgs<TwSrcF> f) {
    using A = ArithF64;
    using C = FusedDb;
    using Gm = C::Gm;
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    double* twl = reinterpret_cast<double*>(lds + 2 * C::BUF);   // C::TWL slots, one per thread
    uint32_t* bc = reinterpret_cast<uint32_t*>(lds + 2 * C::BUF + C::TWL);
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t gl1 = t % 16, tau1 = t / 16;   // pass 1: COLS lanes (column first)
    const uint32_t gl2 = t / 16, tau2 = t % 16;   // pass 2: block lanes (row first)
    const PassArgs<TwSrcF>& a = f.p;
    FusedSync* sy = f.sync;
    const uint32_t K = C::K, D = f.lag, Q = f.nq;
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    // outputs stored nt (streaming, write-back): the lines they overwrite hold this launch's intermediate, dirty in
    // the XCD's L2; an sc1 store (write-through, drops the line) over a dirty line is not used here
    constexpr int kCpolOut = 2;
    // per-limb constants through the constant address space: scalar loads (lgkmcnt), which neither count
    // against the vmcnt waits nor make the compiler wait on vmcnt before their first use
    typedef const __attribute__((address_space(4))) LimbConst* climb_t;
    const climb_t climbs = (climb_t)a.limbs;

    uint32_t q = f.qmap[xcc_id()];
    if (q >= Q) {   // an XCC the census did not see: no hand-off is safe here
        if (t == 0) atomicOr(&sy->err, 4u);
        q = kNone;
    }

    // pass-1 twiddles of limb lmod, cached across tiles in LDS: T = tw[0, 256) of the limb, DMA'd (2 KiB; every
    // column-pass twiddle is in it: tw0[j] = T[1 + j], tw1 of tau at (e, j) = T[((16 + tau) << e) + j])
    int lmod = -1;
    double q1 = 0.0, qi1 = 0.0;
    struct Tw0 {
        const double* T;
        __device__ __forceinline__ double operator[](int j) const { return T[1 + j]; }
    };
    struct Tw1 {
        const double* T;
        uint32_t tau;
        __device__ __forceinline__ double operator[](int i) const {   // i = 2^e - 1 + j, folded at compile time
            const int e = i >= 7 ? 3 : i >= 3 ? 2 : i >= 1 ? 1 : 0;
            return T[((16 + tau) << e) + (uint32_t)(i + 1 - (1 << e))];
        }
    };
    const Tw0 tw0{twl};
    const Tw1 tw1{twl, tau1};
    // the last pass-1 tile of this workgroup whose arrival is not signalled yet (queue-local poly index)
    uint32_t pend = kNone;
    uint32_t qcur = 0;
    auto signal = [&]() {
        if (pend != kNone && t == 0)
            __hip_atomic_fetch_add(&f.arr[(size_t)qcur * f.cap + pend], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend = kNone;
    };

    auto run_queue = [&](uint32_t qq) {
        qcur = qq;
        const uint32_t nloc = qq < f.npl ? (f.npl - qq + Q - 1) / Q : 0;
        const uint32_t total = (nloc + D) * 2 * K;
        // kind: 0 none, 1 pass 1, 2 pass 2; k = local poly
        auto kind_of = [&](uint32_t task, uint32_t& k, uint32_t& u) -> int {
            if (task >= total) return 0;
            const uint32_t blk = task / (2 * K);
            u = task % (2 * K);
            if (u < K) {
                k = blk;
                return blk < nloc ? 1 : 0;
            }
            u -= K;
            if (blk < D) return 0;
            k = blk - D;
            return 2;
        };
        auto loc1 = [&](uint32_t k, uint32_t u) {
            return tile_loc<8, 16, true, true>(a.data, a.batch, a.nl, a.start_limb, a.logN, 0, (k * Q + qq) * K + u, gl1);
        };
        auto loc2 = [&](uint32_t k, uint32_t u) {
            return tile_loc<8, 16, false, true>(a.data, a.batch, a.nl, a.start_limb, a.logN, 8, (k * Q + qq) * K + u, gl2);
        };

        if (t == 0) {
            bc[0] = __hip_atomic_fetch_add(&sy->head[qq][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bc[1] = __hip_atomic_fetch_add(&sy->head[qq][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        uint32_t c = __builtin_amdgcn_readfirstlane(bc[0]), n = __builtin_amdgcn_readfirstlane(bc[1]);
        int slot = 0;
        uint32_t kc = 0, uc = 0;
        int kc_kind = kind_of(c, kc, uc);
        if (kc_kind == 1) {
            const TileLoc L = loc1(kc, uc);
            coldb_dma((const char*)(L.base + (L.off0 - gl1)), (size_t)2048, lds, w, lane);
        }
        // The next task's pass-1 tile goes in flight.  Otherwise the same 8 DMA instructions copy 32 KiB of the
        // (L2-resident) twiddle table into the idle buffer, so every iteration issues exactly 8 vector-memory
        // operations here, and "s_waitcnt vmcnt(8)" right after -- issued on each branch separately, so the count
        // is also the compiler's own on straight-line code -- waits for everything but them.
        auto issue_next_and_wait = [&](int kn_kind, uint32_t kn, uint32_t un, uint64_t* nbuf) {
            const char* src = (const char*)a.tw.p;
            size_t rb = 128;
            if (kn_kind == 1) {
                const TileLoc Ln = loc1(kn, un);
                src = (const char*)(Ln.base + (Ln.off0 - gl1));
                rb = 2048;
            }
            coldb_dma(src, rb, nbuf, w, lane);
            vm_wait<8>();
        };
        while (c < total) {
            uint32_t nxt;   // written and read by thread 0 only
            if (t == 0) nxt = __hip_atomic_fetch_add(&sy->head[qq][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t kn = 0, un = 0;
            const int kn_kind = kind_of(n, kn, un);
            uint64_t* buf = lds + (size_t)slot * C::BUF;
            uint64_t* nbuf = lds + (size_t)(slot ^ 1) * C::BUF;
            // each kind is one straight-line block from its loads to its stores (no code shared after the
            // branch), so the compiler's own waits are exact counts and never a vmcnt(0) behind the prefetch
            if (kc_kind == 2) {
                // the K column tiles of poly kc: signal what this workgroup holds, then wait for all arrivals
                if (pend != kNone) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    lds_barrier();
                    signal();
                }
                if (t == 0) {
                    uint32_t spins = 0;
                    while (ld_agent(&f.arr[(size_t)qq * f.cap + kc]) < K) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++spins == kSpinLimit) { atomicOr(&sy->err, 2u); break; }
                    }
                }
                lds_barrier();
                const TileLoc Lc = loc2(kc, uc);
                double x[C::R], twa[15], twb[15];
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(Lc.base, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
                for (int k = 0; k < C::R; ++k)
                    x[k] = A::from_raw(__builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
                                                                      rs, (int)((Lc.off0 + k * 16 + tau2) * 8u), 0, 16)));
                // this row's twiddles: round 0 (shared by the row), round 1 (per thread)
                const double* tw = a.tw.p + ((size_t)Lc.mod << 16);
                const uint32_t hi = (uint32_t)Lc.hi;
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < (1 << e); ++j) {
                        twa[(1 << e) - 1 + j] = tw[(256u << e) + (hi << e) + j];
                        twb[(1 << e) - 1 + j] = tw[(4096u << e) + ((hi * 16 + tau2) << e) + j];
                    }
                // The compiler does not count LDS-DMA instructions in its own vmcnt scoreboard: a wait it inserts for
                // these loads after the DMA below would be vmcnt(0) and wait for the prefetch too.  So they are
                // waited for here, before the DMA, and re-defined by empty asm statements (the register values are
                // final; the compiler now sees no pending load).  Their L2 latency is exposed once per pass-2 task.
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int k = 0; k < C::R; ++k) asm volatile("" : "+v"(x[k]));
#pragma unroll
                for (int k = 0; k < 15; ++k) {
                    asm volatile("" : "+v"(twa[k]));
                    asm volatile("" : "+v"(twb[k]));
                }
                issue_next_and_wait(kn_kind, kn, un, nbuf);
                const A ar(LimbConst{0, climbs[Lc.mod].qf, climbs[Lc.mod].qinv, 0});
                uint64_t* my = buf + (size_t)gl2 * C::GS;
                static_for<0, 4>([&](auto bi) {
                    constexpr int bb = 3 - decltype(bi)::value, e = 3 - bb, half = 1 << bb;
#pragma unroll
                    for (int k = 0; k < C::R; ++k) {
                        if (k & half) continue;
                        ar.ct(x[k], x[k + half], twa[(1 << e) - 1 + (k >> (bb + 1))]);
                    }
                });
                lds_barrier();   // every thread is past the previous task's use of buf
#pragma unroll
                for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(0, tau2, k))] = A::to_raw(x[k]);
                lds_barrier();
#pragma unroll
                for (int k = 0; k < C::R; ++k) x[k] = ar.round_reduce(A::from_raw(my[Gm::pad(Gm::g_of(1, tau2, k))]));
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
                for (int k = 0; k < C::R; ++k) my[Gm::pad(Gm::g_of(1, tau2, k))] = A::to_raw(x[k]);
                lds_barrier();
#pragma unroll
                for (int k = 0; k < C::R; ++k) x[k] = A::from_raw(my[Gm::pad(Gm::g_of(0, tau2, k))]);
#pragma unroll
                for (int k = 0; k < C::R; ++k)
                    __builtin_amdgcn_raw_buffer_store_b64(
                        __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, ar.canon(x[k])), rs,
                        (int)((Lc.off0 + k * 16 + tau2) * 8u), 0, kCpolOut);
            } else if (kc_kind == 1) {
                const TileLoc Lc = loc1(kc, uc);
                if (Lc.mod != lmod) {
                    lmod = Lc.mod;
                    q1 = climbs[lmod].qf;
                    qi1 = climbs[lmod].qinv;
                    // the limb's tw[0, 256): two 1 KiB LDS-DMA instructions (waves 0 and 1), no VGPR destination
                    if (w < 2) {
                        typedef __attribute__((address_space(3))) void* lds_vp;
                        const double* tw = a.tw.p + ((size_t)lmod << 16);
                        __builtin_amdgcn_global_load_lds((const void*)(tw + w * 128 + lane * 2), (lds_vp)(twl + w * 128),
                                                         16, 0, 0);
                    }
                }
                issue_next_and_wait(kn_kind, kn, un, nbuf);
                lds_barrier();   // the tile (and table) landed for every thread
                signal();        // the previous pass-1 tile's stores were older than the 8 DMAs: complete
                coldb_tile<A>(buf, gl1, tau1, LimbConst{0, q1, qi1, 0}, tw0, tw1, Lc.base, Lc.off0, 8);
                pend = kc;
            } else {
                issue_next_and_wait(kn_kind, kn, un, nbuf);
            }
            // the dequeued task number is consumed only here, after this task's stores: the compiler's wait for the
            // atomic's return then covers the prefetch (long landed) and those stores, never the butterflies
            if (t == 0) bc[2] = nxt;
            lds_barrier();   // bc[2] published; every thread is done with buf (the next DMA goes there)
            const uint32_t nn = __builtin_amdgcn_readfirstlane(bc[2]);
            c = n;
            n = nn;
            kc = kn;
            uc = un;
            kc_kind = kn_kind;
            slot ^= 1;
        }
        // the last (dummy) DMA and the last stores, then the last arrival
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        signal();
    };

    if (q != kNone) run_queue(q);
    // leave; the last workgroup out drains every queue that still has tasks (an XCD with no workgroup)
    __syncthreads();
    if (t == 0) bc[3] = __hip_atomic_fetch_add(&sy->exits, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane(bc[3]) != gridDim.x - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (uint32_t qq = 0; qq < Q; ++qq) {
        lmod = -1;
        run_queue(qq);
    }
}

}  // namespace mfhe
