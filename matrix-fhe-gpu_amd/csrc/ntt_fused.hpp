// ntt_fused.hpp -- both passes of a two-pass NTT (N = 2^15..2^17) in one launch, with the intermediate
// handed from pass 1 to pass 2 inside the XCD's L2.
//
// Why: the two-pass plan moves every element through the L2 <-> fabric path four times (read + write per
// pass; rocprofv3 FETCH/WRITE_SIZE = 2.01x the algorithmic bytes, profiles/r01_pmc_ntt_traffic.json), and
// that path, not the ALU, is what bounds it.  Here pass 2 of a polynomial re-reads the intermediate from
// the L2 of the XCD whose workgroups just wrote it, so the fabric sees 24N bytes per transform, not 32N.
//
// Scheduling.  One task queue per XCD (queue index from HW_REG_XCC_ID through the census map built at
// context creation).  Queue x owns the global polynomials g = j*Q + x (j = its local polynomial index), so
// no binding has to be published.  Task t of a queue: block k = t / 2K, u = t % 2K; u < K is pass-1 tile u
// of local poly k, u >= K is pass-2 tile u - K of local poly k - D (lag D).  A workgroup fetches the number
// of its NEXT task while it works on the current one, so the dequeue atomic is off the critical path.
//
// Forward progress does not depend on which workgroups are resident.  Pass-1 tasks never wait.  A pass-2
// task waits only for the K pass-1 tiles of its polynomial, all of which have smaller task numbers of the
// same queue.  By induction the smallest-numbered unfinished task is always being executed by the running
// workgroup that dequeued it (a workgroup's prefetched task has a larger number than its current one), so
// it finishes.  Only running workgroups dequeue.  Should an XCD get no workgroup at all, its queue is
// drained at the end by the last workgroup to leave (exit counter), which then runs both passes itself.
//
// Visibility.  Producer and consumer of a hand-off sit on the same XCD (the queue is chosen by XCC id, never
// by blockIdx), so that XCD's L2 is the coherence point.  Producer: plain stores (they keep the line in the
// L2) -> every wave s_waitcnt vmcnt(0) -> barrier -> lane 0 relaxed agent atomic add on the poly's arrival
// counter.  That signal is deferred until the workgroup's next tile has issued its loads, and it is always
// sent before the workgroup waits for anything, so the progress argument above still holds.  Consumer: lane 0 polls the counter (relaxed agent loads bypass L1) -> barrier -> every load of
// the intermediate is an sc1 load, served by the L2, so no stale L1 line of this CU can be returned.
// Final outputs are stored sc1 nt: they leave the L2 at once and do not evict intermediates.
#pragma once
#include "ntt_kernels.hpp"

#ifndef MFHE_FUSED_CPOL_IN
#define MFHE_FUSED_CPOL_IN 0        // pass-1 input loads
#endif
#ifndef MFHE_FUSED_CPOL_MID_LD
#define MFHE_FUSED_CPOL_MID_LD 16   // pass-2 intermediate loads: sc1 (L1 bypass) is required
#endif

namespace mfhe {

constexpr int kFusedXcc = 16;    // HW_REG_XCC_ID values 0..15

// Zeroed before every launch.
struct FusedSync {
    uint32_t head[kFusedXcc][32];   // one 128-B line per queue head
    uint32_t exits;                 // workgroups that left the main loop
    uint32_t err;                   // 2: an arrival wait timed out (a bug; the tile was skipped)
    uint32_t pad[30];
    // followed by uint32_t arr[kFusedXcc][cap]: pass-1 arrivals per local polynomial
};

template <class TS>
struct FusedArgs {
    PassArgs<TS> p;        // shared by pass 1 and pass 2 (forward: column then block; inverse: block then column)
    FusedSync* sync;
    uint32_t* arr;
    uint32_t cap;          // local polynomials per queue (entries of arr per queue)
    uint32_t K;            // tiles per polynomial in each pass
    uint32_t npl;          // polynomials (batch * nlimbs)
    uint32_t lag;          // D
    uint32_t nq;           // queues = XCDs found by the census
    uint8_t qmap[kFusedXcc];   // XCC id -> queue (0xFF: unseen id -> queue 0)
};

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x & (kFusedXcc - 1);
}

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint32_t kSpinLimit = 1u << 26;

// Census: which XCC ids exist (bit i of *mask set by a workgroup running on XCC i).
static __global__ void xcc_census_kernel(uint32_t* mask) {
    if (threadIdx.x == 0) atomicOr(mask, 1u << xcc_id());
}

template <class P1, class P2, class TS>
__global__ __launch_bounds__(P1::NT) void ntt_fused_kernel(FusedArgs<TS> f) {
    static_assert(P1::NT == P2::NT, "both passes must use the same workgroup size");
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    constexpr size_t LDSW = (P1::LDS_BYTES > P2::LDS_BYTES ? P1::LDS_BYTES : P2::LDS_BYTES) / 8;
    uint32_t* bc = reinterpret_cast<uint32_t*>(lds + LDSW);   // broadcast words
    const uint32_t t = threadIdx.x;
    FusedSync* sy = f.sync;
    const uint32_t K = f.K, D = f.lag, Q = f.nq;
    const P1 p1(f.p);
    const P2 p2(f.p);

    // Pass-1 arrival of local poly `p` (queue q): every wave's stores drained, then one counter add.  Deferred
    // to the next task's loads so no workgroup idles on its own store acknowledgements.
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    uint32_t pend = kNone;
    uint32_t q = 0;
    auto flush = [&](uint32_t p) {
        if (p == kNone) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) __hip_atomic_fetch_add(&f.arr[(size_t)q * f.cap + p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    q = f.qmap[xcc_id()];
    // an XCC the census did not see: its L2 is no queue's, so it can neither produce nor consume a hand-off.
    // It sets err bit 4 and takes no task (it still counts its exit, and may drain as the last one out).
    bool skip = false;
    if (q >= Q) {
        if (t == 0) atomicOr(&sy->err, 4u);
        skip = true;
        q = 0;
    }
    bool drain = false;   // last workgroup out: draining queues nobody ran
    while (true) {
        // local polys of queue q and its task count
        const uint32_t nloc = q < f.npl ? (f.npl - q + Q - 1) / Q : 0;
        const uint32_t total = (nloc + D) * 2 * K;
        if (t == 0 && !skip) bc[0] = __hip_atomic_fetch_add(&sy->head[q][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        uint32_t task = skip ? total : __builtin_amdgcn_readfirstlane(bc[0]);
        skip = false;
        while (task < total) {
            // prefetch the next task number; lane 0 publishes it at the end of this task
            uint32_t nxt = 0;
            if (t == 0) nxt = __hip_atomic_fetch_add(&sy->head[q][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t k = task / (2 * K), u = task % (2 * K);
            if (u < K) {
                if (k < nloc) {
                    const uint32_t g = k * Q + q;
                    const TileLoc L = p1.locate(g * K + u);
                    uint64_t raw[P1::R];
                    if constexpr (!P1::COL_DMA) p1.template load_pol<MFHE_FUSED_CPOL_IN>(L, raw);
                    flush(pend);   // the previous tile's stores drained behind this tile's loads
                    pend = k;
                    p1.compute_store(L, raw, lds);
                }
            } else if (k >= D) {
                const uint32_t j = k - D;
                flush(pend);   // never wait while holding an unsignalled tile
                pend = kNone;
                if (t == 0) {
                    uint32_t n = 0;
                    while (ld_agent(&f.arr[(size_t)q * f.cap + j]) < K) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++n == kSpinLimit) { atomicOr(&sy->err, 2u); break; }
                    }
                    bc[1] = n == kSpinLimit;
                }
                __syncthreads();
                if (!__builtin_amdgcn_readfirstlane(bc[1])) {
                    const uint32_t g = j * Q + q;
                    const TileLoc L = p2.locate(g * K + (u - K));
                    uint64_t raw[P2::R];
                    p2.template load_pol<MFHE_FUSED_CPOL_MID_LD>(L, raw);
                    p2.compute_store(L, raw, lds);
                }
            }
            __syncthreads();   // readers of bc[] (and of the LDS tile) are done
            if (t == 0) bc[0] = nxt;
            __syncthreads();
            task = __builtin_amdgcn_readfirstlane(bc[0]);
        }
        flush(pend);
        pend = kNone;
        if (drain) {
            if (++q >= Q) break;
            continue;
        }
        // leave; the last workgroup out drains every queue that still has tasks (an XCD with no workgroup)
        __syncthreads();
        if (t == 0) bc[2] = __hip_atomic_fetch_add(&sy->exits, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (__builtin_amdgcn_readfirstlane(bc[2]) != gridDim.x - 1) break;
        drain = true;
        q = 0;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
}

}  // namespace mfhe
