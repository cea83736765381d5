// ntt_fused.hpp -- both passes of a two-pass NTT (N = 2^15..2^17) in one launch, with the intermediate
// handed from pass 1 to pass 2 inside the XCD's L2.
//
// Why: the two-pass plan moves every element through the memory side four times (read + write per
// pass; rocprofv3 FETCH/WRITE_SIZE = 2.03x the algorithmic bytes, profiles/r01_pmc_ntt_traffic.json).
// Here the K tiles of pass 1 of a polynomial and the K tiles of its pass 2 are tasks of one per-XCD
// queue, so pass 2 reads what pass 1 of the same XCD just wrote, out of that XCD's L2.
//
// Scheduling.  Workgroups read their XCD id (HW_REG_XCC_ID) and pull task numbers from that XCD's
// queue head.  Task t of XCD x: block k = t / 2K, u = t % 2K;  u < K is pass-1 tile u of local poly
// k, u >= K is pass-2 tile u - K of local poly k - D (lag D lets pass 1 finish before pass 2 needs
// it).  Local poly j of XCD x is bound to the next global (limb, batch) polynomial by whoever pulls
// its tile 0 (a device-wide counter), so XCDs load-balance and no XCD count is assumed.
// Deadlock freedom: a task only ever waits for tasks with smaller numbers of the same queue, and
// those were pulled by running workgroups that never wait on later tasks.  Every spin is bounded;
// a timeout sets FusedSync::err (read by mfhe_ctx_get_option(MFHE_OPT_NTT_FUSED_ERRORS)).
//
// Visibility.  Producer and consumer of a hand-off always sit on the same XCD (the queue is chosen by
// HW_REG_XCC_ID, never by blockIdx), so the XCD's L2 is the coherence point between them and the
// intermediate never has to leave it (MI355X_MICROARCH.md "inter-workgroup visibility": stores keep
// their lines in the XCD L2; only the CU's own L1 can be stale).  Producer: plain stores -> every wave
// s_waitcnt vmcnt(0) (stores acknowledged by the L2) -> barrier -> lane 0 relaxed agent atomic add on the
// poly's arrival counter.  Consumer: lane 0 polls the counter with sc1 (L1-bypass) loads -> barrier ->
// every load of the intermediate is an sc1 load, served by the L2, so no L1 line of this CU (e.g. the
// original input it read in pass 1) can be returned.  No agent release/acquire fence is needed: the
// release's L2 write-back (buffer_wbl2) is exactly the traffic this kernel exists to avoid.
#pragma once
#include "ntt_kernels.hpp"

namespace mfhe {

constexpr int kFusedXcc = 16;    // queue slots (XCC ids 0..15)

// Zeroed before every launch.  map / arr hold `cap` entries per XCD queue (one per local poly, no
// reuse), cap >= npl + the empty local polys workgroups can open before they exit.
struct FusedSync {
    uint32_t head[kFusedXcc][32];   // one 128-B line per queue head
    uint32_t gcount;                // next global polynomial
    uint32_t err;                   // 1: map wait timed out, 2: arrival wait timed out, 4: cap exceeded
    uint32_t pad[30];
    // followed by uint64_t map[kFusedXcc][cap] ((local poly + 1) << 32 | global poly)
    //         and uint32_t arr[kFusedXcc][cap] (pass-1 arrivals)
};

template <class TS>
struct FusedArgs {
    PassArgs<TS> p;        // shared by pass 1 and pass 2 (forward: column then block; inverse: block then column)
    FusedSync* sync;
    uint64_t* map;
    uint32_t* arr;
    uint32_t cap;          // entries per XCD in map / arr
    uint32_t K;            // tiles per polynomial in each pass
    uint32_t npl;          // polynomials (batch * nlimbs)
    uint32_t lag;          // D
};

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x & (kFusedXcc - 1);
}

__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint32_t kSpinLimit = 1u << 24;

template <class P1, class P2, class TS>
__global__ __launch_bounds__(P1::NT) void ntt_fused_kernel(FusedArgs<TS> f) {
    static_assert(P1::NT == P2::NT, "both passes must use the same workgroup size");
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
    constexpr size_t LDSW = (P1::LDS_BYTES > P2::LDS_BYTES ? P1::LDS_BYTES : P2::LDS_BYTES) / 8;
    uint32_t* bc = reinterpret_cast<uint32_t*>(lds + LDSW);   // broadcast words
    const uint32_t t = threadIdx.x;
    const uint32_t x = xcc_id();
    FusedSync* sy = f.sync;
    const uint32_t K = f.K, D = f.lag;
    const P1 p1(f.p);
    const P2 p2(f.p);

    while (true) {
        __syncthreads();   // previous task's readers of bc[] are done
        if (t == 0) {
            const uint32_t task = __hip_atomic_fetch_add(&sy->head[x][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t k = task / (2 * K), u = task % (2 * K);
            uint32_t kind = 0, j = 0, tile = 0, v = 0xFFFFFFFFu;   // kind: 0 skip, 1 pass 1, 2 pass 2, 3 exit
            uint64_t* const map = f.map + (size_t)x * f.cap;
            uint32_t* const arr = f.arr + (size_t)x * f.cap;
            if (k >= f.cap) {
                // more local polys than provisioned: every real poly was handed out long before this
                atomicOr(&sy->err, 4u);
                kind = 3;
            } else if (u < K) {
                j = k;
                tile = u;
                uint64_t* slot = &map[j];
                const uint64_t tag = (uint64_t)(j + 1) << 32;
                if (tile == 0) {
                    v = __hip_atomic_fetch_add(&sy->gcount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(slot, tag | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    uint32_t n = 0;
                    uint64_t m;
                    while (((m = ld_agent(slot)) >> 32) != (uint64_t)(j + 1)) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++n == kSpinLimit) { atomicOr(&sy->err, 1u); break; }
                    }
                    v = (uint32_t)m;
                }
                kind = v < f.npl ? 1 : 0;
            } else if (k >= D) {
                j = k - D;
                tile = u - K;
                const uint64_t* slot = &map[j];
                uint32_t n = 0;
                uint64_t m;
                while (((m = ld_agent(slot)) >> 32) != (uint64_t)(j + 1)) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++n == kSpinLimit) { atomicOr(&sy->err, 1u); break; }
                }
                v = (uint32_t)m;
                if (v >= f.npl) {
                    kind = 3;
                } else {
                    n = 0;
                    while (ld_agent(&arr[j]) < K) {
                        __builtin_amdgcn_s_sleep(1);
                        if (++n == kSpinLimit) { atomicOr(&sy->err, 2u); break; }
                    }
                    kind = 2;
                }
            }
            bc[0] = kind;
            bc[1] = v * K + tile;   // tile number inside the pass
            bc[2] = j;
        }
        __syncthreads();
        // readfirstlane: the broadcast words are workgroup-uniform, so tile addressing stays in SGPRs
        const uint32_t kind = __builtin_amdgcn_readfirstlane(bc[0]);
        const uint32_t lb = __builtin_amdgcn_readfirstlane(bc[1]);
        const uint32_t j = __builtin_amdgcn_readfirstlane(bc[2]);
        if (kind == 3) break;
        if (kind == 0) continue;
        if (kind == 1) {
            const TileLoc L = p1.locate(lb);
            uint64_t raw[P1::R];
            p1.load(L, raw);
            p1.compute_store(L, raw, lds);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                __hip_atomic_fetch_add(&f.arr[(size_t)x * f.cap + j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            const TileLoc L = p2.locate(lb);
            uint64_t raw[P2::R];
            p2.load_l2(L, raw);
            p2.compute_store(L, raw, lds);
        }
    }
}

}  // namespace mfhe
