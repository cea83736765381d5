// l2_handoff_floor: the memory schedule of a C3 forward NTT (N = 2^16, L = 8, batch 1024 = 4 GiB in place) whose
// intermediate between the column stages and the block stages is handed off inside ONE XCD's L2 instead of going
// through the Infinity Cache -- the per-XCD mini-chunk plan DESIGN.md §8 priced on paper in r04.
// No butterflies: this is the floor any NTT on this schedule could reach, next to the two floors twopass_floor.hip
// measured (B: two in-place sweeps per 228 MiB chunk, the current plan; C: one sweep, the 16N single-pass floor).
//
// Schedule D (one persistent launch over the whole 4 GiB):
//   * a workgroup reads its XCD from HW_REG_XCC_ID and only ever takes tasks from that XCD's queue, so every
//     producer and consumer of a polynomial run on the same XCD by construction (placement is read, not assumed);
//     XCD x owns the limb-major polynomials [1024 x, 1024 x + 1024) (at C3: exactly limb x);
//   * the XCD's polynomials go in mini-chunks of M polynomials; a chunk is 16 M column tasks (A: 256 rows x 16
//     columns = 32 KiB, 128-B row segments, the column pass's tile) and 16 M block tasks (B: 16 contiguous 2 KiB rows
//     = 32 KiB, the block pass's rows);
//   * dequeue order per XCD with lag lam: A(0..lam), then B(0), A(lam + 1), B(1), A(lam + 2), ...; lam = 0 is the
//     "XCD barrier between phases" form (B(c) waits for every A(c) task and nothing else is queued in front of it),
//     lam >= 1 the "two (or more) mini-chunks in flight" form (A(c + 1) runs while B(c) waits);
//   * hand-off: an A task stores its tile back in place with PLAIN stores (the lines stay dirty in the XCD's L2),
//     every wave drains (s_waitcnt vmcnt(0)), workgroup barrier, then one lane adds 1 to done[x][c] (agent-scope
//     atomic, performed at the L2); a B task's lane 0 polls done[x][c] with sc1 loads until it reads 16 M, a barrier
//     releases the workgroup, and EVERY load of the tile is an sc1 buffer load (bypasses the CU's L1: the L2 of this
//     XCD, where the producer's bytes are, is the point of coherence for both workgroups);
//     rel = 1 adds the agent-scope release (buffer_wbl2 sc1 + wait) before the counter add, i.e. the by-the-rules
//     cross-XCD form, to price what it costs;
//   * B stores the final words with cache policy `outpol` (18 = sc1 nt, the NTT's output policy; 0 = plain; 2 = nt).
//   Dequeue is one returning atomic per task, issued one task ahead.  Progress holds for any residency: a B task only
//   waits on A tasks that sit earlier in its XCD's sequence, and a task is only dequeued by a running workgroup.
//
// Modes:
//   sweep [DE]                              time B, C and D / E over M x lam x workgroups-per-CU x outpol (+ D rel = 1)
//   one D|E M lam wpc outpol rel [iters]    time one setting (for rocprofv3 --pmc passes)
//   stress D|E M lam wpc outpol rel iters   every word checked after every launch, half of the launches with a
//                                           concurrent load kernel on another stream (uneven load)
// A word w goes through A as w + 1 and through B as (w + 1) ^ 3: a B task that read a stale (pre-A) line writes
// w ^ 3, which the check counts separately.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm -amdgpu-atomic-optimizer-strategy=None -o l2_handoff_floor l2_handoff_floor.hip
// (without the flag the dequeue atomic is rewritten into a wave-aggregated form whose result is waited for at once)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <csignal>
#include <execinfo.h>
#include <unistd.h>

#define CHECK(x)                                                                                  \
    do {                                                                                          \
        hipError_t e = (x);                                                                       \
        if (e != hipSuccess) {                                                                    \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);          \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

constexpr int LOGN = 16, NPOLY = 8192, NCHUNK2P = 18, PPX = NPOLY / 8;
constexpr uint64_t N = 1ull << LOGN;
constexpr uint32_t kStWords = 256 + 8 * PPX;   // heads (one 128-B line each), then done[8][<= 1024]
constexpr uint32_t kTmo = 255;                 // timeout word

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return (x & 15u) % 8u;
}

__device__ __forceinline__ uint32_t ld_sc1(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One persistent launch of schedule D.  seq[b] = (type 0 = A / 1 = B, chunk) for task block b of every XCD.
template <int OUTPOL>
__global__ __launch_bounds__(256) void xl2_kernel(uint64_t* d, uint32_t* st, const int2* seq, uint32_t M,
                                                  uint32_t nchunk, int rel) {
    __shared__ uint32_t s_task[2];
    const uint32_t t = threadIdx.x;
    const uint32_t x = xcc_id();
    uint32_t* head = st + x * 32;
    uint32_t* done = st + 256 + x * nchunk;
    const uint32_t tpc = 16 * M, ntask = 2 * nchunk * tpc;
    uint64_t* xb = d + (uint64_t)x * PPX * N;
    if (t == 0) s_task[0] = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    uint32_t task = s_task[0], it = 0;
    while (task < ntask) {
        // the next task, dequeued now and read after this task's loads: an asm atomic, so the compiler neither waits
        // for it at the loop head nor at the branch merges; its result is waited for by the counted vmcnt(8) below
        // (this wave's only vector-memory operations after it are the tile's 8 loads, and the B poll's loads, which
        // wait vmcnt(0))
        uint32_t nxt;
        if (t == 0) asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(nxt) : "v"(head), "v"(1u) : "memory");
        const uint32_t b = task / tpc, tile = task - b * tpc;
        const uint64_t sqw = ((const __attribute__((address_space(4))) uint64_t*)seq)[b];   // scalar load (lgkmcnt)
        const int2 sq = make_int2((int)(uint32_t)sqw, (int)(uint32_t)(sqw >> 32));
        const uint32_t c = (uint32_t)sq.y;
        const uint32_t pl = c * M + tile / 16, sub = tile % 16;
        uint64_t* pb = xb + (uint64_t)pl * N;
        if (sq.x == 0) {
            // A: column tile sub (16 columns x 256 rows), 16 B per lane, 8 rows x 128 B per wave instruction
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(pb + sub * 16, 0, 0x7FFFFFFF, 0x00020000);
            u32x4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t q = i * 256 + t;
                v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((q >> 3) * 2048 + (q & 7) * 16), 0, 0);
            }
            if (t == 0) {   // waits for the dequeue only (issued before the loads)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                s_task[(it + 1) & 1] = nxt;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t q = i * 256 + t;
                const uint64_t lo = ((uint64_t)v[i].y << 32 | v[i].x) + 1, hi = ((uint64_t)v[i].w << 32 | v[i].z) + 1;
                v[i] = u32x4{(unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32)};
                __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, (int)((q >> 3) * 2048 + (q & 7) * 16), 0, 0);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
            lds_barrier();
            if (t == 0) {
                if (rel) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __hip_atomic_fetch_add(done + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            // B: rows 16 sub .. 16 sub + 15 (32 KiB contiguous) once every A task of chunk c has signalled
            if (t == 0) {
                uint32_t spins = 0;
                while (ld_sc1(done + c) < tpc) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > (1u << 20) || ld_sc1(st + kTmo)) {   // bounded; one timeout ends every spin
                        __hip_atomic_store(st + kTmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
            lds_barrier();
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(pb + (size_t)sub * 16 * 256, 0, 0x7FFFFFFF, 0x00020000);
            u32x4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (i * 256 + t) * 16, 0, 16);
            if (t == 0) {
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                s_task[(it + 1) & 1] = nxt;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                v[i].x ^= 3u;
                v[i].z ^= 3u;
                __builtin_amdgcn_raw_buffer_store_b128(v[i], rs, (i * 256 + t) * 16, 0, OUTPOL);
            }
        }
        // s_task is double-buffered: slot (it + 1) & 1 is next written in iteration it + 2, after this barrier
        lds_barrier();
        task = s_task[(it + 1) & 1];
        ++it;
    }
}

// Schedule E: D's queues, order and hand-off, software-pipelined the way an NTT kernel on this schedule would run:
// each task's 32 KiB tile goes global -> LDS by LDS-DMA (16 B per lane, 8 instructions per thread; B tiles with sc1),
// the next task's DMA is issued before the current tile is read out of LDS and stored (16 8-B stores per thread in the
// column / block passes' store patterns), so one tile is always landing.  An A task's counter add is issued once its
// stores have drained, at the top of the next iteration (the drain also covers the prefetched DMA, which the next
// tile needs anyway).  A B task's DMA is prefetched only if its chunk is already complete (one non-blocking sc1 poll);
// otherwise the workgroup first finishes and signals its current task, then polls blocking -- so no workgroup ever
// blocks while it holds an unfinished A task (progress: the earliest unfinished task of an XCD is always runnable).
#ifndef NO_E
template <int OUTPOL>
__global__ __launch_bounds__(256) void xl2p_kernel(uint64_t* d, uint32_t* st, const int2* seq, uint32_t M,
                                                   uint32_t nchunk) {
    extern __shared__ __attribute__((aligned(16))) uint64_t lds[];   // two 32 KiB tile buffers
    __shared__ uint32_t s_ctl[2];
    typedef __attribute__((address_space(3))) void* lds_vp;
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t x = xcc_id();
    uint32_t* head = st + x * 32;
    uint32_t* done = st + 256 + x * nchunk;
    const uint32_t tpc = 16 * M, ntask = 2 * nchunk * tpc;
    uint64_t* xb = d + (uint64_t)x * PPX * N;
    struct Task {
        bool a;
        uint32_t c, sub;
        uint64_t* pb;
    };
    auto decode = [&](uint32_t task) {
        const uint32_t b = task / tpc, tile = task - b * tpc;
        const uint64_t sqw = ((const __attribute__((address_space(4))) uint64_t*)seq)[b];
        Task k;
        k.a = (uint32_t)sqw == 0;
        k.c = (uint32_t)(sqw >> 32);
        k.sub = tile % 16;
        k.pb = xb + (uint64_t)(k.c * M + tile / 16) * N;
        return k;
    };
    auto dma = [&](const Task& k, uint64_t* buf) {
        if (k.a) {
            const char* base = (const char*)k.pb + k.sub * 128;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t q = (i * 4 + w) * 64 + lane;   // 16-B chunk: row q / 8, part q % 8
                __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)(q >> 3) * 2048 + (q & 7) * 16),
                                                 (lds_vp)((char*)buf + (i * 4 + w) * 1024), 16, 0, 0);
            }
        } else {
            const char* base = (const char*)(k.pb + (size_t)k.sub * 16 * 256);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t q = (i * 4 + w) * 64 + lane;
                __builtin_amdgcn_global_load_lds((const void*)(base + (size_t)q * 16),
                                                 (lds_vp)((char*)buf + (i * 4 + w) * 1024), 16, 0, 16);
            }
        }
    };
    auto poll = [&](uint32_t c) {   // lane 0 only; bounded
        uint32_t spins = 0;
        while (ld_sc1(done + c) < tpc) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 20) || ld_sc1(st + kTmo)) {
                __hip_atomic_store(st + kTmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    };
    uint32_t nn = 0;   // lane 0: the task after nxt (dequeued one iteration ahead)
    int64_t sig = -1;  // lane 0: chunk whose A task this workgroup stored and has not signalled yet
    if (t == 0) {
        s_ctl[0] = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_ctl[1] = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    uint32_t cur = s_ctl[0], nxt = s_ctl[1];
    if (cur >= ntask) return;
    Task kc = decode(cur);
    if (t == 0 && !kc.a) poll(kc.c);   // holds nothing unfinished: may block
    lds_barrier();
    dma(kc, lds);
    uint32_t cb = 0;
    while (true) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // previous stores + this tile's DMA (+ the dequeue)
        lds_barrier();
        if (t == 0) {
            if (sig >= 0) __hip_atomic_fetch_add(done + sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sig = -1;
            nn = __hip_atomic_fetch_add(head, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint32_t ready = 0;
            if (nxt < ntask) {
                const Task kn = decode(nxt);
                ready = kn.a || ld_sc1(done + kn.c) >= tpc;
            }
            s_ctl[0] = ready;
        }
        lds_barrier();
        const bool ready = s_ctl[0] != 0;
        Task kn{};
        if (nxt < ntask) kn = decode(nxt);
        uint64_t* nbuf = lds + (cb ^ 1) * 4096;
        if (ready) dma(kn, nbuf);
        // the current tile: LDS -> registers -> global (the passes' store patterns)
        const uint64_t* buf = lds + cb * 4096;
        if (kc.a) {
            const uint32_t gl = t & 15, tau = t >> 4;   // column gl, rows 16 tau + k
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(kc.pb + kc.sub * 16, 0, 0x7FFFFFFF, 0x00020000);
            uint64_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = buf[(tau * 16 + k) * 16 + gl] + 1;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v[k]),
                                                      rs, (int)(((tau * 16 + k) * 256 + gl) * 8), 0, 0);
            if (t == 0) sig = kc.c;
        } else {
            const uint32_t gl = t >> 4, tau = t & 15;   // row gl, elements 16 k + tau
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(kc.pb + (size_t)kc.sub * 16 * 256, 0, 0x7FFFFFFF, 0x00020000);
            uint64_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = buf[gl * 256 + k * 16 + tau] ^ 3;
#pragma unroll
            for (int k = 0; k < 16; ++k)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v[k]),
                                                      rs, (int)((gl * 256 + k * 16 + tau) * 8), 0, OUTPOL);
        }
        if (nxt >= ntask) break;
        if (!ready) {   // finish and signal the current task, then wait for nxt's chunk
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();
            if (t == 0) {
                if (sig >= 0) __hip_atomic_fetch_add(done + sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                sig = -1;
                poll(kn.c);
            }
            lds_barrier();
            dma(kn, nbuf);
        }
        cur = nxt;
        kc = kn;
        cb ^= 1;
        if (t == 0) s_ctl[1] = nn;
        lds_barrier();
        nxt = s_ctl[1];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (t == 0 && sig >= 0) __hip_atomic_fetch_add(done + sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#endif
// contiguous in-place read-modify-write, 16 B per lane, grid-stride (twopass_floor.hip's B / C)
__global__ __launch_bounds__(256) void rmw(ulonglong2* o, size_t n16, int nt) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t stp = (size_t)gridDim.x * blockDim.x;
    for (; i < n16; i += stp) {
        ulonglong2 v = o[i];
        v.x += 1;
        v.y ^= 3;
        if (nt) {
            __builtin_nontemporal_store(v.x, &o[i].x);
            __builtin_nontemporal_store(v.y, &o[i].y);
        } else {
            o[i] = v;
        }
    }
}

__device__ __forceinline__ uint64_t pat(uint64_t i) { return (i * 0x9E3779B97F4A7C15ull) ^ (i >> 7); }

__global__ void fill_kernel(uint64_t* d, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) d[i] = pat(i);
}

// cnt[0]: words != (w + 1) ^ 3; cnt[1]: of those, words == w ^ 3 (B read the pre-A line); cnt[2]: == w + 1 (B never ran)
__global__ void check_kernel(const uint64_t* d, size_t n, unsigned long long* cnt) {
    unsigned long long bad = 0, stale = 0, unb = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t w = pat(i), v = d[i];
        const uint64_t xr = 3;   // B xors 3 into the low dword of every word
        if (v != ((w + 1) ^ xr)) {
            ++bad;
            if (v == (w ^ xr)) ++stale;
            if (v == w + 1) ++unb;
        }
    }
    if (bad) atomicAdd(cnt, bad);
    if (stale) atomicAdd(cnt + 1, stale);
    if (unb) atomicAdd(cnt + 2, unb);
}

// a concurrent load for the stress run: 64 workgroups stream over a 256 MiB buffer for ~1 ms
__global__ __launch_bounds__(256) void hog_kernel(ulonglong2* o, size_t n16, int reps) {
    for (int r = 0; r < reps; ++r)
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
            ulonglong2 v = o[i];
            v.x += 1;
            o[i] = v;
        }
}

struct Sched {
    int M, lam;
    uint32_t nchunk;
    int2* dseq;
    uint32_t* st;
};

static Sched make_sched(int M, int lam) {
    Sched s{M, lam, (uint32_t)(PPX / M), nullptr, nullptr};
    std::vector<int2> seq;
    uint32_t na = 0, nb = 0;
    for (int i = 0; i <= lam && na < s.nchunk; ++i) seq.push_back(make_int2(0, (int)na++));
    while (nb < s.nchunk) {
        seq.push_back(make_int2(1, (int)nb++));
        if (na < s.nchunk) seq.push_back(make_int2(0, (int)na++));
    }
    CHECK(hipMalloc(&s.dseq, seq.size() * sizeof(int2)));
    CHECK(hipMemcpy(s.dseq, seq.data(), seq.size() * sizeof(int2), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&s.st, kStWords * 4));
    return s;
}

static void run_d(uint64_t* d, const Sched& s, int wpc, int outpol, int rel, hipStream_t str) {
    CHECK(hipMemsetAsync(s.st, 0, kStWords * 4, str));
    auto k = outpol == 0 ? xl2_kernel<0> : outpol == 2 ? xl2_kernel<2> : xl2_kernel<18>;
    hipLaunchKernelGGL(k, dim3(256 * wpc), dim3(256), 0, str, d, s.st, s.dseq, (uint32_t)s.M, s.nchunk, rel);
}

static void run_e(uint64_t* d, const Sched& s, int wpc, int outpol, hipStream_t str) {
    CHECK(hipMemsetAsync(s.st, 0, kStWords * 4, str));
#ifndef NO_E
    auto k = outpol == 0 ? xl2p_kernel<0> : outpol == 2 ? xl2p_kernel<2> : xl2p_kernel<18>;
    hipLaunchKernelGGL(k, dim3(256 * wpc), dim3(256), 65536, str, d, s.st, s.dseq, (uint32_t)s.M, s.nchunk);
#endif
}

static uint32_t read_tmo(const Sched& s) {
    uint32_t v = 0;
    CHECK(hipMemcpy(&v, s.st + kTmo, 4, hipMemcpyDeviceToHost));
    return v;
}

template <class F>
static float time_ms(F&& run, int iters, hipStream_t str) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int w = 0; w < 5; ++w) run();
    CHECK(hipStreamSynchronize(str));
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e0, str));
    for (int it = 0; it < iters; ++it) run();
    CHECK(hipEventRecord(e1, str));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms / iters;
}

static void report(const char* name, float ms, const char* extra) {
    const double ntt_s = NPOLY / (ms * 1e-3);
    const double alg = 16.0 * N * ntt_s / 1e9;
    printf("{\"variant\": \"%s\", %s\"ms_per_4GiB\": %.4f, \"equiv_fwd_NTT_per_s\": %.0f, \"equiv_frac\": %.4f}\n", name,
           extra, ms, ntt_s, alg / 8000.0);
    fflush(stdout);
}

static void on_fpe(int sig, siginfo_t* si, void*) {
    void* bt[64];
    const int n = backtrace(bt, 64);
    fprintf(stderr, "signal %d at %p\n", sig, si->si_addr);
    backtrace_symbols_fd(bt, n, 2);
    _exit(3);
}

int main(int argc, char** argv) {
    struct sigaction sa = {};
    sa.sa_sigaction = on_fpe;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGFPE, &sa, nullptr);
    const char* mode = argc > 1 ? argv[1] : "sweep";
    const size_t bytes = (size_t)NPOLY * N * 8;
    uint64_t* d;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMemset(d, 1, bytes));
    hipStream_t str;
    CHECK(hipStreamCreateWithFlags(&str, hipStreamNonBlocking));
    auto run = [&](char kind, const Sched& s, int wpc, int outpol, int rel) {
        if (kind == 'E') run_e(d, s, wpc, outpol, str);
        else run_d(d, s, wpc, outpol, rel, str);
    };
    auto line = [&](char kind, const Sched& s, int wpc, int outpol, int rel, int iters) {
        const float ms = time_ms([&]() { run(kind, s, wpc, outpol, rel); }, iters, str);
        char ex[200];
        snprintf(ex, sizeof ex, "\"kind\": \"%c\", \"M\": %d, \"lam\": %d, \"wg_per_cu\": %d, \"outpol\": %d, \"rel\": %d, "
                 "\"tmo\": %u, ", kind, s.M, s.lam, wpc, outpol, rel, read_tmo(s));
        report(kind == 'E' ? "E per-XCD L2 hand-off, LDS-DMA pipelined" : "D per-XCD L2 hand-off", ms, ex);
    };

    if (!strcmp(mode, "sweep")) {
        const uint32_t cb = (NPOLY + NCHUNK2P - 1) / NCHUNK2P;
        auto two = [&]() {
            for (uint32_t p0 = 0; p0 < NPOLY; p0 += cb) {
                const uint32_t np = p0 + cb <= NPOLY ? cb : NPOLY - p0;
                const size_t n16 = (size_t)np * N / 2;
                hipLaunchKernelGGL(rmw, dim3(2048), dim3(256), 0, str, (ulonglong2*)(d + (uint64_t)p0 * N), n16, 0);
                hipLaunchKernelGGL(rmw, dim3(2048), dim3(256), 0, str, (ulonglong2*)(d + (uint64_t)p0 * N), n16, 1);
            }
        };
        auto one = [&]() { hipLaunchKernelGGL(rmw, dim3(2048), dim3(256), 0, str, (ulonglong2*)d, bytes / 16, 1); };
        const char* kinds = argc > 2 ? argv[2] : "DE";
        for (int rep = 0; rep < 2; ++rep) {
            report("B two-pass floor (two in-place sweeps per 228 MiB chunk)", time_ms(two, 20, str), "");
            report("C one-pass floor (one in-place sweep)", time_ms(one, 20, str), "");
            for (const char* kp = kinds; *kp; ++kp) {
                const char kind = *kp;
                for (int M : {1, 2, 4})
                    for (int lam = (kind == 'E' ? 1 : 0); lam <= 2; ++lam) {
                        Sched s = make_sched(M, lam);
                        for (int wpc : {1, 2})
                            for (int outpol : {0, 18}) line(kind, s, wpc, outpol, 0, 20);
                        if (rep == 0 && kind == 'D' && M == 2 && lam == 1) line('D', s, 2, 18, 1, 20);
                        CHECK(hipFree(s.dseq));
                        CHECK(hipFree(s.st));
                    }
            }
        }
    } else if (!strcmp(mode, "one") || !strcmp(mode, "stress")) {
        if (argc < 8) {
            printf("usage: %s %s D|E M lam wpc outpol rel [iters]\n", argv[0], mode);
            return 2;
        }
        const char kind = argv[2][0];
        const int M = atoi(argv[3]), lam = atoi(argv[4]), wpc = atoi(argv[5]), outpol = atoi(argv[6]), rel = atoi(argv[7]);
        const int iters = argc > 8 ? atoi(argv[8]) : 20;
        if (M < 1 || PPX % M || wpc < 1 || wpc > 4 || lam < 0 || (kind != 'D' && kind != 'E')) {
            printf("bad arguments\n");
            return 2;
        }
        Sched s = make_sched(M, lam);
        if (!strcmp(mode, "one")) {
            line(kind, s, wpc, outpol, rel, iters);
        } else {
            unsigned long long* cnt;
            CHECK(hipMalloc(&cnt, 3 * sizeof(unsigned long long)));
            ulonglong2* hog;
            const size_t hog_bytes = 256ull << 20;
            CHECK(hipMalloc(&hog, hog_bytes));
            hipStream_t hs;
            CHECK(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
            unsigned long long tot[3] = {0, 0, 0};
            int bad_launches = 0, tmo_launches = 0;
            for (int it = 0; it < iters; ++it) {
                hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, str, d, bytes / 8);
                CHECK(hipStreamSynchronize(str));
                if (it & 1) hipLaunchKernelGGL(hog_kernel, dim3(64), dim3(256), 0, hs, hog, hog_bytes / 16, 4);
                run(kind, s, wpc, outpol, rel);
                CHECK(hipMemsetAsync(cnt, 0, 3 * sizeof(unsigned long long), str));
                hipLaunchKernelGGL(check_kernel, dim3(4096), dim3(256), 0, str, d, bytes / 8, cnt);
                unsigned long long h[3];
                CHECK(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, str));
                CHECK(hipStreamSynchronize(str));
                CHECK(hipStreamSynchronize(hs));
                CHECK(hipGetLastError());
                const uint32_t tm = read_tmo(s);
                if (h[0]) ++bad_launches;
                if (tm) ++tmo_launches;
                for (int k = 0; k < 3; ++k) tot[k] += h[k];
                if (it % 50 == 49) {
                    printf("{\"stress_progress\": %d, \"bad_launches\": %d, \"tmo_launches\": %d}\n", it + 1, bad_launches,
                           tmo_launches);
                    fflush(stdout);
                }
            }
            printf("{\"stress\": \"%c\", \"M\": %d, \"lam\": %d, \"wg_per_cu\": %d, \"outpol\": %d, "
                   "\"rel\": %d, \"launches\": %d, \"words_per_launch\": %zu, \"bad_launches\": %d, \"tmo_launches\": %d, "
                   "\"bad_words\": %llu, \"stale_words\": %llu, \"unprocessed_words\": %llu}\n",
                   kind, M, lam, wpc, outpol, rel, iters, bytes / 8, bad_launches, tmo_launches, tot[0], tot[1], tot[2]);
        }
    } else {
        printf("unknown mode %s\n", mode);
        return 2;
    }
    CHECK(hipFree(d));
    return 0;
}
