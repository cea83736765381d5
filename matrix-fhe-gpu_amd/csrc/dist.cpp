// dist.cpp -- multi-GPU residue sharding over RCCL (xGMI): the C-ABI exchange + sharded wide-CRT recombine.
//
// NTT, RNS decompose and W-CRT are independent per RNS limb, so rank g of G owns limbs
// [g*L/G, (g+1)*L/G) of every polynomial and transforms them with no communication.  The wide CRT compose
// needs all L residues of a coefficient: that is the one exchange step.  It replaces the reference's
// single-GPU per-lane compose loop (src/core/HE.cu:1653-1668 -> crt_compose_centerlift_big,
// src/core/encoder.cu:191-245); the reference itself has no multi-GPU code.
//
// RCCL is loaded with dlopen on first use (librccl.so.1 from ROCm), so libmfhe.so itself carries no
// link-time RCCL dependency and loads on hosts without it; calls then return MFHE_EUNSUPPORTED.
//
// Exchanges (each rank's slice of the batch is [g*B/G, (g+1)*B/G)):
//   all-gather : every rank receives every shard, [G][B][L/G][n]; composes its slice in place.
//   all-to-all : chunk r of a rank's shard (the polys of rank r's slice) goes to rank r, so each rank
//                receives only the missing limbs of its own slice, [G][B/G][L/G][n].
// Both feed mfhe_crt_compose_f64_sharded, which reads the shards in place (no transpose).  The receive
// buffer is owned by the communicator and grown by mfhe_crt_recombine_reserve, outside timed code.
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include <type_traits>
#include <rccl/rccl.h>

#include "mfhe_ctx.hpp"

namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllToAll)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            return fp != nullptr;
        };
        r.ok = sym(r.GetUniqueId, "ncclGetUniqueId") && sym(r.CommInitRank, "ncclCommInitRank") &&
               sym(r.CommDestroy, "ncclCommDestroy") && sym(r.CommCount, "ncclCommCount") &&
               sym(r.CommUserRank, "ncclCommUserRank") && sym(r.AllGather, "ncclAllGather") &&
               sym(r.AllToAll, "ncclAllToAll") && sym(r.GetErrorString, "ncclGetErrorString");
    });
    return r;
}

int nccl_error(ncclResult_t e, const char* what) {
    const Rccl& r = rccl();
    return mfhe::set_error(MFHE_EHIP, std::string(what) + ": " + (r.GetErrorString ? r.GetErrorString(e) : "RCCL error"));
}

int need_rccl() {
    if (!rccl().ok) return mfhe::set_error(MFHE_EUNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
    return MFHE_OK;
}

}  // namespace

struct mfhe_comm {
    ncclComm_t comm = nullptr;
    bool owned = false;
    int nranks = 1, rank = 0, device = 0;
    void* recv = nullptr;   // receive buffer of the recombine exchange (the chunked form uses two halves)
    size_t recv_bytes = 0;
    int32_t* flags = nullptr;   // comm_agree: [nranks] gathered verdicts + [1] this rank's (allocated at creation)
    // chunked recombine: the exchanges run on xs, the composes on the caller's stream.  ev_x[b]: exchange into
    // receive half b done; ev_c[b]: compose out of half b done (xs waits on it before refilling b, also across
    // calls); ev_in: the caller's stream reached the call (the shard is ready)
    hipStream_t xs = nullptr;
    hipEvent_t ev_in = nullptr, ev_x[2] = {nullptr, nullptr}, ev_c[2] = {nullptr, nullptr};
    bool c_recorded[2] = {false, false};
    // a chunked call's exchanges were issued on xs and no reserve has synchronised them since: only then may the next
    // call skip its ev_in wait (MFHE_RECOMBINE_AFTER_PREV), because xs then runs its exchanges after those
    bool prev_on_xs = false;
};

using mfhe::set_error;

namespace {
void comm_free_resources(mfhe_comm* c) {
    if (c->recv) (void)hipFree(c->recv);
    if (c->flags) (void)hipFree(c->flags);
    for (hipEvent_t e : {c->ev_in, c->ev_x[0], c->ev_x[1], c->ev_c[0], c->ev_c[1]})
        if (e) (void)hipEventDestroy(e);
    if (c->xs) (void)hipStreamDestroy(c->xs);
    c->recv = nullptr;
    c->flags = nullptr;
    c->xs = nullptr;
}

// Everything a communicator needs besides RCCL itself, allocated when it is created: a failure here fails the
// creating call, never a later collective (where one rank returning early would leave its peers blocked).
int comm_alloc_resources(mfhe_comm* c) {
    hipError_t he = hipMalloc(&c->flags, (size_t)(c->nranks + 1) * sizeof(int32_t));
    if (he == hipSuccess) he = hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking);
    for (hipEvent_t* e : {&c->ev_in, &c->ev_x[0], &c->ev_x[1], &c->ev_c[0], &c->ev_c[1]})
        if (he == hipSuccess) he = hipEventCreateWithFlags(e, hipEventDisableTiming);
    if (he != hipSuccess) {
        comm_free_resources(c);
        return mfhe::hip_error(he, "communicator resources (flags, exchange stream, events)");
    }
    return MFHE_OK;
}
}  // namespace

extern "C" int mfhe_comm_unique_id(uint8_t* id) {
    if (!id) return set_error(MFHE_EINVAL, "null id");
    if (int rc = need_rccl()) return rc;
    ncclUniqueId u;
    ncclResult_t e = rccl().GetUniqueId(&u);
    if (e != ncclSuccess) return nccl_error(e, "ncclGetUniqueId");
    std::memcpy(id, u.internal, MFHE_COMM_ID_BYTES);
    return MFHE_OK;
}

extern "C" int mfhe_comm_init(const uint8_t* id, int nranks, int rank, mfhe_comm** out) {
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return set_error(MFHE_EINVAL, "mfhe_comm_init: bad argument");
    *out = nullptr;
    if (int rc = need_rccl()) return rc;
    ncclUniqueId u;
    std::memcpy(u.internal, id, MFHE_COMM_ID_BYTES);
    mfhe_comm* c = new mfhe_comm();
    hipError_t he = hipGetDevice(&c->device);
    if (he != hipSuccess) {
        delete c;
        return mfhe::hip_error(he, "hipGetDevice");
    }
    c->nranks = nranks;
    c->rank = rank;
    // local resources first: a rank that fails here never enters ncclCommInitRank, so its peers' init fails
    // by RCCL's own bootstrap timeout instead of a later collective hanging
    if (int rc = comm_alloc_resources(c)) {
        delete c;
        return rc;
    }
    ncclResult_t e = rccl().CommInitRank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        comm_free_resources(c);
        delete c;
        return nccl_error(e, "ncclCommInitRank");
    }
    c->owned = true;
    *out = c;
    return MFHE_OK;
}

extern "C" int mfhe_comm_wrap(void* nccl_comm, mfhe_comm** out) {
    if (!nccl_comm || !out) return set_error(MFHE_EINVAL, "mfhe_comm_wrap: null argument");
    *out = nullptr;
    if (int rc = need_rccl()) return rc;
    mfhe_comm* c = new mfhe_comm();
    c->comm = (ncclComm_t)nccl_comm;
    ncclResult_t e = rccl().CommCount(c->comm, &c->nranks);
    if (e == ncclSuccess) e = rccl().CommUserRank(c->comm, &c->rank);
    if (e != ncclSuccess) {
        delete c;
        return nccl_error(e, "ncclCommCount/UserRank");
    }
    (void)hipGetDevice(&c->device);
    if (int rc = comm_alloc_resources(c)) {
        delete c;
        return rc;
    }
    *out = c;
    return MFHE_OK;
}

extern "C" int mfhe_comm_destroy(mfhe_comm* c) {
    if (!c) return MFHE_OK;
    int rc = MFHE_OK;
    if (c->xs) {
        hipError_t he = hipStreamSynchronize(c->xs);
        if (he != hipSuccess) rc = mfhe::hip_error(he, "hipStreamSynchronize");
    }
    comm_free_resources(c);
    if (c->owned && c->comm) {
        ncclResult_t e = rccl().CommDestroy(c->comm);
        if (e != ncclSuccess && !rc) rc = nccl_error(e, "ncclCommDestroy");
    }
    delete c;
    return rc;
}

extern "C" int mfhe_comm_info(const mfhe_comm* c, int* nranks, int* rank) {
    if (!c) return set_error(MFHE_EINVAL, "null comm");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return MFHE_OK;
}

extern "C" int mfhe_allgather_limbs(mfhe_comm* c, const uint64_t* d_shard, size_t count, uint64_t* d_recv,
                                    mfhe_stream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null comm");
    if (count == 0) return MFHE_OK;
    if (!d_shard || !d_recv) return set_error(MFHE_EINVAL, "mfhe_allgather_limbs: null buffer");
    ncclResult_t e = rccl().AllGather(d_shard, d_recv, count, ncclUint64, c->comm, (hipStream_t)s);
    return e == ncclSuccess ? MFHE_OK : nccl_error(e, "ncclAllGather");
}

namespace mfhe {
int comm_allgather_bytes(mfhe_comm* c, const void* send, void* recv, size_t bytes, hipStream_t s) {
    if (!c) return set_error(MFHE_EINVAL, "null comm");
    if (bytes == 0) return MFHE_OK;
    if (int rc = need_rccl()) return rc;
    ncclResult_t e = rccl().AllGather(send, recv, bytes, ncclUint8, c->comm, s);
    return e == ncclSuccess ? MFHE_OK : nccl_error(e, "ncclAllGather");
}
int comm_agree(mfhe_comm* c, int local_rc, hipStream_t s) {
    if (!c) return local_rc ? local_rc : set_error(MFHE_EINVAL, "null comm");
    if (c->nranks == 1) return local_rc;
    if (int rc = need_rccl()) return local_rc ? local_rc : rc;
    const std::string mine = local_rc ? mfhe_last_error() : "";
    // c->flags exists since the communicator's creation (comm_alloc_resources): nothing here can fail before
    // this rank has joined the all-gather its peers are waiting in
    std::vector<int32_t> all((size_t)c->nranks, 0);
    const int32_t v = local_rc;
    hipError_t he = hipMemcpyAsync(c->flags + c->nranks, &v, sizeof v, hipMemcpyHostToDevice, s);
    if (he != hipSuccess) return mfhe::hip_error(he, "comm_agree");
    ncclResult_t e = rccl().AllGather(c->flags + c->nranks, c->flags, 1, ncclInt32, c->comm, s);
    if (e != ncclSuccess) return nccl_error(e, "comm_agree: ncclAllGather");
    he = hipMemcpyAsync(all.data(), c->flags, all.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he != hipSuccess) return mfhe::hip_error(he, "comm_agree");
    if (local_rc) return set_error(local_rc, mine);
    for (int r = 0; r < c->nranks; ++r)
        if (all[(size_t)r])
            return set_error(MFHE_EINVAL, "rank " + std::to_string(r) + " rejected the sharded call (code " +
                                              std::to_string(all[(size_t)r]) + "); see that rank's error");
    return MFHE_OK;
}
int comm_size_rank(const mfhe_comm* c, int* size, int* rank) {
    if (!c) return set_error(MFHE_EINVAL, "null comm");
    *size = c->nranks;
    *rank = c->rank;
    return MFHE_OK;
}
}  // namespace mfhe

namespace {

// receive-buffer words of one recombine exchange
int xchg_shape(const mfhe_ctx* ctx, const mfhe_comm* c, int mode, size_t npoly, size_t ncoeff, size_t* words) {
    if (!ctx || !c) return set_error(MFHE_EINVAL, "null ctx / comm");
    const int G = c->nranks;
    if (ctx->L % G) return set_error(MFHE_EINVAL, "recombine: the communicator size must divide L");
    if (npoly % (size_t)G) return set_error(MFHE_EINVAL, "recombine: the communicator size must divide npoly");
    if (mode != MFHE_XCHG_ALLGATHER && mode != MFHE_XCHG_ALLTOALL) return set_error(MFHE_EINVAL, "recombine: bad mode");
    const size_t shard = npoly * (size_t)(ctx->L / G) * ncoeff;   // this rank's [npoly][L/G][ncoeff]
    *words = mode == MFHE_XCHG_ALLGATHER ? shard * G : shard;     // all-to-all: G chunks of shard / G
    return MFHE_OK;
}

int grow(mfhe_comm* c, size_t bytes) {
    if (c->recv_bytes >= bytes) return MFHE_OK;
    if (c->recv) MFHE_HIP(hipFree(c->recv));
    c->recv = nullptr;
    c->recv_bytes = 0;
    hipError_t he = hipMalloc(&c->recv, bytes);
    if (he != hipSuccess) return set_error(MFHE_ENOMEM, "recombine receive buffer: hipMalloc failed");
    c->recv_bytes = bytes;
    return MFHE_OK;
}

}  // namespace

extern "C" int mfhe_crt_recombine_reserve(mfhe_ctx* ctx, mfhe_comm* c, int mode, size_t npoly, size_t ncoeff) {
    size_t words = 0;
    if (int rc = xchg_shape(ctx, c, mode, npoly, ncoeff, &words)) return rc;
    return grow(c, words * sizeof(uint64_t));
}

extern "C" int mfhe_crt_recombine_sharded(mfhe_ctx* ctx, mfhe_comm* c, int mode, const uint64_t* d_shard,
                                          size_t npoly, size_t ncoeff, double* d_out, size_t out_stride,
                                          mfhe_stream_t s) {
    size_t words = 0;
    if (int rc = xchg_shape(ctx, c, mode, npoly, ncoeff, &words)) return rc;
    if (npoly == 0 || ncoeff == 0) return MFHE_OK;
    if (!d_shard || !d_out || out_stride == 0) return set_error(MFHE_EINVAL, "recombine: bad pointer / stride");
    const int G = c->nranks;
    // world 1: the shard already holds every limb of every polynomial, nothing to exchange
    if (G == 1) return mfhe_crt_compose_f64_sharded(ctx, d_shard, 1, npoly * (size_t)ctx->L * ncoeff, npoly, ncoeff,
                                                    d_out, out_stride, s);
    if (int rc = need_rccl()) return rc;
    if (int rc = grow(c, words * sizeof(uint64_t))) return rc;
    const size_t bs = npoly / G, lg = (size_t)(ctx->L / G);
    const size_t shard = npoly * lg * ncoeff;
    uint64_t* recv = static_cast<uint64_t*>(c->recv);
    const hipStream_t st = (hipStream_t)s;
    ncclResult_t e;
    size_t off, stride;
    if (mode == MFHE_XCHG_ALLGATHER) {
        e = rccl().AllGather(d_shard, recv, shard, ncclUint64, c->comm, st);
        off = (size_t)c->rank * bs * lg * ncoeff;   // my slice inside every gathered shard
        stride = shard;
    } else {
        e = rccl().AllToAll(d_shard, recv, bs * lg * ncoeff, ncclUint64, c->comm, st);
        off = 0;
        stride = bs * lg * ncoeff;
    }
    if (e != ncclSuccess) return nccl_error(e, mode == MFHE_XCHG_ALLGATHER ? "ncclAllGather" : "ncclAllToAll");
    return mfhe_crt_compose_f64_sharded(ctx, recv + off, G, stride, bs, ncoeff, d_out, out_stride, s);
}

namespace {
// polys per chunk of the chunked recombine: a multiple of G, at least G, at most npoly
size_t chunk_polys_of(size_t chunk_polys, size_t npoly, int G) {
    size_t cp = chunk_polys / (size_t)G * (size_t)G;
    if (cp < (size_t)G) cp = (size_t)G;
    return cp < npoly ? cp : npoly;
}
}  // namespace

extern "C" int mfhe_crt_recombine_chunked_reserve(mfhe_ctx* ctx, mfhe_comm* c, int mode, size_t chunk_polys,
                                                  size_t ncoeff) {
    if (!c) return set_error(MFHE_EINVAL, "null comm");
    const size_t cp = chunk_polys_of(chunk_polys, (size_t)-1, c->nranks);
    size_t words = 0;
    if (int rc = xchg_shape(ctx, c, mode, cp, ncoeff, &words)) return rc;
    // host-synchronising: the previous calls' composes are done, so the next call waits on no event of theirs
    for (int b = 0; b < 2; ++b)
        if (c->c_recorded[b]) {
            MFHE_HIP(hipEventSynchronize(c->ev_c[b]));
            c->c_recorded[b] = false;
        }
    c->prev_on_xs = false;
    return grow(c, 2 * words * sizeof(uint64_t));
}

// The chunked recombine, pipelined ("chunked all-gather pipelined with compose").  The
// polynomials go in chunks of cp (a multiple of G); chunk k is one exchange of the chunk's shard rows
// [p0, p0 + cp) into receive half k % 2, run on the communicator's stream xs, and one in-place sharded compose of
// this rank's cp / G polys of the chunk out of that half, on the caller's stream s.  Events order them: the
// compose of chunk k waits for its exchange; the exchange of chunk k + 2 waits for the compose of chunk k (the
// half it refills).  So the exchange of chunk k + 1 runs while chunk k composes.  Output rows: compact (row
// k * cp / G + j, the order of mfhe/dist.py owned_polys) or, with MFHE_RECOMBINE_ROWS_GLOBAL, the global
// polynomial index p0 + rank * cp / G + j (rows of other ranks untouched).  Every chunk's exchange is complete
// before s proceeds past this call (the last compose waits for the last exchange, and xs runs them in order).
//
// Collective safety.  Every check that can fail runs before the first exchange, on arguments every rank passes
// alike.  Once the first exchange is issued, a local failure (a compose launch, an event call, the injected
// MFHE_RECOMBINE_DEBUG_FAIL) does not return early: the remaining exchanges are still issued (their composes
// skipped), so no peer is left inside a collective this rank never joins, and the first error is returned at the
// end (with MFHE_RECOMBINE_AGREE every rank then also learns it through comm_agree).
extern "C" int mfhe_crt_recombine_chunked(mfhe_ctx* ctx, mfhe_comm* c, int mode, const uint64_t* d_shard,
                                          size_t npoly, size_t ncoeff, size_t chunk_polys, double* d_out,
                                          size_t out_stride, int flags, mfhe_stream_t s) {
    size_t words = 0;
    if (int rc = xchg_shape(ctx, c, mode, npoly, ncoeff, &words)) return rc;   // G | L, G | npoly, mode
    if (npoly == 0 || ncoeff == 0) return MFHE_OK;
    constexpr int kKnown = MFHE_RECOMBINE_ROWS_GLOBAL | MFHE_RECOMBINE_EXCHANGE_ONLY | MFHE_RECOMBINE_AFTER_PREV |
                           MFHE_RECOMBINE_AGREE | MFHE_RECOMBINE_COMPOSE_ONLY | MFHE_RECOMBINE_SELF_EXCHANGE |
                           MFHE_RECOMBINE_DEBUG_FAIL;
    if (!d_shard || (!d_out && !(flags & MFHE_RECOMBINE_EXCHANGE_ONLY)) || out_stride == 0)
        return set_error(MFHE_EINVAL, "recombine: bad pointer / stride");
    if (flags & ~kKnown) return set_error(MFHE_EINVAL, "recombine: unknown flags");
    if ((flags & MFHE_RECOMBINE_EXCHANGE_ONLY) && (flags & MFHE_RECOMBINE_COMPOSE_ONLY))
        return set_error(MFHE_EINVAL, "recombine: EXCHANGE_ONLY and COMPOSE_ONLY exclude each other");
    const int G = c->nranks;
    if (G == 1 && !(flags & MFHE_RECOMBINE_SELF_EXCHANGE)) {
        // world 1: no exchange (the shard holds every limb of every polynomial) -- compose straight from it, all rows at
        // once (ROWS_GLOBAL and compact rows coincide); the flags keep their meaning
        if (flags & MFHE_RECOMBINE_DEBUG_FAIL)
            return set_error(MFHE_EHIP, "recombine: injected compose failure (MFHE_RECOMBINE_DEBUG_FAIL)");
        if (flags & MFHE_RECOMBINE_EXCHANGE_ONLY) return MFHE_OK;
        return mfhe_crt_compose_f64_sharded(ctx, d_shard, 1, npoly * (size_t)ctx->L * ncoeff, npoly, ncoeff, d_out,
                                            out_stride, s);
    }
    if (int rc = need_rccl()) return rc;
    const size_t lg = (size_t)(ctx->L / G), cp = chunk_polys_of(chunk_polys, npoly, G);
    size_t cw = 0;
    if (int rc = xchg_shape(ctx, c, mode, cp, ncoeff, &cw)) return rc;
    if (int rc = grow(c, 2 * cw * sizeof(uint64_t))) return rc;   // no-op after mfhe_crt_recombine_chunked_reserve
    uint64_t* half[2] = {static_cast<uint64_t*>(c->recv), static_cast<uint64_t*>(c->recv) + cw};
    const hipStream_t st = (hipStream_t)s;
    int err = MFHE_OK;   // first local failure after the exchanges started; later composes are skipped
    std::string err_msg;
    auto fail = [&](int rc) {
        if (rc && !err) {
            err = rc;
            err_msg = mfhe_last_error();
        }
    };
    auto hip = [&](hipError_t he, const char* what) {
        if (he != hipSuccess) fail(mfhe::hip_error(he, what));
    };
    const bool xch = !(flags & MFHE_RECOMBINE_COMPOSE_ONLY);
    if (!xch)   // the composes read what earlier calls' exchanges left in the halves: s is ordered after those
        for (int b = 0; b < 2; ++b) hip(hipStreamWaitEvent(st, c->ev_x[b], 0), "hipStreamWaitEvent");
    // AFTER_PREV is only safe behind a previous call's exchanges still ordered on xs; otherwise (the first call, or
    // the first after a reserve) it is ignored and the exchanges wait for s as usual
    if (xch && (!(flags & MFHE_RECOMBINE_AFTER_PREV) || !c->prev_on_xs)) {
        hip(hipEventRecord(c->ev_in, st), "hipEventRecord");
        hip(hipStreamWaitEvent(c->xs, c->ev_in, 0), "hipStreamWaitEvent");
    }
    size_t k = 0;
    for (size_t p0 = 0; p0 < npoly; p0 += cp, ++k) {
        const size_t n = npoly - p0 < cp ? npoly - p0 : cp;   // polys of this chunk (a multiple of G)
        const size_t bs = n / (size_t)G, shard = n * lg * ncoeff;
        const int b = (int)(k & 1);
        const uint64_t* send = d_shard + p0 * lg * ncoeff;
        const bool ag = mode == MFHE_XCHG_ALLGATHER;
        const size_t off = ag ? (size_t)c->rank * bs * lg * ncoeff : 0, stride = ag ? shard : bs * lg * ncoeff;
        if (xch) {
            if (c->c_recorded[b]) hip(hipStreamWaitEvent(c->xs, c->ev_c[b], 0), "hipStreamWaitEvent");
            const ncclResult_t e = ag ? rccl().AllGather(send, half[b], shard, ncclUint64, c->comm, c->xs)
                                      : rccl().AllToAll(send, half[b], bs * lg * ncoeff, ncclUint64, c->comm, c->xs);
            // an RCCL error leaves the communicator unusable (RCCL's own contract): nothing to keep in step with
            if (e != ncclSuccess) return nccl_error(e, ag ? "ncclAllGather" : "ncclAllToAll");
            hip(hipEventRecord(c->ev_x[b], c->xs), "hipEventRecord");
            hip(hipStreamWaitEvent(st, c->ev_x[b], 0), "hipStreamWaitEvent");
        }
        if ((flags & MFHE_RECOMBINE_DEBUG_FAIL) && k == (npoly > cp ? 1u : 0u))
            fail(set_error(MFHE_EHIP, "recombine: injected compose failure (MFHE_RECOMBINE_DEBUG_FAIL)"));
        if (!err && !(flags & MFHE_RECOMBINE_EXCHANGE_ONLY)) {
            const size_t row = (flags & MFHE_RECOMBINE_ROWS_GLOBAL) ? p0 + (size_t)c->rank * bs : p0 / (size_t)G;
            fail(mfhe_crt_compose_f64_sharded(ctx, half[b] + off, G, stride, bs, ncoeff,
                                              d_out + row * ncoeff * out_stride, out_stride, s));
        }
        // recorded even when the compose was skipped: s has passed the exchange, so half b may be refilled
        hip(hipEventRecord(c->ev_c[b], st), "hipEventRecord");
        c->c_recorded[b] = true;
    }
    if (xch) c->prev_on_xs = true;
    if (flags & MFHE_RECOMBINE_AGREE) return mfhe::comm_agree(c, err ? set_error(err, err_msg) : MFHE_OK, st);
    return err ? set_error(err, err_msg) : MFHE_OK;
}
