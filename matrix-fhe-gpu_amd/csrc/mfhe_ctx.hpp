// mfhe_ctx.hpp -- internal definition of the context object behind include/mfhe.h.
//
// One context = one parameter set on one device: moduli, ring degree N, scale,
// and every device table the hot path needs, built once at create time
// (the reference rebuilds/re-uploads tables lazily from many places and
// keys them on the first caller's limb count).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mfhe.h"
#include "ntt_arith.hpp"

namespace mfhe {

// thread-local error reporting
int set_error(int code, const std::string& msg);
// dist.cpp: in-place-capable all-gather of `bytes` per rank over a libmfhe communicator (RCCL)
int comm_allgather_bytes(mfhe_comm* comm, const void* send, void* recv, size_t bytes, hipStream_t s);
int comm_size_rank(const mfhe_comm* comm, int* size, int* rank);
// dist.cpp: every rank's local verdict (0 or an MFHE_* code) exchanged over the communicator (one tiny
// all-gather + a host sync; nothing for 1 rank).  Returns local_rc if this rank failed, an MFHE_EINVAL naming
// the failing rank if another did, else MFHE_OK -- so every rank reaches the same decision.
int comm_agree(mfhe_comm* comm, int local_rc, hipStream_t s);
int hip_error(hipError_t e, const char* what);
int ensure_xy(mfhe_ctx* c);   // XY encoder matrices, built on first use (ctx.cpp)

#define MFHE_HIP(call)                                          \
    do {                                                        \
        hipError_t _e = (call);                                 \
        if (_e != hipSuccess) return ::mfhe::hip_error(_e, #call); \
    } while (0)

#define MFHE_CHECK_LAUNCH(what)                                 \
    do {                                                        \
        hipError_t _e = hipGetLastError();                      \
        if (_e != hipSuccess) return ::mfhe::hip_error(_e, what); \
    } while (0)

// Per-limb constants of the FP64 wide-CRT fast path (crt.hip compose_fast): one 64-B scalar load per limb.
struct CrtLimbF {
    uint64_t q;
    double qf, invf, qinvf;   // q, (M_k mod q)^-1, 1/q as doubles (exact: q < 2^50)
    uint64_t M0;              // low word of M_k = Q / q_k
    uint64_t qinv64;          // q^-1 mod 2^64 (q odd): exact-divisibility test
    uint64_t lim;             // floor((2^64 - 1) / q)
    uint64_t pad;
};

struct NttTablesF {   // FP64 path: centred w
    double* tw = nullptr;    // [L][N]
    double* itw = nullptr;   // [L][N], itw[1] *= n^-1
    double* ninv = nullptr;  // [L]
};
struct NttTablesU {   // U64 path / phantom format
    uint64_t* tw = nullptr;     // [L][N]
    uint64_t* tws = nullptr;
    uint64_t* itw = nullptr;
    uint64_t* itws = nullptr;
    uint64_t* ninv = nullptr;   // [L]
    uint64_t* ninvs = nullptr;
};

}  // namespace mfhe

namespace mfhe {
// The launch plan a phantom NTT call runs (MFHE_OPT_NTT_PLAN_EFFECTIVE; ntt_plans.hpp run_phantom follows it):
// 4 = the pipelined single pass (N = 2^14, FP64, context limb table), 1 = one pass per polynomial (plain), 2 = two
// passes.  plan: MFHE_OPT_NTT_PLAN (0 / 3 auto, 1 single, 2 two passes from log_n 12).
inline int ntt_phantom_plan(bool f64, int logN, int plan, bool limbs) {
    const bool autoplan = plan == 0 || plan == 3;
    if (f64 && logN == 14 && limbs && autoplan) return 4;
    const bool two = logN > 14 || (plan == 2 && logN >= 12) || (autoplan && logN == 14);
    return two ? 2 : 1;
}
}  // namespace mfhe

struct mfhe_ctx {
    int L = 0;
    int logN = 0;
    uint64_t N = 0;
    int conv = 0;
    int arith = MFHE_ARITH_AUTO;  // effective: F64 or U64
    bool u60_ok = false;          // every modulus < 2^60: U64 NTTs may run ArithU60
    int ntt_u60 = 1;              // MFHE_OPT_NTT_U60
    bool f64_ok = false;          // every q < 2^50
    double delta = 0.0;
    int device = 0;
    std::vector<uint64_t> moduli;
    int64_t ntt_chunk_bytes = 240ll << 20;  // measured best at N = 2^15..2^17 (profiles/r02_chunk.txt)
    int ntt_plan = 0;
    int ntt_wg_per_cu = 16;  // NTT pass grid: workgroups per CU (0 = occupancy, 16 = one tile per WG; measured best)
    int ntt_pack = 0;        // MFHE_OPT_NTT_PACK (measured slower, kept opt-in: DESIGN.md §3.1)
    // MFHE_OPT_NTT_PREFETCH: 1 = persistent passes load the next tile into registers first (slower, r01);
    // 2 (default) = FP64 forward column pass with the next tile's LDS-DMA in flight (ntt_coldb.hpp, +0.5% C3, r02)
    int ntt_prefetch = 2;
    int num_cus = 256;
    int8_t* d_wVdig = nullptr;   // [L][wD][512][512] balanced base-256 digits of V   (i8 MFMA W-CRT)
    int8_t* d_wVidig = nullptr;  // same for V^-1
    uint64_t* d_wrtab = nullptr; // [L][2 wD - 1][2] (256^s mod q, Shoup)
    int wD = 0;                  // 0: no MFMA tables (some q <= 2^27); else the plane stride (max digits)
    std::vector<int> wDl;        // digits limb l needs (<= wD): its higher planes are all zero
    double* d_wepi = nullptr;    // [L][8] FP64 epilogue constants (gemm.hip GemmEpiF), null: integer epilogue
    int8_t* d_wZdig = nullptr;   // [L][wD][256][256] digits of Z[i][k] = zeta^((i+1)(k+1)) (factored forward W-CRT)
    double* d_wfold = nullptr;   // [L][16] factored forward fold constants (gemm.hip mfma_digitize_fold_kernel)
    int8_t* d_wZidig = nullptr;  // [L][wD][256][256] digits of zeta^-((i+1)(k+1)) (factored inverse W-CRT)
    double* d_wifold = nullptr;  // [L][16] factored inverse constants (q, 1/q, lam1[2][3], lam2[2][3])
    double* d_wiz = nullptr;     // [L][48] x1, x2 (zeta^-255, zeta^-256), pad, x1^(16j+1), x2^(16j+1) for j < 16
    uint8_t* d_wphi = nullptr;   // [320] packed Phi_771 rows: byte r2 - 1 (r2 = 1..256; r2 = 0 at byte 256) holds
                                 // phi_r2, phi_(r2-1), phi_(r2+257), phi_(r2+256) as (value + 1) at bits 0, 2, 4, 6
    int wcrt_mfma = 1;           // MFHE_OPT_WCRT_MFMA
    int wcrt_pipe = 0;           // MFHE_OPT_WCRT_PIPE
    int cgemm_mfma = 2;          // MFHE_OPT_CGEMM_MFMA
    int he_fused = 1;            // MFHE_OPT_HE_FUSED
    int limb_base = 0;           // residue shard: global index of this context's limb 0 (mfhe_ctx_set_limb_shard)
    int limbs_total = 0;         // residue shard: L of the whole parameter set (0 = this context's L)
    void* gemm_ws = nullptr;     // B digit planes for the MFMA GEMM, grown on demand
    size_t gemm_ws_bytes = 0;
    // MFHE_OPT_HE_STREAMS (include/mfhe.h): how encode / decode run their two independent W-CRT chains (re / im):
    // side stream (fork / join by events) or one grid per step over both components; the second component's GEMM
    // has its own digit planes
    int he_streams = 3;
    int enc_a_direct = 1;         // MFHE_OPT_ENC_A_DIRECT
    int enc_e_small = 1;          // MFHE_OPT_ENC_E_SMALL
    hipStream_t he_side = nullptr;
    hipEvent_t he_fork = nullptr, he_join = nullptr;
    void* gemm_ws2 = nullptr;
    size_t gemm_ws2_bytes = 0;

    mfhe::LimbConst* d_limbs = nullptr;  // [L]
    uint64_t* d_dmod = nullptr;          // [L][3] phantom DModulus {value, const_ratio[2]}

    // phantom convention tables (psi = minimal primitive 2N-th root)
    mfhe::NttTablesF ph_f;
    mfhe::NttTablesU ph_u;
    // GL / cyclic tables (network root psi' = beta^2, beta = first-found psi4n)
    mfhe::NttTablesF gl_f;
    mfhe::NttTablesU gl_u;
    double *gl_pre_f = nullptr, *gl_post_f = nullptr, *cyc_pre_f = nullptr, *cyc_post_f = nullptr;  // [L][N]
    uint64_t *gl_pre_u = nullptr, *gl_pre_us = nullptr, *gl_post_u = nullptr, *gl_post_us = nullptr;
    uint64_t *cyc_pre_u = nullptr, *cyc_pre_us = nullptr, *cyc_post_u = nullptr, *cyc_post_us = nullptr;
    uint32_t *gl_perm = nullptr, *gl_inv_perm = nullptr;  // [N]

    // wide CRT tables (encoder.cu:341-421), W words
    int W = 0;
    uint64_t* d_crt_M = nullptr;      // [L][W]  M_k = Q / q_k
    uint64_t* d_crt_inv = nullptr;    // [L][2]  (inv_k, shoup(inv_k))
    double* d_crt_qinv = nullptr;     // [L]     1/q_k (quotient estimate)
    uint64_t* d_crt_Q = nullptr;      // [W]
    uint64_t* d_crt_Qhalf = nullptr;  // [W]
    uint64_t* d_rns_mu = nullptr;     // [L][2] (q, floor(2^64/q))
    uint64_t* d_r64 = nullptr;        // [L]     2^64 mod q
    bool crt_qbig = false;            // Q_half >= 2^64
    mfhe::CrtLimbF* d_crt_lf = nullptr;  // [L] FP64 compose constants (null: some q >= 2^50 or even)

    // W axis (MFHE_CONV_WCRT), phi = 512
    static constexpr int PHI = 512;
    uint64_t* d_wV = nullptr;      // [L][512][512]  V_l[w][r]
    uint64_t* d_wVinv = nullptr;   // [L][512][512]  V_l^-1[r][w] (row-major)
    double2* d_wdV = nullptr;      // [512][512]     complex W-DFT
    double2* d_wdVinv = nullptr;   // [512][512]     its inverse (complex Gauss-Jordan)
    // factored W-DFT (MFHE_OPT_CGEMM_MFMA = 2, gemm.hip): zeta = e^(2 pi i / 257)
    double2* d_wdZ = nullptr;      // [256][256] zeta^((i+1)(k+1))
    double2* d_wdZi = nullptr;     // [256][256] zeta^-((i+1)(k+1))
    double2* d_wdlam = nullptr;    // [2][2][3]  lam1 / lam2 [a'][t] of the inverse (771^-1 omega^-at differences)
    double2* d_wdxp = nullptr;     // [2][256]   zeta^(-255 b), zeta^(-256 b), b = 1..256
    int8_t* d_wdphi = nullptr;     // [513]      Phi_771 coefficients
    // the forward factored W-DFT's 257-point DFTs by Rader's algorithm (gemm.hip wdft_rader_kernel, r06), g = 3:
    double2* d_wdrad = nullptr;    // [2][256]   FFT_256(zeta^(+-g^-k mod 257)) / 256: forward, inverse
    int16_t* d_wdgp = nullptr;     // [2][256]   g^n mod 257, g^-m mod 257
    void* wd_ws = nullptr;         // factored inverse W-DFT (c0, c1) per column, grown on demand
    size_t wd_ws_bytes = 0;
    double2 *d_encV = nullptr, *d_encVT = nullptr, *d_encVi = nullptr, *d_encViT = nullptr;  // [n][n]

    int trace_split = 2;              // MFHE_OPT_TRACE_SPLIT: split-digit kernel (2 MFMA, 1 VALU) when every q < 2^45


    // pipeline workspace (allocated on first use / mfhe_ctx_reserve_workspace)
    void* ws = nullptr;
    size_t ws_bytes = 0;

    std::vector<void*> allocs;  // everything above, freed at destroy
};
