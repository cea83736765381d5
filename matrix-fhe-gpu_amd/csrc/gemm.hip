// gemm.hip -- see gemm.hpp.
#include "gemm.hpp"
#include "mfhe_ctx.hpp"

namespace mfhe {

using u128 = unsigned __int128;

constexpr int TM = 64, TP = 64, TK = 16, NTH = 256;

__device__ __forceinline__ uint64_t b_off(uint64_t k, uint32_t p, uint64_t sK, uint64_t sY, int log_n) {
    return k * sK + (uint64_t)(p >> log_n) * sY + (p & ((1u << log_n) - 1));
}

// (hi:lo) mod q by folding hi with r64 = 2^64 mod q, then one Barrett step.
__device__ __forceinline__ uint64_t mod_u128(uint64_t hi, uint64_t lo, uint64_t q, uint64_t mu, uint64_t r64) {
    while (hi) {
        const u128 t = (u128)hi * r64 + lo;
        hi = (uint64_t)(t >> 64);
        lo = (uint64_t)t;
    }
    uint64_t r = lo - __umul64hi(lo, mu) * q;
    return r >= q ? r - q : r;
}

__global__ __launch_bounds__(NTH) void mod_gemm_kernel(ModGemmArgs a) {
    __shared__ uint64_t As[TM][TK + 1];
    __shared__ uint64_t Bs[TK][TP];
    const int l = blockIdx.z;
    const int m0 = blockIdx.y * TM;
    const uint32_t p0 = blockIdx.x * TP;
    const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
    const uint64_t* A = a.A + (uint64_t)l * a.aL;
    const uint64_t* B = a.B + (uint64_t)l * a.bL;
    uint64_t acc_lo[4][4], acc_hi[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc_lo[i][j] = acc_hi[i][j] = 0;

    for (int k0 = 0; k0 < a.K; k0 += TK) {
#pragma unroll
        for (int e = 0; e < (TM * TK) / NTH; ++e) {   // A tile 64 x 16
            const int idx = t + e * NTH, r = idx / TK, c = idx % TK;
            const int m = m0 + r, k = k0 + c;
            As[r][c] = (m < a.M && k < a.K) ? A[(uint64_t)m * a.K + k] : 0;
        }
#pragma unroll
        for (int e = 0; e < (TK * TP) / NTH; ++e) {   // B tile 16 x 64 (coalesced along p)
            const int idx = t + e * NTH, r = idx / TP, c = idx % TP;
            const int k = k0 + r;
            const uint32_t p = p0 + c;
            Bs[r][c] = (k < a.K && p < a.P) ? B[b_off(k, p, a.sbK, a.sbY, a.log_n)] : 0;
        }
        __syncthreads();
#pragma unroll 4
        for (int k = 0; k < TK; ++k) {
            uint64_t av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) av[i] = As[ty + 16 * i][k];
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = Bs[k][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const u128 pr = (u128)av[i] * bv[j];
                    const uint64_t lo = (uint64_t)pr, hi = (uint64_t)(pr >> 64);
                    acc_lo[i][j] += lo;
                    acc_hi[i][j] += hi + (acc_lo[i][j] < lo);
                }
        }
        __syncthreads();
    }
    const uint64_t q = a.qmu[2 * l], mu = a.qmu[2 * l + 1], r64 = a.r64[l];
    uint64_t* C = a.C + (uint64_t)l * a.cL;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty + 16 * i;
        if (m >= a.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t p = p0 + tx + 16 * j;
            if (p >= a.P) continue;
            C[b_off(m, p, a.scM, a.scY, a.log_n)] = mod_u128(acc_hi[i][j], acc_lo[i][j], q, mu, r64);
        }
    }
}

__global__ __launch_bounds__(NTH) void cgemm_kernel(CGemmArgs a) {
    __shared__ double2 As[TM][TK + 1];
    __shared__ double2 Bs[TK][TP];
    const int bt = blockIdx.z;
    const int m0 = blockIdx.y * TM;
    const uint32_t p0 = blockIdx.x * TP;
    const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
    const double2* A = a.A + (uint64_t)bt * a.aB;
    const double2* B = a.B + (uint64_t)bt * a.bB;
    double accr[4][4], acci[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) accr[i][j] = acci[i][j] = 0.0;
    for (int k0 = 0; k0 < a.K; k0 += TK) {
#pragma unroll
        for (int e = 0; e < (TM * TK) / NTH; ++e) {
            const int idx = t + e * NTH, r = idx / TK, c = idx % TK;
            const int m = m0 + r, k = k0 + c;
            As[r][c] = (m < a.M && k < a.K) ? A[(uint64_t)m * a.K + k] : make_double2(0, 0);
        }
#pragma unroll
        for (int e = 0; e < (TK * TP) / NTH; ++e) {
            const int idx = t + e * NTH, r = idx / TP, c = idx % TP;
            const int k = k0 + r;
            const uint32_t p = p0 + c;
            Bs[r][c] = (k < a.K && p < a.P) ? B[b_off(k, p, a.sbK, a.sbY, a.log_n)] : make_double2(0, 0);
        }
        __syncthreads();
#pragma unroll 4
        for (int k = 0; k < TK; ++k) {
            double2 av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) av[i] = As[ty + 16 * i][k];
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = Bs[k][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    // acc += a*b, same term order as cuCmul + add (encoder.cu:323, HE.cu:1168-1169)
                    accr[i][j] += av[i].x * bv[j].x - av[i].y * bv[j].y;
                    acci[i][j] += av[i].x * bv[j].y + av[i].y * bv[j].x;
                }
        }
        __syncthreads();
    }
    double2* C = a.C + (uint64_t)bt * a.cB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty + 16 * i;
        if (m >= a.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t p = p0 + tx + 16 * j;
            if (p >= a.P) continue;
            C[b_off(m, p, a.scM, a.scY, a.log_n)] = make_double2(accr[i][j], acci[i][j]);
        }
    }
}

int launch_mod_gemm(const ModGemmArgs& a, int L, hipStream_t s) {
    dim3 grid((a.P + TP - 1) / TP, (a.M + TM - 1) / TM, L);
    hipLaunchKernelGGL(mod_gemm_kernel, grid, dim3(NTH), 0, s, a);
    MFHE_CHECK_LAUNCH("mod_gemm_kernel");
    return MFHE_OK;
}

int launch_cgemm(const CGemmArgs& a, int batch, hipStream_t s) {
    dim3 grid((a.P + TP - 1) / TP, (a.M + TM - 1) / TM, batch);
    hipLaunchKernelGGL(cgemm_kernel, grid, dim3(NTH), 0, s, a);
    MFHE_CHECK_LAUNCH("cgemm_kernel");
    return MFHE_OK;
}

}  // namespace mfhe
