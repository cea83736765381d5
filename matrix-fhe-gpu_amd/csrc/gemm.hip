// gemm.hip -- see gemm.hpp.
#include "gemm.hpp"
#include "mfhe_ctx.hpp"
#include "ring_row.hpp"

#ifndef MFHE_DEC_WG_CU
#define MFHE_DEC_WG_CU 1   // decrypt-fused digitize: minimum workgroups per CU for the register budget (A/B knob)
#endif
#ifndef MFHE_DEC_TW_LDS
#define MFHE_DEC_TW_LDS 0   // decrypt-fused digitize: ring twiddles read from LDS (A/B knob)
#endif
#ifndef MFHE_DEC_RING_C
#define MFHE_DEC_RING_C 0   // decrypt-fused digitize: 1 = ring_mul_row64_lds from layout-C loads (A/B knob)
#endif
#ifndef MFHE_DEC_SUBS
#define MFHE_DEC_SUBS 4   // decrypt-fused digitize: 16-row substeps loaded together (1, 2 or 4)
#endif
#ifndef MFHE_DEC_NT
#define MFHE_DEC_NT 1   // decrypt-fused digitize: the ciphertext loads nontemporal (read once; 0 for A/B)
#endif
#ifndef MFHE_DEC_SPLIT
#define MFHE_DEC_SPLIT 4   // decrypt-fused digitize: workgroups per (row, limb), each 8 / MFHE_DEC_SPLIT panels
#endif

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

// ---------------- FP64 MFMA complex GEMM (W-DFT, XY transforms) ----------------
//
// C = A B over complex doubles as four real products on v_mfma_f64_16x16x4_f64:
//   Cr += Ar Br + (-Ai) Bi,  Ci += Ar Bi + Ai Br.
// A workgroup computes a 64 x 64 tile of C (four 32 x 32 wave tiles of 2 x 2 MFMA blocks); each
// 16-deep K stage of A and B goes global -> registers -> LDS (split into re / im planes) one stage
// ahead of the MFMAs that read it.  Products are exact-rounded f64 FMAs, so the sum differs from the
// oracle's mul-then-add order by ~1e-16 relative per term -- the FP_TOL parity of the VALU kernel
// above, which stays selectable (MFHE_OPT_CGEMM_MFMA = 0).
// Fragment maps (f64 16x16x4): A lane l = A[l&15][k=l>>4], B lane l = B[k=l>>4][l&15],
// C/D reg j of lane l = C[(l>>4) + 4j][l&15].
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int CKT = 16;          // K per LDS stage
constexpr int CAP = CKT + 1;     // A plane row pitch (doubles): spreads a fragment's 16 rows over the banks

// omega^e, omega = e^(2 pi i / 3) (the order-3 root of the factored W-DFT)
__device__ __forceinline__ double2 omega3(int e) {
    constexpr double h = 0.86602540378443864676;   // sqrt(3) / 2
    return e == 0 ? make_double2(1.0, 0.0) : make_double2(-0.5, e == 1 ? h : -h);
}
__device__ __forceinline__ double2 cmul(double2 x, double2 y) {
    return make_double2(__fma_rn(x.x, y.x, -x.y * y.y), __fma_rn(x.x, y.y, x.y * y.x));
}
// lanes l <-> l ^ 1 (DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ double dpp_swap1(double x) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, true),
                            __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, true));
}

// one output of the factored inverse W-DFT: interleaved complex, or planar (CGemmArgs::Cim)
__device__ __forceinline__ void cstore(const CGemmArgs& a, uint64_t idx, double re, double im) {
    if (a.Cim) {
        ((double*)a.C)[idx] = re;
        a.Cim[idx] = im;
    } else {
        a.C[idx] = make_double2(re, im);
    }
}

// FAC (a.fac): 0 dense; 1 / 2 the factored forward / inverse W-DFT (gemm.hpp CGemmArgs::fac)
template <int FAC>
__global__ __launch_bounds__(NTH, 2) void cgemm_mfma_kernel(CGemmArgs a) {
    __shared__ double Ar[2][TM * CAP], Ai[2][TM * CAP];   // [row][k]
    __shared__ double Br[2][CKT * TP], Bi[2][CKT * TP];   // [k][col]
    const int bt = blockIdx.z;
    const int m0 = blockIdx.y * TM;
    const uint32_t p0 = blockIdx.x * TP;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 32, wp = (w & 1) * 32, r = lane & 15, kq = lane >> 4;
    const double2* A = a.A + (uint64_t)bt * a.aB;
    const double2* B = a.B + (uint64_t)bt * a.bB;
    double2 ra[(TM * CKT) / NTH], rb[(CKT * TP) / NTH];
    auto load = [&](int k0) {
#pragma unroll
        for (int e = 0; e < (TM * CKT) / NTH; ++e) {   // A stage 64 x 16, 16 consecutive k per row
            const int idx = t + e * NTH, m = m0 + (idx >> 4), k = k0 + (idx & 15);
            ra[e] = (m < a.M && k < a.K) ? A[(uint64_t)m * a.K + k] : make_double2(0, 0);
        }
#pragma unroll
        for (int e = 0; e < (CKT * TP) / NTH; ++e) {   // B stage 16 x 64, coalesced along p
            const int idx = t + e * NTH, k = k0 + (idx >> 6);
            const uint32_t p = p0 + (idx & 63);
            if constexpr (FAC == 0) {
                rb[e] = (k < a.K && p < a.P) ? B[b_off(k, p, a.sbK, a.sbY, a.log_n)] : make_double2(0, 0);
            } else if constexpr (FAC == 1) {
                // F_a[r2] = omega^(a t) in[r2] + omega^(a ((t + 2) mod 3)) in[r2 + 257], r2 = k + 1, t = r2 mod 3
                // interleaved columns 2 p + a': lanes 2p, 2p + 1 load the same two inputs (one fetch per pair)
                const bool live = p < a.P;
                const int ap = p & 1;
                const uint32_t pc = live ? p >> 1 : 0;
                const int r2 = k + 1, t3 = r2 % 3, r3 = r2 + 257 < 512 ? r2 + 257 : 511;
                const double2 x1 = B[(uint64_t)r2 * a.Pf + pc], x2 = B[(uint64_t)r3 * a.Pf + pc];
                const double2 f1 = cmul(omega3(((ap + 1) * t3) % 3), x1);
                const double2 f2 = r2 + 257 < 512 ? cmul(omega3(((ap + 1) * ((t3 + 2) % 3)) % 3), x2) : make_double2(0, 0);
                rb[e] = live ? make_double2(f1.x + f2.x, f1.y + f2.y) : make_double2(0, 0);
            } else {
                // y[a'][b] = in[a' 256 + k][p] in interleaved columns 2 p + a'
                const bool live = p < a.P;
                const uint32_t pc = live ? p >> 1 : 0;
                const double2 y = B[(uint64_t)((p & 1) * 256 + k) * a.Pf + pc];
                rb[e] = live ? y : make_double2(0, 0);
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int e = 0; e < (TM * CKT) / NTH; ++e) {
            const int idx = t + e * NTH, o = (idx >> 4) * CAP + (idx & 15);
            Ar[buf][o] = ra[e].x;
            Ai[buf][o] = ra[e].y;
        }
#pragma unroll
        for (int e = 0; e < (CKT * TP) / NTH; ++e) {
            const int idx = t + e * NTH;
            Br[buf][idx] = rb[e].x;
            Bi[buf][idx] = rb[e].y;
        }
    };
    v4d cr[2][2], ci[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) cr[i][j] = ci[i][j] = v4d{0, 0, 0, 0};
    const int nk = (a.K + CKT - 1) / CKT;
    load(0);
    store(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load((kt + 1) * CKT);
#pragma unroll
        for (int ks = 0; ks < CKT / 4; ++ks) {
            const int k = ks * 4 + kq;
            double ar[2], ai[2], nai[2], br[2], bi[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                ar[i] = Ar[buf][(wm + 16 * i + r) * CAP + k];
                ai[i] = Ai[buf][(wm + 16 * i + r) * CAP + k];
                nai[i] = -ai[i];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                br[j] = Br[buf][k * TP + wp + 16 * j + r];
                bi[j] = Bi[buf][k * TP + wp + 16 * j + r];
            }
            // first terms of all eight accumulators, then the second terms: no back-to-back dependence
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    cr[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[i], br[j], cr[i][j], 0, 0, 0);
                    ci[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[i], bi[j], ci[i][j], 0, 0, 0);
                }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    cr[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(nai[i], bi[j], cr[i][j], 0, 0, 0);
                    ci[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[i], br[j], ci[i][j], 0, 0, 0);
                }
        }
        if (kt + 1 < nk) store(buf ^ 1);
        __syncthreads();
    }
    double2* C = a.C + (uint64_t)bt * a.cB;
    if constexpr (FAC == 1) {
        // out[a' 256 + m][p] = GEMM + F_a[0], F_a[0] = in[0] + omega^(2 a) in[257]
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t c = p0 + wp + 16 * j + r;
            if (c >= a.P) continue;
            const int ap = c & 1;
            const uint32_t p = c >> 1;
            const double2 f = cmul(omega3((2 * (ap + 1)) % 3), B[257ull * a.Pf + p]), x0 = B[p];
            const double2 add = make_double2(x0.x + f.x, x0.y + f.y);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int m = m0 + wm + 16 * i + kq + 4 * g;
                    C[(uint64_t)(ap * 256 + m) * a.scM + p] = make_double2(cr[i][j][g] + add.x, ci[i][j][g] + add.y);
                }
        }
        return;
    } else if constexpr (FAC == 2) {
        // E_a'[r2] (r2 = m + 1) in lanes 2p + a'; h_r2 = sum_a lam1[a][t] E_a, h_(r2+257) = sum_a lam2[a][t] E_a
        // (t = r2 mod 3), f_j = h_j - c0 phi_j - c1 phi_(j-1): lane a' = 0 writes row r2, a' = 1 row r2 + 257
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t c = p0 + wp + 16 * j + r;
            const int ap = c & 1;
            const uint32_t p = c >> 1;
            const bool live = c < a.P;   // the same for both lanes of a pair (P even)
            const uint32_t pc = live ? p : 0;
            const double2 c0 = a.cc[2ull * pc], c1 = a.cc[2ull * pc + 1];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int r2 = m0 + wm + 16 * i + kq + 4 * g + 1;
                    const int t3 = r2 % 3;
                    const double2 own = a.lam[(ap * 2 + ap) * 3 + t3], oth = a.lam[((1 - ap) * 2 + ap) * 3 + t3];
                    const double2 e = make_double2(cr[i][j][g], ci[i][j][g]);
                    const double2 po = cmul(own, e), ps = cmul(oth, e);
                    const double hx = po.x + dpp_swap1(ps.x), hy = po.y + dpp_swap1(ps.y);
                    const int jr = ap ? r2 + 257 : r2;
                    if (live && jr < 512) {
                        const double f0 = (double)a.phi[jr], f1 = (double)a.phi[jr - 1];
                        cstore(a, (uint64_t)jr * a.scM + p, hx - c0.x * f0 - c1.x * f1, hy - c0.y * f0 - c1.y * f1);
                    }
                }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t p = p0 + wp + 16 * j + r;
            if (p >= a.P) continue;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int m = m0 + wm + 16 * i + kq + 4 * g;
                if (m < a.M) C[b_off(m, p, a.scM, a.scY, a.log_n)] = make_double2(cr[i][j][g], ci[i][j][g]);
            }
        }
}

// factored inverse W-DFT, rows r2 = 0, 255, 256 of E_a by dot products.  One thread per (column p, a', 32-row
// chunk q): lane = 2 p_local + a' (16 columns per block), q = thread / 32.  S0 = sum y, S1 = sum x1^b y,
// S2 = sum x2^b y over b = 32 q + 1 .. 32 q + 32; the chunks reduce through LDS, a' by a lane exchange; then
// f_0, f_257 and (c0, c1) as in mfma_digitize_ifold_kernel (complex, no reduction mod q).
__global__ __launch_bounds__(256) void cwdft_inv_dots_kernel(CGemmArgs a, const double2* __restrict__ in,
                                                             const double2* __restrict__ xpow) {
    __shared__ double2 red[3][8][32];
    const int lane = threadIdx.x & 31, q = threadIdx.x >> 5;   // 32 threads = 16 columns x 2 a'; 8 chunks
    const uint32_t p = blockIdx.x * 16 + (lane >> 1);
    const int ap = lane & 1;
    const bool live = p < a.Pf;
    const uint32_t pc = live ? p : 0;
    double2 s0 = make_double2(0, 0), s1 = s0, s2 = s0;
#pragma unroll 8
    for (int i = 0; i < 32; ++i) {
        const int k = q * 32 + i;   // b = k + 1
        const double2 y = in[(uint64_t)(ap * 256 + k) * a.Pf + pc];
        const double2 z1 = xpow[k], z2 = xpow[256 + k];
        s0.x += y.x;
        s0.y += y.y;
        s1.x = __fma_rn(z1.x, y.x, __fma_rn(-z1.y, y.y, s1.x));
        s1.y = __fma_rn(z1.x, y.y, __fma_rn(z1.y, y.x, s1.y));
        s2.x = __fma_rn(z2.x, y.x, __fma_rn(-z2.y, y.y, s2.x));
        s2.y = __fma_rn(z2.x, y.y, __fma_rn(z2.y, y.x, s2.y));
    }
    red[0][q][lane] = s0;
    red[1][q][lane] = s1;
    red[2][q][lane] = s2;
    __syncthreads();
    if (q != 0) return;
    double2 e[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        double2 acc = red[v][0][lane];
#pragma unroll
        for (int c = 1; c < 8; ++c) acc = make_double2(acc.x + red[v][c][lane].x, acc.y + red[v][c][lane].y);
        e[v] = acc;
    }
    double2 o[3];
#pragma unroll
    for (int v = 0; v < 3; ++v) o[v] = make_double2(__shfl_xor(e[v].x, 1), __shfl_xor(e[v].y, 1));
    const double2* e1 = ap ? o : e;   // a = 1
    const double2* e2 = ap ? e : o;   // a = 2
    auto lam = [&](int kind, int aa, int t3) { return a.lam[(kind * 2 + aa) * 3 + t3]; };
    auto add2 = [](double2 x, double2 y) { return make_double2(x.x + y.x, x.y + y.y); };
    const double2 h0 = add2(cmul(lam(0, 0, 0), e1[0]), cmul(lam(0, 1, 0), e2[0]));       // r2 = 0
    const double2 h257 = add2(cmul(lam(1, 0, 0), e1[0]), cmul(lam(1, 1, 0), e2[0]));
    const double2 h512 = add2(cmul(lam(1, 0, 0), e1[1]), cmul(lam(1, 1, 0), e2[1]));     // r2 = 255, t = 0
    const double2 h513 = add2(cmul(lam(1, 0, 1), e1[2]), cmul(lam(1, 1, 1), e2[2]));     // r2 = 256, t = 1
    const double p511 = a.phi[511], p0 = a.phi[0], p256 = a.phi[256], p257 = a.phi[257];
    const double2 c1 = h513;
    const double2 c0 = make_double2(h512.x - c1.x * p511, h512.y - c1.y * p511);
    if (!live) return;
    if (ap == 0) {
        cstore(a, p, h0.x - c0.x * p0, h0.y - c0.y * p0);
        ((double2*)a.cc)[2ull * p] = c0;
        ((double2*)a.cc)[2ull * p + 1] = c1;
    } else {
        cstore(a, 257ull * a.scM + p, h257.x - c0.x * p257 - c1.x * p256, h257.y - c0.y * p257 - c1.y * p256);
    }
}

int launch_cwdft_inv_dots(const CGemmArgs& a, const double2* in, const double2* xpow, hipStream_t s) {
    hipLaunchKernelGGL(cwdft_inv_dots_kernel, dim3((a.Pf + 15) / 16), dim3(256), 0, s, a, in, xpow);
    MFHE_CHECK_LAUNCH("cwdft_inv_dots_kernel");
    return MFHE_OK;
}

// ---------------- i8 MFMA modular GEMM (W-CRT, M = K = 512) ----------------
//
// Exact integer product through v_mfma_i32_32x32x32_i8: every operand x < q < 2^(8D-1) is written in
// D balanced base-256 digits x = sum_i d_i 256^i, d_i in [-128, 127].  For each s = i + j the
// digit-pair products accumulate in one i32 tile acc_s = sum_{i+j=s} A_i B_j (|acc_s| <= D * 2^14 * 512
// < 2^26 for D <= 8, exact), and the epilogue folds C = sum_s acc_s * (256^s mod q) mod q.
// A's digit planes are built once per context; B is split by mfma_digitize_kernel into a
// [L][D][Ppad][K] workspace (K contiguous) so both fragments are single 16-byte loads per lane
// (probe: tools/microbench/mfma_i8_probe.hip; any k order shared by A and B is valid).
constexpr int MK = 512;   // K of the W-CRT GEMM

using v4i = int __attribute__((ext_vector_type(4)));
using v16i = int __attribute__((ext_vector_type(16)));

// Digit planes are "k-panel-major": [K/32][rows][32] bytes, so one 32-k panel of 64 consecutive rows (or
// columns) is 2 KiB of contiguous memory: every fragment load (16 B per lane, lanes over rows and k halves)
// and every digitize store below is a fully coalesced sweep.
//
// Balanced base-256 digits by offset: x = sum d_i 256^i with d_i in [-128, 127] iff
// y = x + 128 (256^D - 1) / 255 = x + 0x8080..80 has bytes d_i + 128, so d_i = byte_i(y) ^ 0x80 as an i8.
// Valid for -0x80..80 <= x <= 0x7F..7F (D bytes); the fold kernel's |x| <= q/2 + 1 is well inside.
template <int D>
__device__ __forceinline__ uint64_t balanced_bytes(double v) {   // v integral, |v| < 2^51
    constexpr double kMagic = 6755399441055744.0;                 // 1.5 * 2^52: bits(v + M) - bits(M) = v
    constexpr uint64_t kOff = 0x8080808080808080ull >> (64 - 8 * D);
    return (uint64_t)__double_as_longlong(v + kMagic) - ((uint64_t)__double_as_longlong(kMagic) - kOff);
}
// Byte transpose of digit words into digit-plane words (r06): rows 4c .. 4c + 3 of y (each row's D digit bytes in
// its low D bytes) give word c of every plane i = byte i of those four rows.  v_perm_b32 picks 4 of the 8 bytes of
// (S0:S1): rows (0, 1) and (2, 3) interleaved for two planes at once, then the halves joined -- three perms per two
// planes and four rows, instead of a shift, mask and or per byte.
template <int D, int R>
__device__ __forceinline__ void pack_planes(const uint64_t (&y)[R], uint32_t (&pk)[D][R / 4]) {
#pragma unroll
    for (int c = 0; c < R / 4; ++c)
#pragma unroll
        for (int pi = 0; pi < D; pi += 2) {
            const int sh = pi < 4 ? 0 : 32;
            const uint32_t i = (uint32_t)(pi & 3), j = i + 1;
            const uint32_t sel = i | ((4 + i) << 8) | (j << 16) | ((4 + j) << 24);
            const uint32_t t01 = __builtin_amdgcn_perm((uint32_t)(y[4 * c + 1] >> sh), (uint32_t)(y[4 * c] >> sh), sel);
            const uint32_t t23 = __builtin_amdgcn_perm((uint32_t)(y[4 * c + 3] >> sh), (uint32_t)(y[4 * c + 2] >> sh), sel);
            pk[pi][c] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
            if (pi + 1 < D) pk[pi + 1][c] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
        }
}

// digit planes the GEMM reads per limb (max(limbD, 5), <= D): planes past it are never read, so never written
struct PlaneCounts {
    uint8_t n[64];   // limbs >= 64: all D
};
static PlaneCounts plane_counts(const ModGemmArgs& a, int L) {
    PlaneCounts pc;
    for (int l = 0; l < 64; ++l) pc.n[l] = (uint8_t)(a.limbD && l < L ? std::max(a.limbD[l], 5) : a.D);
    return pc;
}

// one thread: column p (of Ppad; zero past P), one 32-k panel; B (k, p) via the (sbK, sbY, log_n) map
template <int D>
__global__ __launch_bounds__(256) void mfma_digitize_kernel(const uint64_t* __restrict__ B, uint64_t bL,
                                                            uint64_t sbK, uint64_t sbY, int log_n, uint32_t P,
                                                            uint32_t Ppad, int8_t* __restrict__ out, PlaneCounts pc) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    const int kc = blockIdx.y;
    const int l = blockIdx.z;
    if (p >= Ppad) return;
    const uint64_t* Bl = B + (uint64_t)l * bL;
    const uint64_t col = (uint64_t)(p >> log_n) * sbY + (p & ((1u << log_n) - 1));
    // plane i, bytes 4c..4c+3 of the panel's 32 k.  Balanced digits by the offset rule: the bytes of x + 0x80..80
    // (D bytes; x < 2^(8D - 1)) are the digits + 128, so byte ^ 0x80 is the digit mod 256 (r05: a shift-and-carry
    // loop per digit; the same bytes)
    constexpr uint64_t kOff = 0x8080808080808080ull >> (64 - 8 * D);
    uint64_t y[32];
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) {
        const uint64_t x = Bl[(uint64_t)(kc * 32 + kk) * sbK + (p < P ? col : 0)];
        y[kk] = (p < P ? x : 0) + kOff;
    }
    uint32_t pk[D][8];
    pack_planes<D, 32>(y, pk);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
        for (int c = 0; c < 8; ++c) pk[i][c] ^= 0x80808080u;
    const int nd = l < 64 ? pc.n[l] : D;
#pragma unroll
    for (int i = 0; i < D; ++i) {
        if (i >= nd) break;
        int8_t* o = out + (((uint64_t)l * D + i) * (MK / 32) + kc) * Ppad * 32 + (uint64_t)p * 32;
        *(v4i*)o = v4i{(int)pk[i][0], (int)pk[i][1], (int)pk[i][2], (int)pk[i][3]};
        *(v4i*)(o + 16) = v4i{(int)pk[i][4], (int)pk[i][5], (int)pk[i][6], (int)pk[i][7]};
    }
}

// ---- factored forward W-CRT (every q < 2^50) ----
// The 512 evaluation points are eta^e for the units e of Z_771 in the order e = 257 a + 3 b (a = 1, 2;
// b = 1..256; HE.cu:72-105, k_wntt_exp).  With omega = eta^257 (order 3) and zeta = eta^3 (order 257),
// x_w^r = omega^(a (r mod 3)) zeta^(b (r mod 257)), and since r < 512 < 771 each r2 = r mod 257 takes at
// most two r (r2 and r2 + 257):
//   out[a][b] = F_a[0] + sum_{k < 256} zeta^(b (k + 1)) F_a[k + 1],
//   F_a[r2]   = omega^(a (r2 mod 3)) in[r2] + omega^(a ((r2 + 2) mod 3)) in[r2 + 257]   (second term if < 512).
// That is a 256 x 256 GEMM over 2 P columns (a, p) instead of 512 x 512 over P: half the MACs, and the
// same linear map mod q, so bit-exact.  This kernel forms F_a (two FP64 modmuls per term), writes the
// digit planes of F_a[1..256] as the B operand ([L][D][8 panels][2 Ppad][32], column a' Ppad + p for
// a = a' + 1) and F_a[0] to d0[L][2][Ppad] for the GEMM epilogue.
// fold[l][16] = q, 1/q, omega^(a r1) [a'][r1], omega^(a ((r1 + 2) mod 3)) [a'][r1], all centred.
constexpr int FK = 256;   // K (and M) of the factored GEMM

// One thread: column p, one half (16 k) of a 32-k panel, both a; lane pairs share a column, so each
// 16-byte store completes a 1 KiB contiguous run per wave.  The digits need any representative of F_a mod q
// within the limb's digit range, so F_a is only reduced to the centred (-q/2, q/2] and split by the offset
// rule (balanced_bytes).
// SRC 1 (encode): B is not a residue matrix but the W-IDFT's doubles v[r][p] (row stride qf_row, element stride
// qf_step): each limb's residue is formed on the fly as round(v delta) mod q -- the RNS decompose
// (rns_decompose_kernel: llround, then the residue of the int64) fused away, exact for |v delta| < 2^63 (the
// centred FP64 reduction of the rounded double is exact while |x / q| < 2^51).  With any SRC the grid runs the
// limbs fastest (blockIdx.x), so the L blocks of one column range read the same doubles out of the L2.
// SRC 2 / 3 (encrypt): the uniform sampler's residue computed in place (seed from (w, limb, position) exactly as
// he.hip uniform_kernel, so no a[] in HBM), or the Gaussian noise read as one centred integer per coefficient.
struct FoldSrc {
    const double* qf = nullptr;
    uint64_t qf_row = 0, qf_step = 0;
    double delta = 0.0;
    const uint64_t* qmu = nullptr;   // SRC 2: [L][2] (q, floor(2^64 / q))
    int lbase = 0, Ltot = 0;
};
// PAIR (fused sources only): two components in one grid, blockIdx.x in [0, 2 L); the upper half writes fp's planes
// from fp's source (he.hip encode: re and im)
struct FoldPair {
    int L = 0;
    int8_t* out2 = nullptr;
    uint64_t* d02 = nullptr;
    const double* qf2 = nullptr;
};
template <int D, int SRC = 0, bool PAIR = false>
__global__ __launch_bounds__(256, 4) void mfma_digitize_fold_kernel(const uint64_t* __restrict__ B, uint64_t bL,
                                                                 uint64_t sbK, uint64_t sbY, int log_n, uint32_t P,
                                                                 uint32_t Ppad, const double* __restrict__ fold,
                                                                 int8_t* __restrict__ out, uint64_t* __restrict__ d0,
                                                                 PlaneCounts pc, FoldSrc fs = FoldSrc{},
                                                                 FoldPair fp = FoldPair{}) {
    constexpr bool QF = SRC != 0;
    static_assert(!PAIR || QF, "pair launches: fused sources only");
    const double* __restrict__ qf = fs.qf;
    const uint64_t qf_row = fs.qf_row, qf_step = fs.qf_step;
    const double delta = fs.delta;
    const uint32_t p = (QF ? blockIdx.y : blockIdx.x) * 128 + (threadIdx.x >> 1);
    const int hf = threadIdx.x & 1;
    const int kc = QF ? blockIdx.z : blockIdx.y;   // panel: r2 = 32 kc + 16 hf + 1 .. 32 kc + 16 hf + 16
    int lx = QF ? blockIdx.x : blockIdx.z;
    if constexpr (PAIR) {
        if (lx >= fp.L) {
            lx -= fp.L;
            out = fp.out2;
            d0 = fp.d02;
            qf = fp.qf2;
        }
    }
    const int l = lx;
    if (p >= Ppad) return;
    const double* fo = fold + (uint64_t)l * 16;
    LimbConst lc;
    lc.qf = fo[0];
    lc.qinv = fo[1];
    const ArithF64 ar(lc);
    double c1[2][3], c2[2][3];
#pragma unroll
    for (int ap = 0; ap < 2; ++ap)
#pragma unroll
        for (int r1 = 0; r1 < 3; ++r1) {
            c1[ap][r1] = fo[2 + 3 * ap + r1];
            c2[ap][r1] = fo[8 + 3 * ap + r1];
        }
    const uint64_t* Bl = B + (uint64_t)l * bL;
    const uint64_t col = (uint64_t)(p >> log_n) * sbY + (p & ((1u << log_n) - 1));
    const bool live = p < P;
    // unconditional loads (column 0 stands in for the padding columns, then zeroed): a load under `live ? :` is
    // a branch per load, each followed by its own vmcnt(0) -- the 32 loads of a thread ran one at a time
    const uint64_t cl = live ? col : 0;
    uint64_t uq = 0, umu = 0;
    if constexpr (SRC == 2) {
        uq = fs.qmu[2 * l];
        umu = fs.qmu[2 * l + 1];
    }
    // SRC 2: the sampler's LCG output for row r, (123456789 + ((r Ltot + lbase + l) << 2 log n) + p) A + C mod 2^64
    // (he.hip uniform_kernel).  It is affine in r: with the per-row step K = (Ltot << 2 log n) A, row r + 1's word is
    // row r's + K, and row r + 257's is row r's + 257 K -- 64-bit adds in the row loop instead of a 64-bit multiply
    // per value, the same words (sampled_row below; in(r) keeps the direct form for the d0 rows).
    uint64_t lcgK = 0, lcgK257 = 0;
    if constexpr (SRC == 2) {
        lcgK = ((uint64_t)fs.Ltot << (2 * log_n)) * 6364136223846793005ULL;
        lcgK257 = lcgK * 257ull;
    }
    auto lcg_seed = [&](int r) {
        const uint32_t pp = live ? p : 0;
        return (123456789ULL + (((uint64_t)r * (uint64_t)fs.Ltot + (uint64_t)(fs.lbase + l)) << (2 * log_n)) + pp) *
                   6364136223846793005ULL + 1442695040888963407ULL;
    };
    auto sampled = [&](uint64_t seed) {   // Barrett as uniform_kernel: [0, 3q), then two selects
        uint64_t v = seed - __umul64hi(seed, umu) * uq;
        v = v >= uq ? v - uq : v;
        v = v >= uq ? v - uq : v;
        return live ? ArithF64::from_u64(v) : 0.0;
    };
    auto in = [&](int r) {
        double x;
        const uint32_t pp = live ? p : 0;
        if constexpr (SRC == 1) {
            x = ar.reduce(round(qf[(uint64_t)r * qf_row + (uint64_t)pp * qf_step] * delta));
        } else if constexpr (SRC == 2) {
            return sampled(lcg_seed(r));
        } else if constexpr (SRC == 3) {
            x = qf[(uint64_t)r * qf_row + pp];
        } else {
            x = ArithF64::from_u64(Bl[(uint64_t)r * sbK + cl]);
        }
        return live ? x : 0.0;
    };
    uint32_t pk[2][D][4];
    uint32_t ylo[2][4], yhi[2][4];   // the current group of four rows' digit words
    const int rb = kc * 32 + hf * 16 + 1;
    // r06: F_a = omega^(a r1) (x1 + omega^(2a) x2) and omega^2 = -1 - omega, so with m = omega x2
    //   F_1 = omega^r1 (x1 - x2 - m),  F_2 = omega^(2 r1) (x1 + m)
    // -- three modmuls per r2 instead of four (|x1 - x2 - m| <= 3q: inside mulmod's |v| <= 4q); the same residues,
    // other representatives, so other digits but the same GEMM result mod q.  The weights omega^(a r1) are rotated
    // once to this thread's first r2 mod 3, so the unrolled loop indexes them by kk % 3 (the per-row selects by a
    // runtime r1 were ~200 of the kernel's ~1830 VALU instructions).
    const double omega = c1[0][1];
    const int r10 = rb % 3;
    double wr[2][3];
#pragma unroll
    for (int ap = 0; ap < 2; ++ap)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int e0 = j, e1 = (j + 1) % 3, e2 = (j + 2) % 3;   // (r10 + j) mod 3 for r10 = 0, 1, 2
            wr[ap][j] = r10 == 0 ? c1[ap][e0] : (r10 == 1 ? c1[ap][e1] : c1[ap][e2]);
        }
    uint64_t seed1 = 0;
    if constexpr (SRC == 2) seed1 = lcg_seed(rb);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
        const int r2 = rb + kk;
        double x1, x2r;
        if constexpr (SRC == 2) {
            x1 = sampled(seed1);
            x2r = sampled(seed1 + lcgK257);   // row r2 + 257 (unused past row 511)
            seed1 += lcgK;
        } else {
            x1 = in(r2);
            x2r = in(r2 + 257 < 512 ? r2 + 257 : 511);
        }
        const double x2 = r2 + 257 < 512 ? x2r : 0.0;
        const double m = ar.mulmod(x2, omega);
        const double fin[2] = {x1 - x2 - m, x1 + m};
#pragma unroll
        for (int ap = 0; ap < 2; ++ap) {
            const double v = ar.reduce(ar.mulmod(fin[ap], wr[ap][kk % 3]));   // |v| <= q/2 + eps
            const uint64_t y = balanced_bytes<D>(v);
            ylo[ap][kk & 3] = (uint32_t)y;
            yhi[ap][kk & 3] = (uint32_t)(y >> 32);
        }
        if ((kk & 3) == 3) {
            // byte transpose of four rows' digits into the planes' words: plane i's word = byte i of rows 0..3.
            // v_perm_b32 picks 4 of the 8 bytes of (S0:S1): first rows (0, 1) and (2, 3) interleaved for two planes
            // at once, then the two halves joined -- 3 perms per two planes instead of a shift, mask and or per byte
#pragma unroll
            for (int ap = 0; ap < 2; ++ap)
#pragma unroll
                for (int pi = 0; pi < D; pi += 2) {
                    const uint32_t* src = pi < 4 ? ylo[ap] : yhi[ap];
                    const uint32_t i = (uint32_t)(pi & 3), j = i + 1;
                    const uint32_t sel = i | ((4 + i) << 8) | (j << 16) | ((4 + j) << 24);
                    const uint32_t t01 = __builtin_amdgcn_perm(src[1], src[0], sel);
                    const uint32_t t23 = __builtin_amdgcn_perm(src[3], src[2], sel);
                    pk[ap][pi][kk >> 2] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
                    if (pi + 1 < D) pk[ap][pi + 1][kk >> 2] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
                }
        }
    }
    if (kc == 0 && hf == 0) {
        const double x1 = in(0), x2 = in(257);
#pragma unroll
        for (int ap = 0; ap < 2; ++ap)
            d0[((uint64_t)l * 2 + ap) * Ppad + p] = ar.canon(ar.mulmod(x1, c1[ap][0]) + ar.mulmod(x2, c2[ap][0]));
    }
    const int nd = l < 64 ? pc.n[l] : D;
#pragma unroll
    for (int ap = 0; ap < 2; ++ap)
#pragma unroll
        for (int i = 0; i < D; ++i) {
            if (i >= nd) break;
            int8_t* o = out + ((((uint64_t)l * D + i) * (FK / 32) + kc) * 2 * Ppad + (uint64_t)ap * Ppad + p) * 32 + hf * 16;
            const uint32_t* w = pk[ap][i];
            *(v4i*)o = v4i{(int)(w[0] ^ 0x80808080u), (int)(w[1] ^ 0x80808080u), (int)(w[2] ^ 0x80808080u),
                           (int)(w[3] ^ 0x80808080u)};
        }
}

// ---- factored inverse W-CRT (every q < 2^50; tools/wcrt_factor_check.py) ----
// V^-1 y is the 771-point inverse DFT of the 512 values (zeros at the 259 non-unit exponents), reduced mod
// Phi_771.  With the forward's e = 257 a + 3 b order, E_a[r2] = sum_{b=1..256} zeta^(-b r2) y[a][b] (r2 = 0..256) and
//   g_r = 771^-1 sum_a omega^(-a r) E_a[r mod 257]                       (r = 0..770)
//   h_j = g_j - g_(j+514) (j <= 256),  h_j = g_j - g_(j+257) (257 <= j <= 513)   (mod x^514 + x^257 + 1)
//   f_j = h_j - c0 phi_j - c1 phi_(j-1),  c1 = h_513, c0 = h_512 - c1 phi_511       (mod Phi_771, j < 512)
// j = r2, r2 + 257 and r2 + 514 share E_a[r2], so per GEMM row r2 = 1..256 (a 256 x 256 GEMM over 2 P columns
// interleaved as 2 p + a'): h_r2 = sum_a lam1[a][r2 mod 3] E_a[r2], h_(r2+257) = sum_a lam2[a][r2 mod 3] E_a[r2].
// The digitize kernel below also forms the rows r2 = 0 (-> f_0, f_257), 255 and 256 (-> c0, c1 per column) by
// dot products, so the GEMM epilogue writes the final f directly: half the MACs of the dense V^-1 product.
// One thread: column p = 16 blockIdx.x + lane / 4, a' = (lane >> 1) & 1, half panel hf = lane & 1 (16 k), k quarter
// = wave (two 32-k panels): lane l's 16-byte digit store lands at byte 16 l of a contiguous 1 KiB run.
template <int D>
__global__ __launch_bounds__(256) void mfma_digitize_ifold_kernel(ModGemmArgs a, uint32_t Ppad, PlaneCounts pc) {
    __shared__ double red[3][4][64];
    const int lane = threadIdx.x & 63, kq = threadIdx.x >> 6;
    const uint32_t p = blockIdx.x * 16 + (lane >> 2);
    const int ap = (lane >> 1) & 1, hf = lane & 1;
    const int l = blockIdx.y;
    typedef const __attribute__((address_space(4))) double* cdp_t;
    const cdp_t fo = (cdp_t)(a.ifold + (uint64_t)l * 16);
    LimbConst lc;
    lc.qf = fo[0];
    lc.qinv = fo[1];
    const ArithF64 ar(lc);
    // iz[l] = (x1, x2, pad[14], x1^(16 j + 1) for j < 16, x2^(16 j + 1) for j < 16), x1 = zeta^-255, x2 = zeta^-256
    const double* izl = a.iz + (uint64_t)l * 48;
    const double x1 = ((cdp_t)izl)[0], x2 = ((cdp_t)izl)[1];
    const double* zp = izl + 16;
    const uint64_t* Bl = a.B + (uint64_t)l * a.bL;
    const uint32_t nmask = (1u << a.log_n) - 1;
    const uint64_t col = (uint64_t)(p >> a.log_n) * a.sbY + (p & nmask);
    const bool live = p < a.P;
    const uint64_t cl = live ? col : 0;   // unconditional loads (see mfma_digitize_fold_kernel)
    const int nd = l < 64 ? pc.n[l] : D;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;   // E_a'[0], E_a'[255], E_a'[256] over this thread's 32 k
#pragma unroll 1
    for (int pn = 0; pn < 2; ++pn) {
        const int kc = 2 * kq + pn, k0 = kc * 32 + hf * 16;
        uint32_t pk[D][4];
        double v[16];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)   // b = k0 + kk + 1
            v[kk] = ArithF64::from_u64(Bl[(uint64_t)(ap * FK + k0 + kk) * a.sbK + cl]);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) v[kk] = live ? ar.reduce(v[kk]) : 0.0;
        // sum_b x^b v_b over this chunk (b = k0 + 1 + i) as x^(k0+1) * Horner(v, x) for x = zeta^-255, zeta^-256:
        // no per-element table, two independent chains (|h| <= q + 1 between steps: mulmod's range holds)
        double h1 = v[15], h2 = v[15], t0 = 0.0;
#pragma unroll
        for (int kk = 14; kk >= 0; --kk) {
            h1 = ar.mulmod(h1, x1) + v[kk];
            h2 = ar.mulmod(h2, x2) + v[kk];
        }
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) t0 += v[kk];   // |t0| <= 8 q < 2^53
        s0 = ar.reduce(s0 + t0);
        s1 = ar.reduce(s1 + ar.mulmod(h1, zp[(k0 >> 4)]));
        s2 = ar.reduce(s2 + ar.mulmod(h2, zp[16 + (k0 >> 4)]));
        {
            uint64_t y[16];
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) y[kk] = balanced_bytes<D>(v[kk]);
            pack_planes<D, 16>(y, pk);
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            if (i >= nd) break;
            int8_t* o = a.Bdig + (((uint64_t)l * D + i) * (FK / 32) + kc) * 2 * Ppad * 32 + (uint64_t)blockIdx.x * 1024 +
                        lane * 16;
            const uint32_t* w = pk[i];
            *(v4i*)o = v4i{(int)(w[0] ^ 0x80808080u), (int)(w[1] ^ 0x80808080u), (int)(w[2] ^ 0x80808080u),
                           (int)(w[3] ^ 0x80808080u)};
        }
    }
    // halves of a panel -> lanes l, l ^ 1; quarters -> the four waves (LDS); a' -> lanes l, l ^ 2
    s0 += __shfl_xor(s0, 1);
    s1 += __shfl_xor(s1, 1);
    s2 += __shfl_xor(s2, 1);
    red[0][kq][lane] = s0;
    red[1][kq][lane] = s1;
    red[2][kq][lane] = s2;
    __syncthreads();
    if (kq != 0) return;   // wave 0 finishes (no barrier below)
    double e[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) e[t] = ar.reduce(red[t][0][lane] + red[t][1][lane] + red[t][2][lane] + red[t][3][lane]);
    double o[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) o[t] = __shfl_xor(e[t], 2);
    const double e1[3] = {ap ? o[0] : e[0], ap ? o[1] : e[1], ap ? o[2] : e[2]};   // a = 1
    const double e2[3] = {ap ? e[0] : o[0], ap ? e[1] : o[1], ap ? e[2] : o[2]};   // a = 2
    // fo[2 + 3 a' + t] = lam1[a'][t], fo[8 + 3 a' + t] = lam2[a'][t]
    const double h0 = ar.mulmod(e1[0], fo[2]) + ar.mulmod(e2[0], fo[5]);          // r2 = 0, t = 0
    const double h257 = ar.mulmod(e1[0], fo[8]) + ar.mulmod(e2[0], fo[11]);
    const double h512 = ar.mulmod(e1[1], fo[8]) + ar.mulmod(e2[1], fo[11]);       // r2 = 255, t = 0
    const double h513 = ar.mulmod(e1[2], fo[9]) + ar.mulmod(e2[2], fo[12]);       // r2 = 256, t = 1
    // packed Phi_771 rows (mfhe_ctx::d_wphi): byte r2 - 1 (r2 = 1..256; r2 = 0 at byte 256) holds phi_r2, phi_(r2-1),
    // phi_(r2+257), phi_(r2+256) as 2-bit fields (value + 1) at shifts 0, 2, 4, 6
    auto phi = [&](int byte, int sh) { return (double)((int)((a.phi[byte] >> sh) & 3) - 1); };
    const double c1 = ar.reduce(h513);
    const double c0 = ar.reduce(h512 - c1 * phi(254, 6));   // phi_511 = phi_(r2+256) at r2 = 255
    if (!live || hf) return;
    uint64_t* Cl = a.C + (uint64_t)l * a.cL + (uint64_t)(p >> a.log_n) * a.scY + (p & nmask);
    if (ap == 0) {
        Cl[0] = ar.canon(h0 - c0 * phi(256, 0));
        a.cc[((uint64_t)l * Ppad + p) * 2] = c0;
        a.cc[((uint64_t)l * Ppad + p) * 2 + 1] = c1;
    } else {
        Cl[257 * a.scM] = ar.canon(h257 - c0 * phi(256, 4) - c1 * phi(256, 6));
    }
}

// rows r2 = 0, 255, 256 of the factored inverse from the column sums E_a'[0], E_a'[255], E_a'[256] (a = 1: e1,
// a = 2: e2), as at the end of mfma_digitize_ifold_kernel: f_0 and f_257 into C, (c0, c1) into cc
template <class FO>
__device__ __forceinline__ void ifold_finish(const ModGemmArgs& a, const ArithF64& ar, FO fo, const double (&e1)[3],
                                             const double (&e2)[3], int l, uint32_t Ppad, uint32_t p) {
    const double h0 = ar.mulmod(e1[0], fo[2]) + ar.mulmod(e2[0], fo[5]);
    const double h257 = ar.mulmod(e1[0], fo[8]) + ar.mulmod(e2[0], fo[11]);
    const double h512 = ar.mulmod(e1[1], fo[8]) + ar.mulmod(e2[1], fo[11]);
    const double h513 = ar.mulmod(e1[2], fo[9]) + ar.mulmod(e2[2], fo[12]);
    auto phi = [&](int byte, int sh) { return (double)((int)((a.phi[byte] >> sh) & 3) - 1); };
    const double c1 = ar.reduce(h513);
    const double c0 = ar.reduce(h512 - c1 * phi(254, 6));
    const uint32_t nmask = (1u << a.log_n) - 1;
    uint64_t* Cl = a.C + (uint64_t)l * a.cL + (uint64_t)(p >> a.log_n) * a.scY + (p & nmask);
    Cl[0] = ar.canon(h0 - c0 * phi(256, 0));
    Cl[257 * a.scM] = ar.canon(h257 - c0 * phi(256, 4) - c1 * phi(256, 6));
    a.cc[((uint64_t)l * Ppad + p) * 2] = c0;
    a.cc[((uint64_t)l * Ppad + p) * 2 + 1] = c1;
}

// The same digitize with the decrypt fused in front of it (n = 64, he.hip mfhe_decrypt_and_decode): B is never
// written to HBM.  One workgroup owns limb l and row y: the 64 columns p = 64 y + x over all 512 k (= w), so the
// whole X row of every (w, l, y) -- what the ring product needs -- is inside the workgroup, and the column sums
// s0 / s1 / s2 stay in it.  Per 32-k panel kc (eight iterations):
//   ring: 64 rows w = a' 256 + 32 kc + (0..31) (a' = 0, 1), 16 lanes per row (ring_row.hpp), B = ct.b +
//         INTT(NTT(ct.a) s) mod q exactly as dec_ring_kernel, reduced as the digitize reduces it, into LDS [row][x];
//   digitize: wave c = 2 a' + hf takes the 16 k of (a', hf) at column x = lane, the four waves fill each column's
//         64-byte (a', hf) group of the kc plane: 4 KiB contiguous per plane and iteration.
// Reads: ct (16 B per element) + s (L2-resident); writes: the digit planes.  The B round trip of the unfused path
// (8 B written by dec_ring_kernel + 8 B read here per element) and one launch per component are gone.
template <int D>
__device__ __forceinline__ void ifold_dec_impl(const ModGemmArgs& a, uint32_t Ppad, const PlaneCounts& pc, const int l,
                                               const int L) {
    constexpr int LOGN = 6, N = 64, RS = N + 2;   // row stride 528 B: the ring's 16-B row writes spread over banks
    __shared__ __attribute__((aligned(16))) double bt[64 * RS];
#if MFHE_DEC_RING_C
    __shared__ double rscr[16 * 68];   // ring_mul_row64_lds transposes, one row per 16 lanes
#endif
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t y = blockIdx.x;
    typedef const __attribute__((address_space(4))) double* cdp_t;
    const cdp_t fo = (cdp_t)(a.ifold + (uint64_t)l * 16);
    LimbConst lc;
    lc.qf = fo[0];
    lc.qinv = fo[1];
    const ArithF64 ar(lc);
    const LimbConst rl = ((const LimbConst*)a.dlf)[l];
    const ArithF64 rar(rl);
    const double* izl = a.iz + (uint64_t)l * 48;
    const double x1 = ((cdp_t)izl)[0], x2 = ((cdp_t)izl)[1];
    const double* zp = izl + 16;
    const int nd = l < 64 ? pc.n[l] : D;
    // ring-stage lane: 4 coefficients 4 j .. 4 j + 3 of row 16 s + rs (s = 0..3)
    const int j = t & 15, rs = t >> 4;
#if MFHE_DEC_TW_LDS
    // the limb's X-NTT tables in LDS: read per butterfly inside the panel loop instead of held in ~40 VGPRs
    __shared__ double twl[2 * N];
    if (t < N) twl[t] = a.dtw[(uint64_t)l * N + t];
    else if (t < 2 * N) twl[t] = a.ditw[(uint64_t)l * N + t - N];
    __syncthreads();
    const double* tw = twl;
    const double* itw = twl + N;
#else
    const double* tw = a.dtw + (uint64_t)l * N;
    const double* itw = a.ditw + (uint64_t)l * N;
#endif
    const double ninv = a.dninv[l];
    // digitize-stage lane: column x = lane, (a', hf) = wave
    const int ap = wv >> 1, hf = wv & 1;
    const uint32_t p = y * N + lane;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    // all four substeps' loads are issued before the first ring product (measured: a one-substep-ahead rolling
    // prefetch needs 186 VGPRs, 2 workgroups per CU, or spills at 3: 2-5% slower, profiles/r04_dec_fused_ab.txt)
    const int kpg = FK / 32 / (int)gridDim.z, kc0 = blockIdx.z * kpg;   // this block's share of the panels
#pragma unroll 1
    for (int kc = kc0; kc < kc0 + kpg; ++kc) {
#pragma unroll
        for (int sb = 0; sb < 4; sb += MFHE_DEC_SUBS) {   // MFHE_DEC_SUBS substeps' loads in flight together
        uint64_t av[MFHE_DEC_SUBS][4], sk[MFHE_DEC_SUBS][4], bv[MFHE_DEC_SUBS][4];
#pragma unroll
        for (int si = 0; si < MFHE_DEC_SUBS; ++si) {
            const int st = sb + si;
            const int rr = st * 16 + rs;
            const uint64_t w = (uint64_t)(rr >> 5) * FK + kc * 32 + (rr & 31);
            const uint64_t wl = w * L + l, r0 = (wl * N + y) * N;
            ld4<MFHE_DEC_NT>(a.dct + a.dtotal + r0 + 4 * j, av[si]);
            ld4(a.dsk + wl * N + 4 * j, sk[si]);
            ld4<MFHE_DEC_NT>(a.dct + r0 + 4 * j, bv[si]);
        }
        // ring product per row (the shuffle ring_mul_row: ring_mul_row64_lds measured slower here, 198 vs 183 us)
#pragma unroll
        for (int si = 0; si < MFHE_DEC_SUBS; ++si) {
            const int st = sb + si;
            double x[4], sv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                x[e] = ArithF64::from_u64(av[si][e]);
                sv[e] = centred_f(sk[si][e], rl.qf);
            }
#if MFHE_DEC_RING_C
            // ring_mul_row64_lds from 32-byte layout-C loads (one extra transpose in); b in layout C too, so the
            // product comes back to C through the row scratch before the add
            ring_mul_row64_lds<true>(x, sv, j, rar, tw, itw, ninv, rscr + rs * 68);
            {
                double* scr = rscr + rs * 68;
#pragma unroll
                for (int e = 0; e < 4; ++e) scr[(j + 16 * e) + ((j + 16 * e) >> 4)] = x[e];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int e = 0; e < 4; ++e) x[e] = scr[(4 * j + e) + ((4 * j + e) >> 4)];
                asm volatile("" ::: "memory");
            }
#else
            ring_mul_row<LOGN>(x, sv, j, rar, tw, itw, ninv);
#endif
            double v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint64_t sum = bv[si][e] + rar.canon(x[e]);
                v[e] = ar.reduce(ArithF64::from_u64(sum >= rl.q ? sum - rl.q : sum));
            }
            double* row = bt + (st * 16 + rs) * RS + 4 * j;
            *(double2*)row = make_double2(v[0], v[1]);
            *(double2*)(row + 2) = make_double2(v[2], v[3]);
        }
        }
        __syncthreads();
        const int k0 = kc * 32 + hf * 16;
        double v[16];
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) v[kk] = bt[(wv * 16 + kk) * RS + lane];   // b = k0 + kk + 1 of a = a' + 1
        // as mfma_digitize_ifold_kernel: Horner chains for x1, x2 and the plain sum over this chunk
        double h1 = v[15], h2 = v[15], t0 = 0.0;
#pragma unroll
        for (int kk = 14; kk >= 0; --kk) {
            h1 = ar.mulmod(h1, x1) + v[kk];
            h2 = ar.mulmod(h2, x2) + v[kk];
        }
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) t0 += v[kk];
        s0 = ar.reduce(s0 + t0);
        s1 = ar.reduce(s1 + ar.mulmod(h1, zp[(k0 >> 4)]));
        s2 = ar.reduce(s2 + ar.mulmod(h2, zp[16 + (k0 >> 4)]));
        uint32_t pk[D][4];
        {
            uint64_t yb[16];
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) yb[kk] = balanced_bytes<D>(v[kk]);
            pack_planes<D, 16>(yb, pk);
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            if (i >= nd) break;
            int8_t* o = a.Bdig + (((uint64_t)l * D + i) * (FK / 32) + kc) * (uint64_t)Ppad * 64 + (uint64_t)p * 64 + wv * 16;
            const uint32_t* w = pk[i];
            *(v4i*)o = v4i{(int)(w[0] ^ 0x80808080u), (int)(w[1] ^ 0x80808080u), (int)(w[2] ^ 0x80808080u),
                           (int)(w[3] ^ 0x80808080u)};
        }
        __syncthreads();   // the next panel's ring stage rewrites bt
    }
    // column sums: (a', hf) are the four waves
    bt[(0 * 4 + wv) * 64 + lane] = s0;
    bt[(1 * 4 + wv) * 64 + lane] = s1;
    bt[(2 * 4 + wv) * 64 + lane] = s2;
    __syncthreads();
    if (gridDim.z > 1) {
        // a share of the panels: this block's sums per (column, a') to the partials, finished by dec_colsum_kernel
        if (wv >= 2) return;
        double* o = a.dpart + (((uint64_t)blockIdx.z * L + l) * Ppad + p) * 6 + wv * 3;
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
            o[tt] = ar.reduce(bt[(tt * 4 + 2 * wv) * 64 + lane] + bt[(tt * 4 + 2 * wv + 1) * 64 + lane]);
        return;
    }
    if (wv != 0) return;
    double e1[3], e2[3];   // a = 1 (a' = 0), a = 2 (a' = 1)
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
        e1[tt] = ar.reduce(bt[(tt * 4 + 0) * 64 + lane] + bt[(tt * 4 + 1) * 64 + lane]);
        e2[tt] = ar.reduce(bt[(tt * 4 + 2) * 64 + lane] + bt[(tt * 4 + 3) * 64 + lane]);
    }
    ifold_finish(a, ar, fo, e1, e2, l, Ppad, p);
}
template <int D>
__global__ __launch_bounds__(256, MFHE_DEC_WG_CU) void mfma_digitize_ifold_dec_kernel(ModGemmArgs a, uint32_t Ppad, PlaneCounts pc) {
    ifold_dec_impl<D>(a, Ppad, pc, (int)blockIdx.y, (int)gridDim.y);
}
// two components in one grid (he.hip decrypt_and_decode: re and im): blockIdx.y in [0, 2 L), the upper half is b
template <int D>
__global__ __launch_bounds__(256, MFHE_DEC_WG_CU) void mfma_digitize_ifold_dec_pair_kernel(ModGemmArgs a, ModGemmArgs b,
                                                                                         uint32_t Ppad, PlaneCounts pc) {
    const int L = (int)gridDim.y / 2, y = (int)blockIdx.y;
    const bool hi = y >= L;
    ifold_dec_impl<D>(hi ? b : a, Ppad, pc, hi ? y - L : y, L);
}

// the column sums of a split decrypt-fused digitize (gridDim.z = G shares of the panels): one thread per (column, limb)
__device__ __forceinline__ void dec_colsum_impl(const ModGemmArgs& a, uint32_t Ppad, int G, const int l, const int L) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= Ppad) return;
    typedef const __attribute__((address_space(4))) double* cdp_t;
    const cdp_t fo = (cdp_t)(a.ifold + (uint64_t)l * 16);
    LimbConst lc;
    lc.qf = fo[0];
    lc.qinv = fo[1];
    const ArithF64 ar(lc);
    double e[6] = {0, 0, 0, 0, 0, 0};
    for (int g = 0; g < G; ++g) {   // |partial| <= q / 2: 8 terms stay exact, so reduce after every 8
        const double* o = a.dpart + (((uint64_t)g * L + l) * Ppad + p) * 6;
#pragma unroll
        for (int t = 0; t < 6; ++t) e[t] += o[t];
        if ((g & 7) == 7)
#pragma unroll
            for (int t = 0; t < 6; ++t) e[t] = ar.reduce(e[t]);
    }
    double e1[3], e2[3];
#pragma unroll
    for (int tt = 0; tt < 3; ++tt) {
        e1[tt] = ar.reduce(e[tt]);
        e2[tt] = ar.reduce(e[3 + tt]);
    }
    ifold_finish(a, ar, fo, e1, e2, l, Ppad, p);
}
__global__ __launch_bounds__(256) void dec_colsum_kernel(ModGemmArgs a, uint32_t Ppad, int G) {
    dec_colsum_impl(a, Ppad, G, (int)blockIdx.y, (int)gridDim.y);
}
__global__ __launch_bounds__(256) void dec_colsum_pair_kernel(ModGemmArgs a, ModGemmArgs b, uint32_t Ppad, int G) {
    const int L = (int)gridDim.y / 2, y = (int)blockIdx.y;
    const bool hi = y >= L;
    dec_colsum_impl(hi ? b : a, Ppad, G, hi ? y - L : y, L);
}


// C = sum_s acc_s * 256^s mod q for the 32 x 32 wave tile at (m0, p0) of limb l (lane = (r, h)).
// MODE 1 (factored forward): column p0 + r is (a', p) = divmod(., Ppad), output row a' * 256 + row, plus d0.
// MODE 2 (factored inverse): column p0 + r is 2 p + a', row r2 - 1; lanes r, r ^ 1 hold a' = 0, 1 of one column
// and trade their lam products, then write f_r2 (a' = 0) and f_(r2+257) (a' = 1, r2 <= 254).
// lanes l <-> l ^ 1 (DPP quad_perm [1, 0, 3, 2]: a VALU move, no LDS crossbar)
__device__ __forceinline__ double swap_pair(double x) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, true),
                            __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, true));
}

// MODE 2: this lane's column's (c0, c1), loaded before the K loop so the epilogue does not wait for them
struct InvCC {
    double c0 = 0.0, c1 = 0.0;
};
template <int MODE>
__device__ __forceinline__ InvCC inv_cc(const ModGemmArgs& a, int l, uint32_t p0, int r, uint32_t Ppad) {
    InvCC c;
    if constexpr (MODE == 2) {
        const uint32_t p = (p0 + r) >> 1;
        const double* src = a.cc + ((uint64_t)l * Ppad + (p < a.P ? p : 0)) * 2;
        c.c0 = src[0];
        c.c1 = src[1];
    }
    return c;
}

template <int D, int MODE = 0>
__device__ __forceinline__ void mfma_epilogue(const ModGemmArgs& a, const v16i (&acc)[2 * D - 1], int l, int m0,
                                              uint32_t p0, int r, int h, uint32_t Ppad = 0, InvCC cc = InvCC{}) {
    constexpr int NS = 2 * D - 1;
    constexpr bool FAC = MODE != 0;
    uint64_t* Cl = a.C + (uint64_t)l * a.cL;
    if constexpr (MODE == 2) {
        typedef const __attribute__((address_space(4))) double* cdp_t;
        const cdp_t ep = (cdp_t)(a.epi + (uint64_t)l * 8);
        const cdp_t fo = (cdp_t)(a.ifold + (uint64_t)l * 16);
        LimbConst lc;
        lc.qf = ep[0];
        lc.qinv = ep[1];
        const ArithF64 ar(lc);
        const double c32[3] = {ep[2], ep[3], ep[4]};
        const uint32_t colf = p0 + r;
        const int ap = colf & 1;
        const uint32_t p = colf >> 1;
        const bool live = p < a.P;   // the same for both lanes of a pair
        // this lane's output takes lam_own (lam1 for a' = 0, lam2 for a' = 1) of its own E and the partner's share
        // lam_oth; both rotated once by r2 mod 3 of the lane's first row, so row reg uses index (reg's offset) mod 3
        const int r2b = m0 + 4 * h + 1;   // r2 of reg 0; reg adds (reg & 3) + 8 (reg >> 2)
        const int tb = r2b % 3;
        double own[3], oth[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int t = tb + k >= 3 ? tb + k - 3 : tb + k;
            const double l1 = t == 0 ? (ap ? fo[5] : fo[2]) : (t == 1 ? (ap ? fo[6] : fo[3]) : (ap ? fo[7] : fo[4]));
            const double l2 = t == 0 ? (ap ? fo[11] : fo[8]) : (t == 1 ? (ap ? fo[12] : fo[9]) : (ap ? fo[13] : fo[10]));
            own[k] = ap ? l2 : l1;
            oth[k] = ap ? l1 : l2;
        }
        const double c0 = cc.c0, c1 = cc.c1;
        uint64_t* Cp = Cl + (uint64_t)(p >> a.log_n) * a.scY + (p & ((1u << a.log_n) - 1));
        // the packed Phi rows of this wave tile's 32 rows r2 = m0 + 1 .. m0 + 32 (bytes m0 .. m0 + 31) by scalar loads
        typedef const __attribute__((address_space(4))) uint32_t* cu32_t;
        const cu32_t pw = (cu32_t)(a.phi + m0);
        uint32_t win[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) win[i] = pw[i];
        const int sh = ap ? 4 : 0;   // fields (phi_j, phi_(j-1)) of this lane's output row j
        constexpr int NZ = (NS + 1) / 2, NY = (NZ + 1) / 2;
        // every row computed first, the guarded stores after: a store under a branch inside the row loop splits it
        // into 16 serial blocks, each paying the full FP64 latency chain
        uint64_t outw[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int k = ((reg & 3) + 8 * (reg >> 2)) % 3;
            const uint32_t pb = ((h ? win[2 * (reg >> 2) + 1] : win[2 * (reg >> 2)]) >> (8 * (reg & 3) + sh)) & 15u;
            double zz[NZ];
#pragma unroll
            for (int t = 0; t < NZ; ++t)
                zz[t] = 2 * t + 1 < NS ? __fma_rn(256.0, (double)acc[2 * t + 1][reg], (double)acc[2 * t][reg])
                                       : (double)acc[2 * t][reg];
            double v = 0.0;
#pragma unroll
            for (int u = 0; u < NY; ++u) {
                const double y = 2 * u + 1 < NZ ? __fma_rn(65536.0, zz[2 * u + 1], zz[2 * u]) : zz[2 * u];
                v += u == 0 ? y : ar.mulmod(y, c32[u - 1]);
            }
            // |v| < 2^51 + 2 q, so v * lam / q < 2^51 with |lam| <= q / 2: mulmod needs no reduction of v first
            const double hv = ar.mulmod(v, own[k]) + swap_pair(ar.mulmod(v, oth[k]));
            // phi in {-1, 0, 1}: exact products, so one fma each
            const double fj = __fma_rn(-c0, (double)((int)(pb & 3u) - 1), __fma_rn(-c1, (double)((int)(pb >> 2) - 1), hv));
            outw[reg] = ar.canon(fj);
        }
        if (live) {
            const uint64_t jb = (uint64_t)(ap ? r2b + 257 : r2b);
            if (m0 + 32 <= 254) {   // wave-uniform: every row of this tile has an output in both halves
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) Cp[(jb + (reg & 3) + 8 * (reg >> 2)) * a.scM] = outw[reg];
            } else {
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int r2 = r2b + (reg & 3) + 8 * (reg >> 2);
                    if (ap == 0 || r2 <= 254) Cp[(jb + (reg & 3) + 8 * (reg >> 2)) * a.scM] = outw[reg];
                }
            }
        }
        return;
    }
    if (FAC || a.epi) {
        // FP64 (every q < 2^50): |acc_s| < 2^26, so z_t = acc_2t + 256 acc_2t+1 (< 2^35) and
        // y_u = z_2u + 2^16 z_2u+1 (< 2^51) are exact doubles; C = y_0 + sum_u y_u (2^32u mod q), each
        // product an exact FP64 modmul with a centred constant (|y c / q| < 2^50), then one canonical
        // reduction -- about 25 FP64 ops per output instead of 2D-1 64-bit Shoup products.
        // per-limb constants by scalar loads (constant address space): no vmcnt wait, so the persistent ring's
        // DMAs in flight are not waited for here
        typedef const __attribute__((address_space(4))) double* cdp_t;
        const cdp_t ep = (cdp_t)(a.epi + (uint64_t)l * 8);
        LimbConst lc;
        lc.qf = ep[0];
        lc.qinv = ep[1];
        const ArithF64 ar(lc);
        const double c32[3] = {ep[2], ep[3], ep[4]};
        uint32_t colf = p0 + r;
        int rbase = 0;
        double add = 0.0;
        if (FAC) {
            const int ap = colf >= Ppad;
            colf -= ap * Ppad;
            if (colf >= a.P) return;
            rbase = ap * FK;
            add = ArithF64::from_u64(a.d0[((uint64_t)l * 2 + ap) * Ppad + colf]);
        }
        if (colf >= a.P) return;
        constexpr int NZ = (NS + 1) / 2, NY = (NZ + 1) / 2;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = rbase + m0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
            double z[NZ];
#pragma unroll
            for (int t = 0; t < NZ; ++t)
                z[t] = 2 * t + 1 < NS ? __fma_rn(256.0, (double)acc[2 * t + 1][reg], (double)acc[2 * t][reg])
                                      : (double)acc[2 * t][reg];
            double v = add;
#pragma unroll
            for (int u = 0; u < NY; ++u) {
                const double y = 2 * u + 1 < NZ ? __fma_rn(65536.0, z[2 * u + 1], z[2 * u]) : z[2 * u];
                v += u == 0 ? y : ar.mulmod(y, c32[u - 1]);
            }
            const uint64_t o = (uint64_t)row * a.scM + (uint64_t)(colf >> a.log_n) * a.scY + (colf & ((1u << a.log_n) - 1));
            const uint64_t cv = ar.canon(v);
            Cl[o] = cv;
            if (a.C2) a.C2[(uint64_t)l * a.cL + o] = cv;
        }
        return;
    }
    if constexpr (FAC) return;   // factored mode always has the FP64 epilogue (launch_mod_gemm checks)
    typedef const __attribute__((address_space(4))) uint64_t* cup_t;
    const uint64_t q = ((cup_t)a.qmu)[2 * l], mu = ((cup_t)a.qmu)[2 * l + 1];
    // rtab rows are [L][2 a.D - 1][2] for the context's plane stride a.D: a limb run with fewer digits (NS < 2 a.D - 1)
    // must still step by the table's row length (r06: stepping by NS gave limbs >= 1 of a D = 7 run in a D = 8 context
    // another limb's constants, tests/test_wcrt_sizes_gpu.py at 55 bits)
    const cup_t rt = (cup_t)(a.rtab + (uint64_t)l * (2 * a.D - 1) * 2);
    uint64_t* C = Cl;
    const uint32_t col = p0 + r;
    if (col >= a.P) return;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = m0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        uint64_t sum = 0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int64_t v = acc[s][reg];
            const uint64_t x = v < 0 ? (uint64_t)(v + (int64_t)q) : (uint64_t)v;   // |v| < 2^26 < q
            uint64_t t = x * rt[2 * s] - __umul64hi(x, rt[2 * s + 1]) * q;        // Shoup: [0, 2q)
            sum += t;                                                              // < 2 NS q < 2^64
        }
        uint64_t red = sum - __umul64hi(sum, mu) * q;   // Barrett: [0, 2q)
        red = red >= q ? red - q : red;
        C[(uint64_t)row * a.scM + (uint64_t)(col >> a.log_n) * a.scY + (col & ((1u << a.log_n) - 1))] = red;
    }
}

template <int D>
__global__ __launch_bounds__(256, D <= 5 ? 2 : 1) void mod_gemm_mfma_kernel(ModGemmArgs a, uint32_t Ppad, int limb0) {
    constexpr int NS = 2 * D - 1;
    const int l = limb0 + blockIdx.z;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int m0 = blockIdx.y * 64 + (w & 1) * 32;
    const uint32_t p0 = blockIdx.x * 64 + (w >> 1) * 32;
    const int8_t* Al = a.Adig + (uint64_t)l * a.adL;
    const int8_t* Bl = a.Bdig + (uint64_t)l * a.D * Ppad * MK;   // planes beyond this limb's D are zero
    v16i acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = v16i{0};
    for (int kc = 0; kc < MK / 32; ++kc) {
        v4i av[D], bv[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            av[i] = *(const v4i*)(Al + (uint64_t)i * 512 * MK + ((uint64_t)kc * 512 + m0 + r) * 32 + 16 * h);
            bv[i] = *(const v4i*)(Bl + (uint64_t)i * Ppad * MK + ((uint64_t)kc * Ppad + p0 + r) * 32 + 16 * h);
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int j = 0; j < D; ++j) acc[i + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av[i], bv[j], acc[i + j], 0, 0, 0);
    }
    mfma_epilogue<D>(a, acc, l, m0, p0, r, h);
}

// LDS-staged variant (default).  Same digit planes, tile (64 x 64 outputs, four 32 x 32 wave tiles) and
// exact accumulation as mod_gemm_mfma_kernel, but each 64-deep K stage (two 32-k panels) of both operands
// goes global -> LDS once per workgroup by LDS-DMA (global_load_lds_dwordx4: no VGPR staging; the
// k-panel-major planes make each wave's 1 KiB destination lane-linear, as the DMA requires), double-
// buffered one stage ahead of the MFMAs that read it.  Waves 0-1 move A's planes, waves 2-3 B's.
// RAW order for the DMA'd bytes: issuing waves' s_waitcnt vmcnt(0), then the barrier, then the reads.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int D, int MODE>
__global__ __launch_bounds__(256, D <= 5 ? 2 : 1) void mod_gemm_mfma_lds_kernel(ModGemmArgs a, uint32_t Ppad, int limb0) {
    // MODE 1 / 2 (factored forward / inverse): M = K = 256 and 2 Ppad B columns; 0: M = K = 512 and Ppad columns
    constexpr bool FAC = MODE != 0;
    constexpr int KK = FAC ? FK : MK, AM = FAC ? FK : 512;
    const uint32_t Pcols = FAC ? 2 * Ppad : Ppad;
    constexpr int NS = 2 * D - 1;
    constexpr int KS = 64;                       // K per stage: two 32-k panels
    constexpr int PANEL = 64 * 32;               // 64 rows x 32 k of one digit plane (bytes)
    constexpr int PLANE = 2 * PANEL;             // one digit plane of one operand per stage
    constexpr int STAGE = 2 * D * PLANE;         // A planes then B planes
    __shared__ __attribute__((aligned(16))) int8_t lds[2 * STAGE];
    const int l = limb0 + blockIdx.z;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int mb = blockIdx.y * 64, pb = blockIdx.x * 64;
    const int wm = (w & 1) * 32, wp = (w >> 1) * 32;
    // DMA slot li: bytes [16 li, 16 li + 16) of a 2 KiB panel image (row li / 2, k half li & 1)
    const bool ldA = t < 128;
    const int li = t & 127;
    const uint64_t rows = ldA ? AM : Pcols;                        // rows of the operand's planes
    const int8_t* src = (ldA ? a.Adig + (uint64_t)l * a.adL : a.Bdig + (uint64_t)l * a.D * Pcols * KK) +
                        (uint64_t)(ldA ? mb : pb) * 32 + li * 16;
    const uint64_t pstride = rows * KK, kstride = rows * 32;      // digit-plane / k-panel strides
    const int wbase = (ldA ? 0 : D * PLANE) + (li & ~63) * 16;     // this wave's LDS destination base
    auto issue = [&](int s, int buf) {
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int pp = 0; pp < 2; ++pp)
                __builtin_amdgcn_global_load_lds((const void*)(src + i * pstride + (uint64_t)(2 * s + pp) * kstride),
                                                 (lds_ptr_t)(lds + buf * STAGE + wbase + i * PLANE + pp * PANEL), 16,
                                                 0, 0);
    };
    const InvCC icc = inv_cc<MODE>(a, l, (uint32_t)(pb + wp), r, Ppad);
    v16i acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = v16i{0};
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int s = 0; s < KK / KS; ++s) {
        const int buf = s & 1;
        if (s + 1 < KK / KS) issue(s + 1, buf ^ 1);   // buf ^ 1's last readers all passed the previous barrier
        const int8_t* st = lds + buf * STAGE;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
            v4i bv[D];
#pragma unroll
            for (int j = 0; j < D; ++j)
                bv[j] = *(const v4i*)(st + (D + j) * PLANE + pp * PANEL + (wp + r) * 32 + 16 * h);
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const v4i av = *(const v4i*)(st + i * PLANE + pp * PANEL + (wm + r) * 32 + 16 * h);
#pragma unroll
                for (int j = 0; j < D; ++j)
                    acc[i + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv[j], acc[i + j], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA into buf ^ 1 has landed
        __syncthreads();
    }
    mfma_epilogue<D, MODE>(a, acc, l, mb + wm, (uint32_t)(pb + wp), r, h, Ppad, icc);
}

// Ring variant (MFHE_OPT_WCRT_PIPE 2 / 3, and 0 = auto on the factored launch): the same tile, digit planes and
// epilogue, but the K loop runs over 32-k stages (one panel per digit plane per operand, 4 D KiB) held in an
// NSLOT-slot LDS ring: stage s + NSLOT - 1 is DMA'd while stage s is multiplied, so a stage's bytes have NSLOT - 1
// stage times to land instead of one, and the wait at the end of stage s is a counted vmcnt that leaves the later
// stages in flight (D DMA instructions per thread per stage; nothing else in the loop touches vector memory).  The
// barrier after it is a raw s_barrier (__syncthreads' fence would wait for the DMAs in flight).  Slot
// (s + NSLOT - 1) % NSLOT = (s - 1) % NSLOT was last read in stage s - 1, which every wave has left at that barrier.
// NSLOT = 4 at D = 5 (80 KiB, 2 workgroups per CU); 3 at D = 6 (72 KiB): with its registers held to 256 (launch
// bounds) the D = 6 limb (the reference's 44-bit q0) also runs 2 workgroups per CU -- r03 ran it at 96 KiB and 384
// VGPRs, one workgroup per CU and 0.22 MFMA busy (profiles/r03_gemm_sq_pmc.txt).
// AHEAD: the next A fragment's LDS read is issued before the current fragment's D MFMAs (sched_barrier-pinned),
// so its latency hides behind them instead of being waited for in front of them (D <= 5 only: at D >= 6 the
// extra fragment spills).
template <int D>
constexpr int ring_slots() { return D <= 5 ? 4 : 3; }
template <int D, int MODE>
constexpr int ring_lds_bytes() { return ring_slots<D>() * 2 * D * 64 * 32; }
template <int D, int MODE, bool AHEAD>
__device__ __forceinline__ void ring_tile(const ModGemmArgs& a, uint32_t Ppad, int l, int8_t* lds) {
    constexpr bool FAC = MODE != 0;
    constexpr int KK = FAC ? FK : MK, AM = FAC ? FK : 512;
    const uint32_t Pcols = FAC ? 2 * Ppad : Ppad;
    constexpr int NS = 2 * D - 1;
    constexpr int NST = KK / 32;                 // 32-k stages
    constexpr int PANEL = 64 * 32;               // 64 rows x 32 k of one digit plane (bytes)
    constexpr int STAGE = 2 * D * PANEL;         // A planes then B planes
    constexpr int NSLOT = ring_slots<D>(), LEAD = NSLOT - 1;
    static_assert(NST >= NSLOT, "ring prologue assumes at least NSLOT stages");
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int mb = blockIdx.y * 64, pb = blockIdx.x * 64;
    const int wm = (w & 1) * 32, wp = (w >> 1) * 32;
    const bool ldA = t < 128;
    const int li = t & 127;
    const uint64_t rows = ldA ? AM : Pcols;
    const int8_t* src = (ldA ? a.Adig + (uint64_t)l * a.adL : a.Bdig + (uint64_t)l * a.D * Pcols * KK) +
                        (uint64_t)(ldA ? mb : pb) * 32 + li * 16;
    const uint64_t pstride = rows * KK, kstride = rows * 32;
    const int wbase = (ldA ? 0 : D * PANEL) + (li & ~63) * 16;
    auto issue = [&](int s) {
        int8_t* dst = lds + (s % NSLOT) * STAGE + wbase;
#pragma unroll
        for (int i = 0; i < D; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src + i * pstride + (uint64_t)s * kstride),
                                             (lds_ptr_t)(dst + i * PANEL), 16, 0, 0);
    };
    auto barrier = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    const InvCC icc = inv_cc<MODE>(a, l, (uint32_t)(pb + wp), r, Ppad);   // older than every DMA: the counted waits cover it
    v16i acc[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] = v16i{0};
#pragma unroll
    for (int s = 0; s < LEAD; ++s) issue(s);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((LEAD - 1) * D) : "memory");   // stage 0 landed (1 .. LEAD - 1 in flight)
    barrier();
#pragma unroll
    for (int s = 0; s < NST; ++s) {
        if (s + LEAD < NST) issue(s + LEAD);
        const int8_t* st = lds + (s % NSLOT) * STAGE;
        v4i bv[D];
#pragma unroll
        for (int j = 0; j < D; ++j) bv[j] = *(const v4i*)(st + (D + j) * PANEL + (wp + r) * 32 + 16 * h);
        if constexpr (AHEAD) {
            v4i an = *(const v4i*)(st + (wm + r) * 32 + 16 * h);
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const v4i av = an;
                if (i + 1 < D) an = *(const v4i*)(st + (i + 1) * PANEL + (wm + r) * 32 + 16 * h);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < D; ++j)
                    acc[i + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv[j], acc[i + j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < D; ++i) {
                const v4i av = *(const v4i*)(st + i * PANEL + (wm + r) * 32 + 16 * h);
#pragma unroll
                for (int j = 0; j < D; ++j)
                    acc[i + j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv[j], acc[i + j], 0, 0, 0);
            }
        }
        // stage s + 1 landed for this wave: newer are the DMAs of the stages after it that were issued
        if (s + 1 < NST) {
            const int newer = (s + LEAD < NST ? s + LEAD : NST - 1) - (s + 1);
            if (newer == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D) : "memory");
            else if (newer == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            barrier();
        }
    }
    mfma_epilogue<D, MODE>(a, acc, l, mb + wm, (uint32_t)(pb + wp), r, h, Ppad, icc);
}

template <int D, int MODE, bool AHEAD>
__global__ __launch_bounds__(256, D <= 5 || (D == 6 && MODE != 0) ? 2 : 1)   // dense D = 6 spills at 256 VGPRs
void mod_gemm_mfma_ring_kernel(ModGemmArgs a, uint32_t Ppad, int limb0) {
    __shared__ __attribute__((aligned(16))) int8_t lds[ring_lds_bytes<D, MODE>()];
    ring_tile<D, MODE, AHEAD>(a, Ppad, limb0 + (int)blockIdx.z, lds);
}

// r04: the factored launches' limbs at D = 5 and D = 6 in one grid (the reference's 44-bit q0 needs six
// digits and ran as its own one-limb launch at 0.22 MFMA busy).  The digit count is per limb (bit l of d6, workgroup-
// uniform: blockIdx.z), the two bodies share one LDS ring (max of 80 KiB at D = 5 and 72 KiB at D = 6) and one
// register budget (<= 256: 2 workgroups per CU for both); limb 0's tiles dispatch first (z slowest), so the heavier
// tiles do not form the tail.
template <int MODE>
__global__ __launch_bounds__(256, 2) void mod_gemm_mfma_ring56_kernel(ModGemmArgs a, uint32_t Ppad, int limb0, uint64_t d6) {
    constexpr int B5 = ring_lds_bytes<5, MODE>(), B6 = ring_lds_bytes<6, MODE>();
    __shared__ __attribute__((aligned(16))) int8_t lds[B5 > B6 ? B5 : B6];
    const int l = limb0 + (int)blockIdx.z;
    if ((d6 >> blockIdx.z) & 1) ring_tile<6, MODE, false>(a, Ppad, l, lds);
    else ring_tile<5, MODE, false>(a, Ppad, l, lds);
}
// two components in one grid (blockIdx.z in [0, 2 L), the upper half is b): encode's / decode's re and im, whose
// tiles then share the GPU without a stream fork (he.hip MFHE_OPT_HE_STREAMS 2)
template <int MODE>
__global__ __launch_bounds__(256, 2) void mod_gemm_mfma_ring56_pair_kernel(ModGemmArgs a, ModGemmArgs b, uint32_t Ppad,
                                                                           uint64_t d6) {
    constexpr int B5 = ring_lds_bytes<5, MODE>(), B6 = ring_lds_bytes<6, MODE>();
    __shared__ __attribute__((aligned(16))) int8_t lds[B5 > B6 ? B5 : B6];
    const int L = (int)gridDim.z / 2, z = (int)blockIdx.z;
    const bool hi = z >= L;
    const int l = hi ? z - L : z;
    const ModGemmArgs& x = hi ? b : a;
    if ((d6 >> l) & 1) ring_tile<6, MODE, false>(x, Ppad, l, lds);
    else ring_tile<5, MODE, false>(x, Ppad, l, lds);
}

// The ring kernel's waits are counted (vmcnt(D) / vmcnt(2D): the DMAs of the stages still in flight).  A build in
// which it spills would add scratch traffic to the counted ops; checked once per instantiation from the code
// object's metadata, and such a build runs the two-stage LDS kernel (vmcnt(0) waits) instead.  AHEAD is D <= 5
// only: at D = 6 its extra A fragment spills (tests/test_isa.py pins the shipped instantiations' instruction mix).
template <int D, int MODE, bool AHEAD>
static bool ring_usable() {
    static int ok = -1;
    if (ok < 0) {
        hipFuncAttributes fa{};
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(mod_gemm_mfma_ring_kernel<D, MODE, AHEAD>)) ==
                     hipSuccess &&
             fa.localSizeBytes == 0;
    }
    return ok == 1;
}

template <int MODE>
static bool ring56_usable() {
    static int ok = -1;
    if (ok < 0) {
        hipFuncAttributes fa{};
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(mod_gemm_mfma_ring56_kernel<MODE>)) == hipSuccess &&
             fa.localSizeBytes == 0;
    }
    return ok == 1;
}

// factored launches, pipe 0 (auto): every limb at D = 5 or 6 in one ring56 grid.  Returns false (nothing launched)
// when that does not apply: another pipe, a digit count outside {5, 6}, more than 64 limbs, or a spilling build.
template <int MODE>
static bool launch_ring56(const ModGemmArgs& f, int L, uint32_t Ppad, hipStream_t s) {
    if (f.pipe != 0 || L > 64 || !ring56_usable<MODE>()) return false;
    uint64_t d6 = 0;
    for (int l = 0; l < L; ++l) {
        const int d = f.limbD ? std::max(f.limbD[l], 5) : f.D;
        if (d != 5 && d != 6) return false;
        if (d == 6) d6 |= 1ull << l;
    }
    const dim3 grid(2 * Ppad / 64, FK / 64, L);
    hipLaunchKernelGGL((mod_gemm_mfma_ring56_kernel<MODE>), grid, dim3(256), 0, s, f, Ppad, 0, d6);
    return true;
}

// pipe: 1 = two-stage LDS kernel; 3 = ring + one-ahead A read (D <= 5); anything else = ring
template <int D, int MODE>
static void launch_staged(int pipe, dim3 grid, hipStream_t s, const ModGemmArgs& f, uint32_t Ppad, int l0) {
    if constexpr (D <= 5) {
        if (pipe == 3 && ring_usable<D, MODE, true>()) {
            hipLaunchKernelGGL((mod_gemm_mfma_ring_kernel<D, MODE, true>), grid, dim3(256), 0, s, f, Ppad, l0);
            return;
        }
    }
    if (pipe != 1 && ring_usable<D, MODE, false>()) {
        hipLaunchKernelGGL((mod_gemm_mfma_ring_kernel<D, MODE, false>), grid, dim3(256), 0, s, f, Ppad, l0);
        return;
    }
    hipLaunchKernelGGL((mod_gemm_mfma_lds_kernel<D, MODE>), grid, dim3(256), 0, s, f, Ppad, l0);
}

// ---- the W-CRT forward of a small signed operand (r06): the encrypt's Gaussian noise ----
// The noise e is one small integer per (w, pos), the same in every limb: the reference's Box-Muller draw
// (HE.cu:581-627) is 3.2 sqrt(-2 ln u1) cos(2 pi u2) with u1 >= 2^-53, so |e| <= 3.2 sqrt(106 ln 2) < 27.5 and e is its
// own balanced base-256 digit.  The dense product V_l e then needs D_l x 1 digit pairs per MAC (acc_i = sum_k v_i e,
// shift i only) against the factored forward's D_l x D_l at half the MACs: 2 D_l / D_l^2 = 0.4 of its MFMAs at
// D_l = 5, with no digitize kernel (gaussian_i8_kernel writes the one plane, shared by every limb, in the GEMM's
// k-panel-major layout) and no per-limb residue array.
// Tile 64 rows x 64 NC columns, four waves as 2 x 2 (each 32 rows x 32 NC columns, NC accumulator sets per digit);
// 64-k LDS-DMA stages, double-buffered, per stage every thread issues DA + NC DMAs (A's DA planes, then B's NC).
// A's DA planes are the bulk of a stage, so NC = 2 halves the A bytes per MAC (r06 counters at NC = 1: MFMA busy
// 0.21, waits 0.54 of wave cycles; a third stage buffer was slower).  FP64 epilogue (every q < 2^50):
// |acc_i| <= 512 * 128 * 28 < 2^21, z / y as in mfma_epilogue.
template <int DA, int NC>
__device__ __forceinline__ void smallb_mma(const ModGemmArgs& a, const int8_t* __restrict__ b8, uint32_t Ppad, int l,
                                           int mb, int pb, int8_t* lds, v16i (&acc)[NC][DA]) {
    constexpr int KS = 64, PANEL = 64 * 32, PLANE = 2 * PANEL;   // one stage: two 32-k panels per 64-row plane
    constexpr int STAGE = (DA + NC) * PLANE;                        // A's DA planes, then B's NC (64 columns each)
    constexpr int NS = MK / KS;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wm = (w & 1) * 32, wp = (w >> 1) * 32 * NC;          // this wave's rows / first column in the tile
    const int pp = t >> 7, li = t & 127;                            // this thread's k-panel of a stage and 16-B chunk
    const int8_t* srcA = a.Adig + (uint64_t)l * a.adL + (uint64_t)mb * 32 + li * 16;
    const int8_t* srcB = b8 + (uint64_t)pb * 32 + li * 16;
    constexpr uint64_t kstrA = 512ull * 32, plA = 512ull * MK;      // A: k-panel / digit-plane strides
    const uint64_t kstrB = (uint64_t)Ppad * 32;
    const int wdst = pp * PANEL + ((li & ~63) * 16);                // this wave's LDS destination inside a plane
    auto issue = [&](int s, int buf) {
        int8_t* st = lds + buf * STAGE + wdst;
        const uint64_t kp = (uint64_t)(2 * s + pp);
#pragma unroll
        for (int i = 0; i < DA; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(srcA + i * plA + kp * kstrA), (lds_ptr_t)(st + i * PLANE), 16,
                                             0, 0);
#pragma unroll
        for (int c = 0; c < NC; ++c)
            __builtin_amdgcn_global_load_lds((const void*)(srcB + c * 64 * 32 + kp * kstrB),
                                             (lds_ptr_t)(st + (DA + c) * PLANE), 16, 0, 0);
    };
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int i = 0; i < DA; ++i) acc[c][i] = v16i{0};
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 1
    for (int s = 0; s < NS; ++s) {
        const int buf = s & 1;
        if (s + 1 < NS) issue(s + 1, buf ^ 1);   // buf ^ 1's last readers all passed the previous barrier
        const int8_t* st = lds + buf * STAGE;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            v4i bv[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int tc = wp + 32 * c;   // tile column of this 32-column block: 64-column plane tc / 64
                bv[c] = *(const v4i*)(st + (DA + tc / 64) * PLANE + q * PANEL + (tc % 64 + r) * 32 + 16 * h);
            }
#pragma unroll
            for (int i = 0; i < DA; ++i) {
                const v4i av = *(const v4i*)(st + i * PLANE + q * PANEL + (wm + r) * 32 + 16 * h);
#pragma unroll
                for (int c = 0; c < NC; ++c) acc[c][i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv[c], acc[c][i], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs into buf ^ 1 have landed
        __syncthreads();
    }
}

// C = sum_i acc_i 256^i mod q, canonical, for accumulator register `reg` (FP64: z / y as in mfma_epilogue)
template <int DA>
__device__ __forceinline__ uint64_t smallb_value(const ArithF64& ar, const double (&c32)[3], const v16i (&acc)[DA],
                                                 int reg) {
    constexpr int NZ = (DA + 1) / 2, NY = (NZ + 1) / 2;
    double z[NZ];
#pragma unroll
    for (int u = 0; u < NZ; ++u)
        z[u] = 2 * u + 1 < DA ? __fma_rn(256.0, (double)acc[2 * u + 1][reg], (double)acc[2 * u][reg])
                              : (double)acc[2 * u][reg];
    double v = 0.0;
#pragma unroll
    for (int u = 0; u < NY; ++u) {
        const double y = 2 * u + 1 < NZ ? __fma_rn(65536.0, z[2 * u + 1], z[2 * u]) : z[2 * u];
        v += u == 0 ? y : ar.mulmod(y, c32[u - 1]);
    }
    return ar.canon(v);
}

template <int DA, int NC>
__global__ __launch_bounds__(256, 2) void mod_gemm_mfma_smallb_kernel(ModGemmArgs a, const int8_t* __restrict__ b8,
                                                                      uint32_t Ppad, int limb0) {
    __shared__ __attribute__((aligned(16))) int8_t lds[2 * (DA + NC) * 64 * 64];
    const int l = limb0 + blockIdx.z;
    const int mb = blockIdx.y * 64, pb = blockIdx.x * 64 * NC;
    v16i acc[NC][DA];
    smallb_mma<DA, NC>(a, b8, Ppad, l, mb, pb, lds, acc);
    typedef const __attribute__((address_space(4))) double* cdp_t;
    const cdp_t ep = (cdp_t)(a.epi + (uint64_t)l * 8);
    LimbConst lc;
    lc.qf = ep[0];
    lc.qinv = ep[1];
    const ArithF64 ar(lc);
    const double c32[3] = {ep[2], ep[3], ep[4]};
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
    const int wm = (w & 1) * 32, wp = (w >> 1) * 32 * NC;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t col = pb + wp + 32 * c + r;
        if (col >= a.P) continue;
        uint64_t* Cl = a.C + (uint64_t)l * a.cL + (uint64_t)(col >> a.log_n) * a.scY + (col & ((1u << a.log_n) - 1));
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
            Cl[(uint64_t)(mb + wm + (reg & 3) + 8 * (reg >> 2) + 4 * h) * a.scM] = smallb_value<DA>(ar, c32, acc[c], reg);
    }
}

// b8: [512 / 32][Ppad][32] with Ppad = P rounded up to 64; the two-block tile (NC = 2) needs Ppad % 128 == 0 so that
// no stage reads past the plane
int launch_mod_gemm_smallb(const ModGemmArgs& a, const int8_t* b8, int L, hipStream_t s) {
    if (!a.Adig || !a.epi || a.M != 512 || a.K != MK || a.fold || a.ifold || a.D < 5 || a.D > 6 || a.adL == 0)
        return set_error(MFHE_EINVAL, "mod_gemm_smallb: needs the dense per-limb V planes (5 or 6 digits) and the FP64 epilogue");
    const uint32_t Ppad = (a.P + 63) / 64 * 64;
    const int nc = Ppad % 128 == 0 ? 2 : 1;
    for (int l0 = 0; l0 < L;) {
        const int d = a.limbD ? std::max(a.limbD[l0], 5) : a.D;
        int l1 = l0 + 1;
        while (l1 < L && (a.limbD ? std::max(a.limbD[l1], 5) : a.D) == d) ++l1;
        const dim3 grid(Ppad / (64 * nc), 512 / 64, l1 - l0);
        if (d == 5 && nc == 2) hipLaunchKernelGGL((mod_gemm_mfma_smallb_kernel<5, 2>), grid, dim3(256), 0, s, a, b8, Ppad, l0);
        else if (d == 5) hipLaunchKernelGGL((mod_gemm_mfma_smallb_kernel<5, 1>), grid, dim3(256), 0, s, a, b8, Ppad, l0);
        else if (nc == 2) hipLaunchKernelGGL((mod_gemm_mfma_smallb_kernel<6, 2>), grid, dim3(256), 0, s, a, b8, Ppad, l0);
        else hipLaunchKernelGGL((mod_gemm_mfma_smallb_kernel<6, 1>), grid, dim3(256), 0, s, a, b8, Ppad, l0);
        MFHE_CHECK_LAUNCH("mod_gemm_mfma_smallb_kernel");
        l0 = l1;
    }
    return MFHE_OK;
}

size_t mod_gemm_mfma_ws(uint32_t P, int L, int D) {
    const uint64_t Ppad = ((uint64_t)P + 63) / 64 * 64;
    // digit planes, then the factored d0 / (c0, c1), then the split decrypt-fused digitize's column partials
    return (size_t)L * D * Ppad * MK + (size_t)L * 2 * Ppad * 8 + (size_t)MFHE_DEC_SPLIT * L * Ppad * 6 * 8;
}

void balanced_digits(uint64_t x, int D, int8_t* out) {
    for (int i = 0; i < D; ++i) {
        int v = (int)(x & 255);
        x >>= 8;
        if (v >= 128) {
            v -= 256;
            ++x;
        }
        out[i] = (int8_t)v;
    }
}

static FoldSrc fold_src(const ModGemmArgs& a) {
    FoldSrc fs;
    fs.qf = a.qf;
    fs.qf_row = a.qf_row;
    fs.qf_step = a.qf_step;
    fs.delta = a.delta;
    fs.qmu = a.qmu;
    fs.lbase = a.lbase;
    fs.Ltot = a.Ltot;
    return fs;
}
// the factored forward's digitize from a fused source (a.qsrc 1..3) into a.Bdig / d0
static int launch_fold_src(const ModGemmArgs& a, uint64_t* d0, int L, uint32_t Ppad, const PlaneCounts& pc,
                           hipStream_t s) {
    const FoldSrc fs = fold_src(a);
    const dim3 gq(L, (Ppad + 127) / 128, FK / 32);
#define MFHE_FOLD_SRC(d, src)                                                                                    \
    hipLaunchKernelGGL((mfma_digitize_fold_kernel<d, src>), gq, dim3(256), 0, s, a.B, a.bL, a.sbK, a.sbY, a.log_n, \
                       a.P, Ppad, a.fold, a.Bdig, d0, pc, fs)
    if (a.qsrc == 1) { if (a.D == 5) MFHE_FOLD_SRC(5, 1); else MFHE_FOLD_SRC(6, 1); }
    else if (a.qsrc == 2) { if (a.D == 5) MFHE_FOLD_SRC(5, 2); else MFHE_FOLD_SRC(6, 2); }
    else if (a.qsrc == 3) { if (a.D == 5) MFHE_FOLD_SRC(5, 3); else MFHE_FOLD_SRC(6, 3); }
    else return set_error(MFHE_EINVAL, "mod_gemm: unknown digitize source");
#undef MFHE_FOLD_SRC
    return MFHE_OK;
}

static int launch_factored(const ModGemmArgs& a, int L, hipStream_t s) {
    const uint32_t Ppad = (a.P + 63) / 64 * 64;
    ModGemmArgs f = a;
    f.d0 = (uint64_t*)(a.Bdig + (size_t)L * a.D * Ppad * MK);
    const dim3 gd((Ppad + 127) / 128, FK / 32, L);
    const PlaneCounts pc = plane_counts(a, L);
    if (a.qsrc) {
        if (int rc = launch_fold_src(a, f.d0, L, Ppad, pc, s)) return rc;
    } else if (a.D == 5) {
        hipLaunchKernelGGL(mfma_digitize_fold_kernel<5>, gd, dim3(256), 0, s, a.B, a.bL, a.sbK, a.sbY, a.log_n,
                           a.P, Ppad, a.fold, a.Bdig, f.d0, pc);
    } else {
        hipLaunchKernelGGL(mfma_digitize_fold_kernel<6>, gd, dim3(256), 0, s, a.B, a.bL, a.sbK, a.sbY, a.log_n, a.P,
                           Ppad, a.fold, a.Bdig, f.d0, pc);
    }
    MFHE_CHECK_LAUNCH("mfma_digitize_fold_kernel");
    if (launch_ring56<1>(f, L, Ppad, s)) {
        MFHE_CHECK_LAUNCH("mod_gemm_mfma_ring56_kernel (factored)");
        return MFHE_OK;
    }
    for (int l0 = 0; l0 < L;) {
        const int d = a.limbD ? std::max(a.limbD[l0], 5) : a.D;
        int l1 = l0 + 1;
        while (l1 < L && (a.limbD ? std::max(a.limbD[l1], 5) : a.D) == d) ++l1;
        const dim3 grid(2 * Ppad / 64, FK / 64, l1 - l0);
        // 0 (auto) and 2: the ring (K = 256: four 64-k stages leave the fill exposed)
        if (d == 5) launch_staged<5, 1>(a.pipe, grid, s, f, Ppad, l0);
        else launch_staged<6, 1>(a.pipe, grid, s, f, Ppad, l0);
        MFHE_CHECK_LAUNCH("mod_gemm_mfma_lds_kernel (factored)");
        l0 = l1;
    }
    return MFHE_OK;
}

// factored inverse: digitize (+ rows 0 / 255 / 256 by dot products), then the 256 x 256 GEMM per run of equal
// digit counts with the MODE 2 epilogue
static int launch_factored_inv(const ModGemmArgs& a, int L, hipStream_t s) {
    const uint32_t Ppad = (a.P + 63) / 64 * 64;
    ModGemmArgs f = a;
    f.cc = (double*)(a.Bdig + (size_t)L * a.D * Ppad * MK);   // the d0 region: L * Ppad * 2 doubles
    const PlaneCounts pc = plane_counts(a, L);
    if (a.dct) {
        // decrypt fused (n = 64 rows: one workgroup per (y, l), 64 columns)
        if (a.log_n != 6 || a.P != 64u * 64u || Ppad != a.P || !a.dsk || !a.dlf || !a.dtw || !a.ditw || !a.dninv)
            return set_error(MFHE_EINVAL, "mod_gemm: the decrypt-fused inverse W-CRT needs n = 64 and the ring tables");
        // MFHE_DEC_SPLIT workgroups per (row, limb), each a share of the 8 panels, the column sums finished after
        constexpr int GS = MFHE_DEC_SPLIT;
        static_assert(GS == 1 || GS == 2 || GS == 4 || GS == 8, "the 8 panels split evenly");
        const int G = GS;
        f.dpart = f.cc + (size_t)L * Ppad * 2;
        const dim3 gr(64, L, GS);
        if (a.D == 5) hipLaunchKernelGGL(mfma_digitize_ifold_dec_kernel<5>, gr, dim3(256), 0, s, f, Ppad, pc);
        else hipLaunchKernelGGL(mfma_digitize_ifold_dec_kernel<6>, gr, dim3(256), 0, s, f, Ppad, pc);
        MFHE_CHECK_LAUNCH("mfma_digitize_ifold_dec_kernel");
        if (G > 1) {
            hipLaunchKernelGGL(dec_colsum_kernel, dim3((Ppad + 255) / 256, L), dim3(256), 0, s, f, Ppad, G);
            MFHE_CHECK_LAUNCH("dec_colsum_kernel");
        }
    } else {
        const dim3 gd(Ppad / 16, L);
        if (a.D == 5) hipLaunchKernelGGL(mfma_digitize_ifold_kernel<5>, gd, dim3(256), 0, s, f, Ppad, pc);
        else hipLaunchKernelGGL(mfma_digitize_ifold_kernel<6>, gd, dim3(256), 0, s, f, Ppad, pc);
        MFHE_CHECK_LAUNCH("mfma_digitize_ifold_kernel");
    }
    if (launch_ring56<2>(f, L, Ppad, s)) {
        MFHE_CHECK_LAUNCH("mod_gemm_mfma_ring56_kernel (factored inverse)");
        return MFHE_OK;
    }
    for (int l0 = 0; l0 < L;) {
        const int d = a.limbD ? std::max(a.limbD[l0], 5) : a.D;
        int l1 = l0 + 1;
        while (l1 < L && (a.limbD ? std::max(a.limbD[l1], 5) : a.D) == d) ++l1;
        const dim3 grid(2 * Ppad / 64, FK / 64, l1 - l0);
        if (d == 5) launch_staged<5, 2>(a.pipe, grid, s, f, Ppad, l0);
        else launch_staged<6, 2>(a.pipe, grid, s, f, Ppad, l0);
        MFHE_CHECK_LAUNCH("mod_gemm_mfma kernel (factored inverse)");
        l0 = l1;
    }
    return MFHE_OK;
}

static bool ring56_all(const ModGemmArgs& f, int L, uint64_t& d6) {
    d6 = 0;
    if (f.pipe != 0 || L > 64) return false;
    for (int l = 0; l < L; ++l) {
        const int d = f.limbD ? std::max(f.limbD[l], 5) : f.D;
        if (d != 5 && d != 6) return false;
        if (d == 6) d6 |= 1ull << l;
    }
    return true;
}
template <int MODE>
static bool ring56_pair_usable() {
    static int ok = -1;
    if (ok < 0) {
        hipFuncAttributes fa{};
        ok = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(mod_gemm_mfma_ring56_pair_kernel<MODE>)) ==
                     hipSuccess &&
             fa.localSizeBytes == 0;
    }
    return ok == 1;
}

// Two independent W-CRT transforms of the same shape (encode's re / im from the W-IDFT's doubles, decode's decrypt-fused
// re / im) as one launch per step: digitize pair, (column sums pair), ring56 GEMM pair -- grids of 2 L limbs, the upper
// half the second component.  Their workgroups share the GPU without a stream fork and its event waits (8-13 us of
// idle per fork or join, profiles/r05_pipeline_chain_trace.txt).  Anything else runs the two sequentially.
int launch_mod_gemm_pair(const ModGemmArgs& a, const ModGemmArgs& b, int L, hipStream_t s) {
    const uint32_t Ppad = (a.P + 63) / 64 * 64;
    uint64_t d6a = 0, d6b = 0;
    const bool inv = a.Adig && a.ifold && a.dct && b.Adig && b.ifold && b.dct && ring56_pair_usable<2>();
    const bool fwd = a.Adig && a.fold && a.qsrc && b.Adig && b.fold && b.qsrc && ring56_pair_usable<1>();
    const bool same = a.P == b.P && a.D == b.D && a.M == 512 && a.K == MK && a.epi && b.epi && a.lds_stage &&
                      a.D >= 5 && a.D <= 6 && 2 * L <= 128 && ring56_all(a, L, d6a) && ring56_all(b, L, d6b) &&
                      d6a == d6b;
    if (!(inv || fwd) || !same || (inv && (a.log_n != 6 || a.P != 64u * 64u || Ppad != a.P || !a.iz || !a.phi))) {
        if (int rc = launch_mod_gemm(a, L, s)) return rc;
        return launch_mod_gemm(b, L, s);
    }
    const PlaneCounts pc = plane_counts(a, L);
    ModGemmArgs f[2] = {a, b};
    const dim3 gg(2 * Ppad / 64, FK / 64, 2 * L);
    if (inv) {
        const int G = MFHE_DEC_SPLIT;
        for (auto& x : f) {
            if (!x.dsk || !x.dlf || !x.dtw || !x.ditw || !x.dninv)
                return set_error(MFHE_EINVAL, "mod_gemm: the decrypt-fused inverse W-CRT needs the ring tables");
            x.cc = (double*)(x.Bdig + (size_t)L * x.D * Ppad * MK);
            x.dpart = x.cc + (size_t)L * Ppad * 2;
        }
        const dim3 gr(64, 2 * L, G);
        if (a.D == 5) hipLaunchKernelGGL(mfma_digitize_ifold_dec_pair_kernel<5>, gr, dim3(256), 0, s, f[0], f[1], Ppad, pc);
        else hipLaunchKernelGGL(mfma_digitize_ifold_dec_pair_kernel<6>, gr, dim3(256), 0, s, f[0], f[1], Ppad, pc);
        MFHE_CHECK_LAUNCH("mfma_digitize_ifold_dec_pair_kernel");
        if (G > 1) {
            hipLaunchKernelGGL(dec_colsum_pair_kernel, dim3((Ppad + 255) / 256, 2 * L), dim3(256), 0, s, f[0], f[1], Ppad, G);
            MFHE_CHECK_LAUNCH("dec_colsum_pair_kernel");
        }
        hipLaunchKernelGGL(mod_gemm_mfma_ring56_pair_kernel<2>, gg, dim3(256), 0, s, f[0], f[1], Ppad, d6a);
        MFHE_CHECK_LAUNCH("mod_gemm_mfma_ring56_pair_kernel (factored inverse)");
        return MFHE_OK;
    }
    for (auto& x : f) x.d0 = (uint64_t*)(x.Bdig + (size_t)L * x.D * Ppad * MK);
    // the two digitizes: one launch when both read the same doubles' rows (encode's re / im), else one each (the
    // encrypt's uniform a and Gaussian e)
    if (!(a.qsrc == 1 && b.qsrc == 1 && a.B == b.B && a.qf_row == b.qf_row && a.qf_step == b.qf_step &&
          a.delta == b.delta)) {
        for (const auto& x : f)
            if (int rc = launch_fold_src(x, x.d0, L, Ppad, pc, s)) return rc;
        MFHE_CHECK_LAUNCH("mfma_digitize_fold_kernel");
        hipLaunchKernelGGL(mod_gemm_mfma_ring56_pair_kernel<1>, gg, dim3(256), 0, s, f[0], f[1], Ppad, d6a);
        MFHE_CHECK_LAUNCH("mod_gemm_mfma_ring56_pair_kernel (factored)");
        return MFHE_OK;
    }
    const FoldSrc fs = fold_src(a);
    FoldPair fp;
    fp.L = L;
    fp.out2 = f[1].Bdig;
    fp.d02 = f[1].d0;
    fp.qf2 = b.qf;
    const dim3 gq(2 * L, (Ppad + 127) / 128, FK / 32);
#define MFHE_FOLD_PAIR(d, src)                                                                                     \
    hipLaunchKernelGGL((mfma_digitize_fold_kernel<d, src, true>), gq, dim3(256), 0, s, a.B, a.bL, a.sbK, a.sbY,   \
                       a.log_n, a.P, Ppad, a.fold, f[0].Bdig, f[0].d0, pc, fs, fp)
    if (a.D == 5) MFHE_FOLD_PAIR(5, 1);
    else MFHE_FOLD_PAIR(6, 1);
#undef MFHE_FOLD_PAIR
    MFHE_CHECK_LAUNCH("mfma_digitize_fold_kernel (pair)");
    hipLaunchKernelGGL(mod_gemm_mfma_ring56_pair_kernel<1>, gg, dim3(256), 0, s, f[0], f[1], Ppad, d6a);
    MFHE_CHECK_LAUNCH("mod_gemm_mfma_ring56_pair_kernel (factored)");
    return MFHE_OK;
}

int launch_mod_gemm(const ModGemmArgs& a, int L, hipStream_t s) {
    if (a.dct && !(a.Adig && a.ifold)) return set_error(MFHE_EINVAL, "mod_gemm: a decrypt-fused B needs the factored inverse");
    if (a.Adig && a.ifold) {
        if (a.M != 512 || a.K != MK || !a.epi || a.D < 5 || a.D > 6 || !a.lds_stage || !a.iz || !a.phi)
            return set_error(MFHE_EINVAL, "mod_gemm: factored inverse W-CRT needs M = K = 512, the FP64 epilogue and D in {5, 6}");
        return launch_factored_inv(a, L, s);
    }
    if (a.Adig && a.fold) {
        if (a.M != 512 || a.K != MK || !a.epi || a.D < 5 || a.D > 6 || !a.lds_stage)
            return set_error(MFHE_EINVAL, "mod_gemm: factored W-CRT needs M = K = 512, the FP64 epilogue and D in {5, 6}");
        return launch_factored(a, L, s);
    }
    if (a.Adig && a.M == 512 && a.K == MK) {
        const uint32_t Ppad = (a.P + 63) / 64 * 64;
        const dim3 gd((Ppad + 255) / 256, MK / 32, L);
        switch (a.D) {
#define MFHE_DIG_CASE(d)                                                                                         \
    case d:                                                                                                      \
        hipLaunchKernelGGL(mfma_digitize_kernel<d>, gd, dim3(256), 0, s, a.B, a.bL, a.sbK, a.sbY, a.log_n, a.P,   \
                           Ppad, a.Bdig, plane_counts(a, L));                                                    \
        break;
            MFHE_DIG_CASE(5)
            MFHE_DIG_CASE(6)
            MFHE_DIG_CASE(7)
            MFHE_DIG_CASE(8)
#undef MFHE_DIG_CASE
            default: return set_error(MFHE_EINVAL, "mod_gemm: MFMA digit count must be 5..8");
        }
        MFHE_CHECK_LAUNCH("mfma_digitize_kernel");
        // one GEMM launch per run of consecutive limbs that need the same number of digits
        for (int l0 = 0; l0 < L;) {
            const int d = a.limbD ? std::max(a.limbD[l0], 5) : a.D;
            int l1 = l0 + 1;
            while (l1 < L && (a.limbD ? std::max(a.limbD[l1], 5) : a.D) == d) ++l1;
            const dim3 grid(Ppad / 64, 512 / 64, l1 - l0);
            switch (d) {
#define MFHE_MFMA_CASE(dd)                                                                                    \
    case dd:                                                                                                  \
        if (a.lds_stage) launch_staged<dd, 0>(a.pipe >= 2 ? a.pipe : 1, grid, s, a, Ppad, l0);                  \
        else hipLaunchKernelGGL(mod_gemm_mfma_kernel<dd>, grid, dim3(256), 0, s, a, Ppad, l0);                 \
        break;
                MFHE_MFMA_CASE(5)
                MFHE_MFMA_CASE(6)
                MFHE_MFMA_CASE(7)
                MFHE_MFMA_CASE(8)
#undef MFHE_MFMA_CASE
                default: return set_error(MFHE_EINVAL, "mod_gemm: MFMA digit count must be 5..8");
            }
            MFHE_CHECK_LAUNCH("mod_gemm_mfma_kernel");
            l0 = l1;
        }
        return MFHE_OK;
    }
    dim3 grid((a.P + TP - 1) / TP, (a.M + TM - 1) / TM, L);
    hipLaunchKernelGGL(mod_gemm_kernel, grid, dim3(NTH), 0, s, a);
    MFHE_CHECK_LAUNCH("mod_gemm_kernel");
    return MFHE_OK;
}

// ---- the per-lane XY product out = A M B in one launch (r06, n = 64) ----
// he.hip xy3 at n = 64: A and B the shared 64 x 64 encoder matrices, M one lane's 64 x 64 block; one workgroup per
// lane, eight waves of 16 x 32 outputs.  Phase 1 is cgemm_mfma_kernel<0>'s T = A M (v_mfma_f64_16x16x4_f64 blocks,
// each output accumulated in the same order, k-step by k-step: first the Ar Br / Ar Bi terms, then -Ai Bi / Ai Br),
// with all of K in LDS at once; T then goes to LDS instead of HBM and phase 2 is out = T B the same way.  So the
// doubles are those of the two launches, without T's round trip and the second launch's fill.  LDS: A / T planes
// [64][65] (the row pitch spreads a fragment's 16 rows over the banks), M / B planes [64][64]: 130.5 KiB, one
// workgroup per CU, two waves per SIMD (four waves: 61.8 us per call; eight: 51.3 us; the two launches ~54 us).
constexpr int XYN = 64, XYP = 65, XYT = 512;   // eight waves: two per SIMD at one workgroup per CU
__global__ __launch_bounds__(XYT, 1) void xy_fused_kernel(const double2* __restrict__ A, const double2* __restrict__ M,
                                                          const double2* __restrict__ Bm, double2* __restrict__ out) {
    __shared__ double Lr[XYN * XYP], Li[XYN * XYP];   // left operand: A, then T   ([row][k])
    __shared__ double Rr[XYN * XYN], Ri[XYN * XYN];   // right operand: M, then B  ([k][col])
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = (w >> 1) * 16, wp = (w & 1) * 32, r = lane & 15, kq = lane >> 4;   // each wave 16 x 32
    const uint64_t lb = (uint64_t)blockIdx.x * XYN * XYN;
    auto load_left = [&](const double2* src) {
#pragma unroll 4
        for (int e = 0; e < XYN * XYN / XYT; ++e) {
            const int idx = t + e * XYT;
            const double2 v = src[idx];
            Lr[(idx >> 6) * XYP + (idx & 63)] = v.x;
            Li[(idx >> 6) * XYP + (idx & 63)] = v.y;
        }
    };
    auto load_right = [&](const double2* src) {
#pragma unroll 4
        for (int e = 0; e < XYN * XYN / XYT; ++e) {
            const int idx = t + e * XYT;
            const double2 v = src[idx];
            Rr[idx] = v.x;
            Ri[idx] = v.y;
        }
    };
    v4d cr[1][2], ci[1][2];
    auto product = [&]() {
#pragma unroll
        for (int i = 0; i < 1; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) cr[i][j] = ci[i][j] = v4d{0, 0, 0, 0};
#pragma unroll 4
        for (int ks = 0; ks < XYN / 4; ++ks) {
            const int k = ks * 4 + kq;
            double ar[1], ai[1], nai[1], br[2], bi[2];
#pragma unroll
            for (int i = 0; i < 1; ++i) {
                ar[i] = Lr[(wm + 16 * i + r) * XYP + k];
                ai[i] = Li[(wm + 16 * i + r) * XYP + k];
                nai[i] = -ai[i];
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                br[j] = Rr[k * XYN + wp + 16 * j + r];
                bi[j] = Ri[k * XYN + wp + 16 * j + r];
            }
#pragma unroll
            for (int i = 0; i < 1; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    cr[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[i], br[j], cr[i][j], 0, 0, 0);
                    ci[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[i], bi[j], ci[i][j], 0, 0, 0);
                }
#pragma unroll
            for (int i = 0; i < 1; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    cr[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(nai[i], bi[j], cr[i][j], 0, 0, 0);
                    ci[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[i], br[j], ci[i][j], 0, 0, 0);
                }
        }
    };
    load_left(A);
    load_right(M + lb);
    __syncthreads();
    product();   // T = A M
    __syncthreads();   // every wave is done reading A and M
#pragma unroll
    for (int i = 0; i < 1; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int m = wm + 16 * i + kq + 4 * g, p = wp + 16 * j + r;
                Lr[m * XYP + p] = cr[i][j][g];
                Li[m * XYP + p] = ci[i][j][g];
            }
    load_right(Bm);
    __syncthreads();
    product();   // out = T B
    double2* o = out + lb;
#pragma unroll
    for (int i = 0; i < 1; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                o[(wm + 16 * i + kq + 4 * g) * XYN + wp + 16 * j + r] = make_double2(cr[i][j][g], ci[i][j][g]);
}

int launch_xy_fused(const double2* A, const double2* M, const double2* B, double2* out, int lanes, hipStream_t s) {
    if (!A || !M || !B || !out || lanes <= 0) return set_error(MFHE_EINVAL, "xy_fused: bad arguments");
    hipLaunchKernelGGL(xy_fused_kernel, dim3((uint32_t)lanes), dim3(XYT), 0, s, A, M, B, out);
    MFHE_CHECK_LAUNCH("xy_fused_kernel");
    return MFHE_OK;
}

// ---- the forward factored W-DFT by Rader's algorithm (r06) ----
// cgemm_mfma_kernel<1> computes, per column p and a = a' + 1, X_a[b] = F_a[0] + sum_{j=1..256} zeta^(b j) F_a[j]
// (b = 1..256, zeta = e^(2 pi i / 257); F_a folded from in[j] and in[j + 257] with omega = e^(2 pi i / 3)) as a
// 256 x 256 complex GEMM.  That is a 257-point DFT: with g = 3 (a primitive root of 257), j = g^n and b = g^-m,
// X_a[g^-m] - F_a[0] = sum_n F_a[g^n] zeta^(g^(n - m)) is the cyclic convolution of a[n] = F_a[g^n] with
// bk[k] = zeta^(g^-k), taken as IFFT_256(FFT_256(a) . FFT_256(bk)) -- 2 x 1024 butterflies per column instead of
// 65536 complex MACs, so the transform becomes bound by its 64 MB of HBM traffic.  Same outputs to rounding
// (~1e-15 relative; the GEMM's are already not the reference's own rounding, HE.cu:1147-1172).
// One workgroup: 8 columns x both a; 16 threads per column, each holding 16 points of each a's FFT: 256 = 16 x 16
// (a 16-point radix-2 FFT in registers over s, the twiddle W256^(t k1), a transpose through LDS, the 16-point FFT
// over t), the product with FFT(bk) / 256, and the inverse the same way.
__device__ __forceinline__ double2 cadd(double2 x, double2 y) { return make_double2(x.x + y.x, x.y + y.y); }
__device__ __forceinline__ double2 csub(double2 x, double2 y) { return make_double2(x.x - y.x, x.y - y.y); }
__device__ __forceinline__ double2 cconj(double2 x) { return make_double2(x.x, -x.y); }
// e^(SIGN 2 pi i k / 16), k = 0..7
template <int SIGN>
__device__ __forceinline__ double2 w16(int k) {
    constexpr double C[8] = {1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173,
                             0.0, -0.38268343236508977173, -0.70710678118654752440, -0.92387953251128675613};
    constexpr double S[8] = {0.0, 0.38268343236508977173, 0.70710678118654752440, 0.92387953251128675613,
                             1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173};
    return make_double2(C[k], SIGN * S[k]);
}
// in-register 16-point DFT, natural order in and out: X[k] = sum_s x[s] e^(SIGN 2 pi i s k / 16)
template <int SIGN>
__device__ __forceinline__ void fft16(double2 (&x)[16]) {
    auto sw = [&](int i, int j) {
        const double2 t = x[i];
        x[i] = x[j];
        x[j] = t;
    };
    sw(1, 8); sw(2, 4); sw(3, 12); sw(5, 10); sw(7, 14); sw(11, 13);   // 4-bit reversal
#pragma unroll
    for (int len = 2; len <= 16; len <<= 1)
#pragma unroll
        for (int i = 0; i < 16; i += len)
#pragma unroll
            for (int j = 0; j < len / 2; ++j) {
                const int k = j * (16 / len);
                const double2 u = x[i + j], v = k == 0 ? x[i + j + len / 2] : cmul(x[i + j + len / 2], w16<SIGN>(k));
                x[i + j] = cadd(u, v);
                x[i + j + len / 2] = csub(u, v);
            }
}
constexpr int RDC = 8;   // columns per workgroup
__global__ __launch_bounds__(RDC * 16) void wdft_rader_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                              uint32_t Pf, const double2* __restrict__ rb,
                                                              const int16_t* __restrict__ gp) {
    __shared__ double2 tw[256];                  // e^(-2 pi i k / 256)
    __shared__ double2 fb[256];                  // FFT(bk) / 256
    __shared__ int16_t sg[512];                  // g^n, g^-m
    __shared__ double2 xs[RDC][2][16][17];       // transposes: [column][a'][row][col], padded
    const int t = threadIdx.x & 15, pc = threadIdx.x >> 4;
    for (int i = threadIdx.x; i < 256; i += RDC * 16) {
        double sn, cs;
        sincospi(-(double)i / 128.0, &sn, &cs);
        tw[i] = make_double2(cs, sn);
        fb[i] = rb[i];
        sg[i] = gp[i];
        sg[256 + i] = gp[256 + i];
    }
    __syncthreads();
    const uint32_t p = blockIdx.x * RDC + pc;
    const bool live = p < Pf;
    const uint32_t pr = live ? p : 0;
    // F_a[j] for a' = 0, 1: omega^(a (j mod 3)) in[j] + omega^(a ((j + 2) mod 3)) in[j + 257] (second term if j <= 254)
    auto fold = [&](int j, double2& f0, double2& f1) {
        const double2 x1 = in[(uint64_t)j * Pf + pr];
        const double2 x2 = j <= 254 ? in[(uint64_t)(j + 257) * Pf + pr] : make_double2(0.0, 0.0);
        const int t3 = j % 3, t3b = (t3 + 2) % 3;
        f0 = cadd(cmul(omega3(t3), x1), cmul(omega3(t3b), x2));
        f1 = cadd(cmul(omega3((2 * t3) % 3), x1), cmul(omega3((2 * t3b) % 3), x2));
    };
    double2 x[2][16];
#pragma unroll
    for (int s = 0; s < 16; ++s) fold(sg[t + 16 * s], x[0][s], x[1][s]);
    double2 F0[2];
    fold(0, F0[0], F0[1]);
    // forward FFT_256 of a[n] = F[g^n], n = t + 16 s: over s, twiddle W256^(t k1), transpose, over t
#pragma unroll
    for (int ap = 0; ap < 2; ++ap) {
        fft16<-1>(x[ap]);
#pragma unroll
        for (int k1 = 1; k1 < 16; ++k1) x[ap][k1] = cmul(x[ap][k1], tw[(t * k1) & 255]);
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) xs[pc][ap][k1][t] = x[ap][k1];
    }
    __syncthreads();
#pragma unroll
    for (int ap = 0; ap < 2; ++ap) {
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) x[ap][tt] = xs[pc][ap][t][tt];   // this thread is now k1 = t
        fft16<-1>(x[ap]);                                                 // A[t + 16 k2] in x[ap][k2]
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) x[ap][k2] = cmul(x[ap][k2], fb[t + 16 * k2]);
        // inverse: over k2 (this thread k1 = t) gives C[t][u]; twiddle e^(+2 pi i u t / 256); transpose; over k1
        fft16<1>(x[ap]);
#pragma unroll
        for (int u = 1; u < 16; ++u) x[ap][u] = cmul(x[ap][u], cconj(tw[(u * t) & 255]));
    }
    __syncthreads();   // every thread has read its transposed row
#pragma unroll
    for (int ap = 0; ap < 2; ++ap)
#pragma unroll
        for (int u = 0; u < 16; ++u) xs[pc][ap][u][t] = x[ap][u];
    __syncthreads();
#pragma unroll
    for (int ap = 0; ap < 2; ++ap) {
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) x[ap][k1] = xs[pc][ap][t][k1];   // this thread is now u = t
        fft16<1>(x[ap]);                                                  // y[t + 16 v] in x[ap][v]
        if (live) {
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int b = sg[256 + t + 16 * v];   // output b = g^-m, m = t + 16 v
                out[(uint64_t)(ap * 256 + b - 1) * Pf + p] = cadd(F0[ap], x[ap][v]);
            }
        }
    }
}

// ---- the inverse factored W-DFT by Rader's algorithm (r06) ----
// cgemm_mfma_kernel<2> + cwdft_inv_dots_kernel: E_a'[r2] = sum_{b=1..256} zeta^(-b r2) y_a'[b], y_a'[b] =
// in[a' 256 + b - 1][p] (r2 = 0..256), then h_j = sum_a' lam1[a'][r2 mod 3] E_a'[r2] (j = r2) and
// h_(r2+257) with lam2, c1 = h_513, c0 = h_512 - c1 phi_511, f_j = h_j - c0 phi_j - c1 phi_(j-1) (j < 512).  For
// r2 != 0 the sum is the cyclic convolution of a[n] = y[g^n] with conj(bk) (E[g^-m] = conv[m]); E[0] = sum_b y[b]
// is FFT(a)[0].  E at r2 = 0, 255, 256 (the c's and f_0, f_257) reach every thread of the column through LDS.
__global__ __launch_bounds__(RDC * 16) void wdft_rader_inv_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                                  double* __restrict__ out_im, uint32_t Pf,
                                                                  const double2* __restrict__ rb,
                                                                  const int16_t* __restrict__ gp,
                                                                  const double2* __restrict__ lam,
                                                                  const int8_t* __restrict__ phi) {
    __shared__ double2 tw[256];
    __shared__ double2 fb[256];
    __shared__ int16_t sg[512];
    __shared__ double2 xs[RDC][2][16][17];
    __shared__ double2 ex[RDC][2][3];            // E_a'[0], E_a'[255], E_a'[256] per column
    const int t = threadIdx.x & 15, pc = threadIdx.x >> 4;
    for (int i = threadIdx.x; i < 256; i += RDC * 16) {
        double sn, cs;
        sincospi(-(double)i / 128.0, &sn, &cs);
        tw[i] = make_double2(cs, sn);
        fb[i] = rb[i];
        sg[i] = gp[i];
        sg[256 + i] = gp[256 + i];
    }
    __syncthreads();
    const uint32_t p = blockIdx.x * RDC + pc;
    const bool live = p < Pf;
    const uint32_t pr = live ? p : 0;
    double2 x[2][16];
#pragma unroll
    for (int ap = 0; ap < 2; ++ap)
#pragma unroll
        for (int s = 0; s < 16; ++s) x[ap][s] = in[(uint64_t)(ap * 256 + sg[t + 16 * s] - 1) * Pf + pr];
#pragma unroll
    for (int ap = 0; ap < 2; ++ap) {
        fft16<-1>(x[ap]);
#pragma unroll
        for (int k1 = 1; k1 < 16; ++k1) x[ap][k1] = cmul(x[ap][k1], tw[(t * k1) & 255]);
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) xs[pc][ap][k1][t] = x[ap][k1];
    }
    __syncthreads();
#pragma unroll
    for (int ap = 0; ap < 2; ++ap) {
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) x[ap][tt] = xs[pc][ap][t][tt];
        fft16<-1>(x[ap]);
        if (t == 0) ex[pc][ap][0] = x[ap][0];   // E[0] = sum_b y[b] = FFT(a)[0]
#pragma unroll
        for (int k2 = 0; k2 < 16; ++k2) x[ap][k2] = cmul(x[ap][k2], fb[t + 16 * k2]);
        fft16<1>(x[ap]);
#pragma unroll
        for (int u = 1; u < 16; ++u) x[ap][u] = cmul(x[ap][u], cconj(tw[(u * t) & 255]));
    }
    __syncthreads();
#pragma unroll
    for (int ap = 0; ap < 2; ++ap)
#pragma unroll
        for (int u = 0; u < 16; ++u) xs[pc][ap][u][t] = x[ap][u];
    __syncthreads();
#pragma unroll
    for (int ap = 0; ap < 2; ++ap) {
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) x[ap][k1] = xs[pc][ap][t][k1];
        fft16<1>(x[ap]);   // E[g^-m] for m = t + 16 v in x[ap][v]
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int r2 = sg[256 + t + 16 * v];
            if (r2 == 255) ex[pc][ap][1] = x[ap][v];
            if (r2 == 256) ex[pc][ap][2] = x[ap][v];
        }
    }
    __syncthreads();
    auto L = [&](int kind, int aa, int t3) { return lam[(kind * 2 + aa) * 3 + t3]; };
    auto comb = [&](int kind, int t3, double2 e0, double2 e1) { return cadd(cmul(L(kind, 0, t3), e0), cmul(L(kind, 1, t3), e1)); };
    const double2 E00 = ex[pc][0][0], E10 = ex[pc][1][0];
    const double2 c1 = comb(1, 1, ex[pc][0][2], ex[pc][1][2]);                         // h_513 (r2 = 256, t = 1)
    const double2 h512 = comb(1, 0, ex[pc][0][1], ex[pc][1][1]);                       // r2 = 255, t = 0
    const double p511 = (double)phi[511];
    const double2 c0 = make_double2(h512.x - c1.x * p511, h512.y - c1.y * p511);
    if (!live) return;
    auto put = [&](int j, double2 h) {   // f_j = h_j - c0 phi_j - c1 phi_(j-1)
        const double f0 = (double)phi[j], f1 = j > 0 ? (double)phi[j - 1] : 0.0;
        const double re = h.x - c0.x * f0 - c1.x * f1, im = h.y - c0.y * f0 - c1.y * f1;
        const uint64_t idx = (uint64_t)j * Pf + p;
        if (out_im) {
            ((double*)out)[idx] = re;
            out_im[idx] = im;
        } else {
            out[idx] = make_double2(re, im);
        }
    };
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int r2 = sg[256 + t + 16 * v], t3 = r2 % 3;
        put(r2, comb(0, t3, x[0][v], x[1][v]));
        if (r2 <= 254) put(r2 + 257, comb(1, t3, x[0][v], x[1][v]));
    }
    if (t == 0) {
        put(0, comb(0, 0, E00, E10));
        put(257, comb(1, 0, E00, E10));
    }
}

int launch_wdft_rader_inv(const double2* in, double2* out, double* out_im, uint32_t Pf, const double2* rb,
                          const int16_t* gp, const double2* lam, const int8_t* phi, hipStream_t s) {
    if (!in || !out || !rb || !gp || !lam || !phi || Pf == 0 || in == out)
        return set_error(MFHE_EINVAL, "wdft_rader_inv: bad arguments");
    hipLaunchKernelGGL(wdft_rader_inv_kernel, dim3((Pf + RDC - 1) / RDC), dim3(RDC * 16), 0, s, in, out, out_im, Pf, rb,
                       gp, lam, phi);
    MFHE_CHECK_LAUNCH("wdft_rader_inv_kernel");
    return MFHE_OK;
}

int launch_wdft_rader(const double2* in, double2* out, uint32_t Pf, const double2* rb, const int16_t* gp, hipStream_t s) {
    if (!in || !out || !rb || !gp || Pf == 0 || in == out) return set_error(MFHE_EINVAL, "wdft_rader: bad arguments");
    hipLaunchKernelGGL(wdft_rader_kernel, dim3((Pf + RDC - 1) / RDC), dim3(RDC * 16), 0, s, in, out, Pf, rb, gp);
    MFHE_CHECK_LAUNCH("wdft_rader_kernel");
    return MFHE_OK;
}

// ---- the per-lane XY transforms by FFT (r06, n = 64) ----
// V[j][k] = zeta^(g_j k), zeta = e^(2 pi i / 256), g_j = 5^j mod 256 (ctx.cpp ensure_xy, encoder.cu:425-444).  Every
// g_j is 1 mod 4 and j -> (g_j - 1) / 4 is a permutation of 0..63, so (V x)[j] = sum_k (x[k] zeta^k) w^(k (g_j-1)/4)
// with w = e^(2 pi i / 64): a 64-point DFT of the twisted column, its output i' landing at j = jinv[i'].  V^-1 =
// V^H / 64 runs backwards: the input permuted to u[i'] = z[jinv[i']], the DFT with e^(-2 pi i / 64), the output
// times zeta^-k / 64.  xy3's out = V M V^T (decode) or V^-1 M V^-T (encode) is the transform of every column, a
// transpose, the transform of every row: 2 x 64 DFTs of 64 points per lane instead of two 64^3 complex GEMMs, so
// the launch is bound by its 64 KB in and out per lane.  The twiddles are single cos / sin values, the GEMMs' V a
// chain of products: equal to rounding (~1e-15 relative), not bit for bit.  One workgroup per lane, eight waves:
// in each pass thread (c, q) holds x[q + 8 s] (s = 0..7) of transform c, runs the 8-point DFT over s and the
// twiddle w^(q k1), and after an exchange through LDS the 8-point DFT over q for k1 = q; the results go back to
// LDS transposed, so the second pass reads rows the way the first read columns.  (Four waves with a 16 x 4
// split: 18.9 / 21.3 us per call.)
constexpr int XFP = 65;   // LDS row pitch (double2)
// in-register 8-point DFT, natural order in and out: X[k] = sum_s x[s] e^(SIGN 2 pi i s k / 8)
template <int SIGN>
__device__ __forceinline__ void fft8(double2 (&x)[8]) {
    auto sw = [&](int i, int j) {
        const double2 t = x[i];
        x[i] = x[j];
        x[j] = t;
    };
    sw(1, 4); sw(3, 6);   // 3-bit reversal
#pragma unroll
    for (int len = 2; len <= 8; len <<= 1)
#pragma unroll
        for (int i = 0; i < 8; i += len)
#pragma unroll
            for (int j = 0; j < len / 2; ++j) {
                const int k = j * (8 / len);
                const double2 u = x[i + j], v = k == 0 ? x[i + j + len / 2] : cmul(x[i + j + len / 2], w16<SIGN>(2 * k));
                x[i + j] = cadd(u, v);
                x[i + j + len / 2] = csub(u, v);
            }
}
template <bool INV>
__global__ __launch_bounds__(512) void xy_fft_kernel(const double2* __restrict__ in, double2* __restrict__ out) {
    __shared__ double2 S[64 * XFP];
    __shared__ double2 tz[256];   // e^(2 pi i m / 256)
    __shared__ int jinv[64];
    constexpr int SG = INV ? -1 : 1;
    const int t = threadIdx.x, c = t & 63, q = t >> 6;
    if (t < 256) {
        double sn, cs;
        sincospi((double)t / 128.0, &sn, &cs);
        tz[t] = make_double2(cs, sn);
    } else if (t < 320) {
        int g = 1;
        for (int i = 0; i < t - 256; ++i) g = (g * 5) & 255;
        jinv[(g - 1) >> 2] = t - 256;
    }
    const uint64_t lb = (uint64_t)blockIdx.x * 4096;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int idx = t + 512 * e;
        S[(idx >> 6) * XFP + (idx & 63)] = in[lb + idx];
    }
    __syncthreads();
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        double2 x[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            const int n = q + 8 * s;
            x[s] = INV ? S[jinv[n] * XFP + c] : cmul(S[n * XFP + c], tz[n]);
        }
        fft8<SG>(x);
#pragma unroll
        for (int k1 = 1; k1 < 8; ++k1) {
            const double2 w = tz[(4 * q * k1) & 255];
            x[k1] = cmul(x[k1], INV ? cconj(w) : w);
        }
        __syncthreads();   // every thread has read its inputs
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) S[(8 * q + k1) * XFP + c] = x[k1];
        __syncthreads();
#pragma unroll
        for (int qq = 0; qq < 8; ++qq) x[qq] = S[(8 * qq + q) * XFP + c];   // k1 = q
        fft8<SG>(x);                                                          // X[q + 8 k2] in x[k2]
        __syncthreads();   // every thread has read the exchange
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2) {
            const int i = q + 8 * k2;
            if (INV) {
                const double2 v = cmul(x[k2], cconj(tz[i]));
                S[c * XFP + i] = make_double2(v.x * 0.015625, v.y * 0.015625);
            } else {
                S[c * XFP + jinv[i]] = x[k2];
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int idx = t + 512 * e;
        out[lb + idx] = S[(idx >> 6) * XFP + (idx & 63)];
    }
}

int launch_xy_fft(const double2* in, double2* out, bool inv, int lanes, hipStream_t s) {
    if (!in || !out || lanes <= 0) return set_error(MFHE_EINVAL, "xy_fft: bad arguments");
    if (inv) hipLaunchKernelGGL(xy_fft_kernel<true>, dim3((uint32_t)lanes), dim3(512), 0, s, in, out);
    else hipLaunchKernelGGL(xy_fft_kernel<false>, dim3((uint32_t)lanes), dim3(512), 0, s, in, out);
    MFHE_CHECK_LAUNCH("xy_fft_kernel");
    return MFHE_OK;
}

int launch_cgemm(const CGemmArgs& a, int batch, hipStream_t s) {
    dim3 grid((a.P + TP - 1) / TP, (a.M + TM - 1) / TM, batch);
    if (a.mfma) {
        if (a.fac == 1) hipLaunchKernelGGL(cgemm_mfma_kernel<1>, grid, dim3(NTH), 0, s, a);
        else if (a.fac == 2) hipLaunchKernelGGL(cgemm_mfma_kernel<2>, grid, dim3(NTH), 0, s, a);
        else hipLaunchKernelGGL(cgemm_mfma_kernel<0>, grid, dim3(NTH), 0, s, a);
        MFHE_CHECK_LAUNCH("cgemm_mfma_kernel");
    } else {
        hipLaunchKernelGGL(cgemm_kernel, grid, dim3(NTH), 0, s, a);
        MFHE_CHECK_LAUNCH("cgemm_kernel");
    }
    return MFHE_OK;
}

}  // namespace mfhe
