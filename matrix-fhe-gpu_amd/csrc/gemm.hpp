// gemm.hpp -- dense contractions on the W and XY axes.
//
//  * modular GEMM  C[m][p] = sum_k A[m][k] B[k][p] mod q   (W-CRT, HE.cu:716-781, 1245-1270)
//    u64 operands (< 2^59), exact u128 accumulation over K = 512, one reduction per output.
//    The reference does an __int128 % per term (HE.cu:742); we reduce once.
//  * complex GEMM  C = A B  in FP64                           (W-DFT HE.cu:1147-1172, w_idft
//    batched_encoder.cu:104-123, XY DFT mat_mul_kernel_complex encoder.cu:318-326)
//
// Both are LDS-tiled 64x64 output tiles, 256 threads, 4x4 outputs per thread.  B and C are
// addressed through a (k|m, pos) -> offset map  k*sK + (pos >> log_n)*sY + (pos & (n-1)) so the
// same kernel serves matrix-major and poly-major layouts (HE.cu:744-746, 773, 778).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mfhe {

struct ModGemmArgs {
    const uint64_t* A;     // [L][M][K] row-major, limb stride aL
    const uint64_t* B;     // limb l at B + l*bL
    uint64_t* C;           // limb l at C + l*cL
    uint64_t* C2 = nullptr;   // factored forward only: a second copy of C, same layout (he.hip: the encrypt's shared a
                              // written into both ciphertexts by the GEMM instead of by the ring kernel)
    uint64_t aL, bL, cL;
    uint64_t sbK, sbY, scM, scY;
    int M, K, log_n;
    uint32_t P;
    const uint64_t* qmu;   // [L][2] (q, floor(2^64/q))
    const uint64_t* r64;   // [L] 2^64 mod q
    // i8 MFMA path (M = K = 512): A pre-split into D balanced base-256 digit planes [L][D][M][K] (limb
    // stride adL bytes), rtab [L][2D-1][2] = (256^s mod q, Shoup), Bdig workspace >= L*D*Ppad*K bytes.
    // Adig == nullptr selects the VALU u128 kernel.
    const int8_t* Adig = nullptr;
    uint64_t adL = 0;
    int D = 0;                   // digit-plane stride (max over limbs)
    const uint64_t* rtab = nullptr;
    int8_t* Bdig = nullptr;
    const int* limbD = nullptr;  // host: digits limb l needs (<= D); null = D for every limb
    const double* epi = nullptr; // [L][8] FP64 epilogue (q, 1/q, centred 2^32k mod q); null = integer epilogue
    bool lds_stage = true;       // LDS-staged MFMA kernel (false: fragments straight from global memory)
    int pipe = 0;                // LDS-staged K pipeline (MFHE_OPT_WCRT_PIPE): 0 auto (factored: ring, dense: two
                                 // 64-k stages), 1 two 64-k stages, 2 4-slot 32-k ring, 3 ring + one-ahead A reads
    // factored forward W-CRT (gemm.hip, 771 = 3 x 257): Adig holds the [L][D][256][256] planes of
    // Z[i][k] = zeta^((i+1)(k+1)) and fold [L][16] its FP64 fold constants; null = dense GEMM
    const double* fold = nullptr;
    uint64_t* d0 = nullptr;      // set by the launcher (workspace after the digit planes)
    // factored inverse W-CRT (gemm.hip): Adig holds the planes of Zi[i][k] = zeta^-((i+1)(k+1)), ifold [L][16]
    // (q, 1/q, lam1[2][3], lam2[2][3]), iz [L][48] the dot-product points and chunk powers, phi the packed Phi_771
    // rows; null = dense
    const double* ifold = nullptr;
    const double* iz = nullptr;
    const uint8_t* phi = nullptr;
    double* cc = nullptr;        // set by the launcher: [L][Ppad][2] (c0, c1) per column (the d0 workspace)
    // factored forward only: where the digitize kernel takes B from (gemm.hip mfma_digitize_fold_kernel<D, SRC>)
    //  qsrc 0: B (residues); 1: the doubles v[r][p] at qf[r * qf_row + p * qf_step], residue round(v delta) mod q
    //  (the encode's RNS decompose fused away); 2: the encrypt's uniform sampler (he.hip uniform_kernel) evaluated
    //  in place, limb lbase + l of Ltot; 3: one centred integer per (r, p) at qf[r * qf_row + p] (the Gaussian
    //  noise, drawn once per coefficient, he.hip gaussian_compact_kernel), the same integer in every limb
    int qsrc = 0;
    const double* qf = nullptr;
    uint64_t qf_row = 0, qf_step = 0;
    double delta = 0.0;
    int lbase = 0, Ltot = 0;
    // factored inverse only (n = 64): B is not read; the digitize kernel forms it as the decrypt of the ciphertext
    // dct (gemm.hip mfma_digitize_ifold_dec_kernel): B[w][l][y][.] = ct.b + INTT(NTT(ct.a) * s) mod q over each
    // X row (ring_row.hpp, he.hip dec_ring_kernel), ct matrix-major, b at dct and a at dct + dtotal
    const uint64_t* dct = nullptr;
    uint64_t dtotal = 0;
    const uint64_t* dsk = nullptr;    // s [w][L][n], NTT form
    const void* dlf = nullptr;        // LimbConst [L]
    const double* dtw = nullptr;      // X-NTT tables [L][n] (ph_f)
    const double* ditw = nullptr;
    const double* dninv = nullptr;    // [L]
    double* dpart = nullptr;          // set by the launcher: [G][L][Ppad][6] column partials of a split launch
};

// bytes of B digit workspace the MFMA path needs for P columns and L limbs at D digits
size_t mod_gemm_mfma_ws(uint32_t P, int L, int D);
// host: balanced base-256 digits of x (< 2^(8D-1)), D in [1, 8]
void balanced_digits(uint64_t x, int D, int8_t* out);

struct CGemmArgs {
    const double2* A;      // batch b at A + b*aB, row-major [M][K] (lda = K)
    const double2* B;      // batch b at B + b*bB, element (k,p) at k*sbK + (p>>log_n)*sbY + (p&(n-1))
    double2* C;            // batch b at C + b*cB, element (m,p) at m*scM + (p>>log_n)*scY + (p&(n-1))
    uint64_t aB, bB, cB;
    uint64_t sbK, sbY, scM, scY;
    int M, K, log_n;
    uint32_t P;
    bool mfma = true;      // f64 MFMA kernel; false = VALU mul-then-add kernel (oracle term order)
    // factored W-DFT (gemm.hip, 771 = 3 x 257, as the W-CRT): 0 dense; 1 forward: A = Z [256][256], B read as
    // F_a[k + 1] folded from in[k + 1], in[k + 258] on load, columns 2 p + a', rows of C a' 256 + m, plus F_a[0];
    // 2 inverse: A = Z^-1, B = in[a' 256 + k][p] in interleaved columns 2 p + a', epilogue lam / Phi_771 as the
    // integer inverse (rows 0 and 257 and (c0, c1) come from cwdft_inv_dots_kernel).  in / out row-major [512][Pf].
    int fac = 0;
    uint32_t Pf = 0;
    const double2* cc = nullptr;    // fac 2: [Pf][2] (c0, c1)
    const double2* lam = nullptr;   // fac 2: [2: lam1, lam2][2: a'][3: t]
    const int8_t* phi = nullptr;    // fac 2: [513] Phi_771 coefficients
    double* Cim = nullptr;          // fac 2 only: planar output -- the real parts at (double*)C, the imaginary at Cim,
                                    // element (row, p) at row * scM + p in each (he.hip encode: the fold then reads
                                    // 8-byte lanes, not every other double of 16-byte pairs)
};

int launch_mod_gemm(const ModGemmArgs& a, int L, hipStream_t s);
// the dense W-CRT forward of one small signed int8 operand shared by every limb (the encrypt's Gaussian noise, |e| <=
// 27): b8 is its one digit plane [K/32][Ppad][32]; a as launch_mod_gemm's dense MFMA arguments (gemm.hip)
int launch_mod_gemm_smallb(const ModGemmArgs& a, const int8_t* b8, int L, hipStream_t s);
// two independent W-CRT transforms of the same shape as one launch per step (gemm.hip; he.hip encode / decode)
int launch_mod_gemm_pair(const ModGemmArgs& a, const ModGemmArgs& b, int L, hipStream_t s);
int launch_cgemm(const CGemmArgs& a, int batch, hipStream_t s);
// the forward factored W-DFT (cgemm_mfma_kernel<1>'s outputs, to rounding) by Rader's algorithm: in / out [512][Pf]
// complex, rb = FFT_256(zeta^(g^-k)) / 256, gp = [g^n, g^-m] (mfhe_ctx d_wdrad / d_wdgp; gemm.hip)
int launch_wdft_rader(const double2* in, double2* out, uint32_t Pf, const double2* rb, const int16_t* gp, hipStream_t s);
// the inverse (cgemm_mfma_kernel<2> + cwdft_inv_dots_kernel, to rounding): rb = the inverse table (d_wdrad + 256),
// lam / phi as CGemmArgs; out_im: planar output (real parts at (double*)out), else interleaved (gemm.hip)
int launch_wdft_rader_inv(const double2* in, double2* out, double* out_im, uint32_t Pf, const double2* rb,
                          const int16_t* gp, const double2* lam, const int8_t* phi, hipStream_t s);
// out = A M B per lane for 64 x 64 complex blocks (A, B shared; M, out [lanes][64][64]) in one launch: the two
// launch_cgemm products of he.hip xy3 without the intermediate's HBM round trip, the same doubles (gemm.hip)
int launch_xy_fused(const double2* A, const double2* M, const double2* B, double2* out, int lanes, hipStream_t s);
// the same products at n = 64 by 64-point FFTs (V = ensure_xy's encoder matrix; inv: V^-1 M V^-T), equal to
// rounding; whole lanes go through LDS, so in == out is allowed (gemm.hip xy_fft_kernel)
int launch_xy_fft(const double2* in, double2* out, bool inv, int lanes, hipStream_t s);
// factored inverse W-DFT, first step: per column the rows r2 = 0, 255, 256 of E_a by dot products (xpow [2][256]:
// zeta^(-255 b), zeta^(-256 b)), then f_0, f_257 into out and (c0, c1) into a.cc (gemm.hip)
int launch_cwdft_inv_dots(const CGemmArgs& a, const double2* in, const double2* xpow, hipStream_t s);

}  // namespace mfhe
