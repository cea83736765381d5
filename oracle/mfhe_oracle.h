/*
 * mfhe_oracle.h -- CPU restatement of Shaibk/Matrix-FHE-GPU's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker: it may be
 * loaded by tests/, by __graft_entry__.smoke() and by bench.py's cpu_baseline
 * leg, and by nothing else.  The product (matrix-fhe-gpu_amd/) never links or
 * calls it.
 *
 * Every function restates the reference algorithm it names (file:line under
 * /root/reference) in plain C with exact integer arithmetic
 * (unsigned __int128).  The reference itself cannot be built in this
 * container (no nvcc; its phantom-fhe submodule is empty), so the oracle is
 * pinned against the reference's own known-answer tests (SURVEY.md §4/§8c,
 * see tests/test_oracle_kat.py) rather than against reference outputs.
 *
 * Layouts (u64 unless noted):
 *   batch layout       [npoly][L][N]            (phantom fnwt_1d per poly)
 *   matrix-major       [phi][L][n*n]            (HE.cu:17-26)
 *   poly-major         [phi*n][L][n]            (HE.cu:744-746)
 *   wide CRT output    mag [count][W] u64 + neg [count] u8  (encoder.cu:191-230)
 *   complex            interleaved doubles (re, im)
 */
#ifndef MFHE_ORACLE_H
#define MFHE_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- number theory (ntt_core.cu:24-70, HE.cu:108-133) ----------- */
uint64_t orc_mulmod(uint64_t a, uint64_t b, uint64_t q);
uint64_t orc_powmod(uint64_t a, uint64_t e, uint64_t q);
uint64_t orc_invmod(uint64_t a, uint64_t q);
int      orc_is_prime(uint64_t n);
/* Largest `count` primes q < 2^bits with q == 1 (mod m), descending. Returns count found. */
int      orc_gen_primes(int bits, uint64_t m, int count, uint64_t* out);
/* SEAL/phantom try_minimal_primitive_root(degree, q): smallest primitive degree-th root. */
uint64_t orc_minimal_primitive_root(uint64_t degree, uint64_t q);
/* Reference get_psi (ntt_core.cu:49-70): first g^((q-1)/4n), g=2,3,.., with order 4n. 0 if none. */
uint64_t orc_get_psi4n(uint64_t q, int n);
/* Reference h_find_eta (HE.cu:119-133): first element of exact order 771. 0 if none. */
uint64_t orc_find_eta(uint64_t q);

/* ---------------- phantom-convention negacyclic NTT ---------- */
/* Host tables of phantom::arith::NTT(log_n, q): tw[k] = psi^brev(k), itw[k] = psi^-brev(k),
 * itw[1] premultiplied by n^-1; Shoup companions floor(w*2^64/q). Each array has n entries. */
void orc_phantom_tables(int log_n, uint64_t q, uint64_t* tw, uint64_t* tw_shoup,
                        uint64_t* itw, uint64_t* itw_shoup, uint64_t* n_inv, uint64_t* n_inv_shoup);
/* Batched forward/inverse over [npoly][L][N]; limb l of every poly uses moduli[l].
 * Forward output: bit-reversed evaluations a(psi^(2 brev(i)+1)), canonical [0,q). */
void orc_phantom_fwd(uint64_t* data, size_t npoly, int L, int log_n, const uint64_t* moduli);
void orc_phantom_inv(uint64_t* data, size_t npoly, int L, int log_n, const uint64_t* moduli);
/* Same, single-threaded (CPU baseline with cores = 1). */
void orc_phantom_fwd_1t(uint64_t* data, size_t npoly, int L, int log_n, const uint64_t* moduli);

/* ---------------- reference GL custom NTT (ntt_core.cu) ----------------------- */
/* custom_ntt_forward/backward (ntt_core.cu:394-431): cyclic DIT with omega = psi4n^4. */
void orc_custom_ntt_fwd(uint64_t* data, size_t npoly, int L, int n, const uint64_t* moduli);
void orc_custom_ntt_bwd(uint64_t* data, size_t npoly, int L, int n, const uint64_t* moduli);
/* xy_ntt_forward_gl / backward_gl (ntt_core.cu:462-481): evaluation mod X^n - i. */
void orc_gl_ntt_fwd(uint64_t* data, size_t npoly, int L, int n, const uint64_t* moduli);
void orc_gl_ntt_bwd(uint64_t* data, size_t npoly, int L, int n, const uint64_t* moduli);
/* init_gl_perm_tables (ntt_core.cu:150-173) and apply_gl_perm (ntt_core.cu:433-441). */
void orc_gl_perm_table(int n, uint32_t* perm, uint32_t* inv_perm);
void orc_gl_perm(const uint64_t* in, uint64_t* out, size_t npoly, int L, int n, int inverse);

/* ---------------- W-CRT over Phi_771 (HE.cu) ----------------------------------- */
/* k_wntt_exp order (HE.cu:72-105 == batched_encoder.cu:276-282): 512 entries. */
void orc_wcrt_exp(uint16_t* exp512);
/* V[w][r] = (eta^exp[w])^r ; Vinv_T[w][r] = V^-1[r][w]  (HE.cu:237-273). gauss=1 restates the
 * reference Gauss-Jordan (HE.cu:135-185); gauss=0 uses exact Lagrange interpolation (same
 * unique inverse, O(phi^2)). Returns 0 on success. */
int  orc_wcrt_tables(uint64_t q, uint64_t* V, uint64_t* Vinv_T, int gauss);
/* wntt_forward_matrix_kernel (HE.cu:716-747): matrix-major in -> poly-major out.
 * V_all / Vinv_T_all: [L][512][512]. */
void orc_wntt_forward_matrix(const uint64_t* in, uint64_t* out, int n, int L, int phi,
                             const uint64_t* moduli, const uint64_t* V_all);
/* wntt_inverse_matrix_kernel (HE.cu:751-781): poly-major in -> matrix-major out. */
void orc_wntt_inverse_matrix(const uint64_t* in, uint64_t* out, int n, int L, int phi,
                             const uint64_t* moduli, const uint64_t* Vinv_T_all);
/* wntt_forward_vector_kernel (HE.cu:1245-1270): [phi][L][n] -> [phi][L][n]. */
void orc_wntt_forward_vector(const uint64_t* in, uint64_t* out, int n, int L, int phi,
                             const uint64_t* moduli, const uint64_t* V_all);
/* wntt_forward_centered_kernel / wntt_inverse_centered_kernel (HE.cu:1029-1114). */
void orc_wntt_forward_centered(const int64_t* in, int64_t* out, int n, int phi, int L,
                               const uint64_t* moduli, const uint64_t* V_all, int W);
void orc_wntt_inverse_centered(const int64_t* in, int64_t* out, int n, int phi,
                               const uint64_t* moduli, const uint64_t* Vinv_T_all);

/* ---------------- wide CRT (encoder.cu:341-421, 191-230; HE.cu:917-924,1007-1027) ---- */
/* Minimum words: ceil((bitlen(Q)+1)/64). */
int  orc_crt_min_words(const uint64_t* moduli, int L);
/* M [L][W], inv [L], Q [W], Q_half [W]. Returns 0, or -1 if W too small. */
int  orc_crt_tables(const uint64_t* moduli, int L, int W, uint64_t* M, uint64_t* inv,
                    uint64_t* Q, uint64_t* Q_half);
/* crt_compose_centerlift_big over [npoly][L][N] -> mag [npoly][N][W], neg [npoly][N]. */
void orc_crt_compose(const uint64_t* in, size_t npoly, int L, size_t N, const uint64_t* moduli,
                     int W, uint64_t* mag, uint8_t* neg);
void orc_crt_compose_1t(const uint64_t* in, size_t npoly, int L, size_t N, const uint64_t* moduli,
                        int W, uint64_t* mag, uint8_t* neg);
/* crt_compose_centerlift_kernel (encoder.cu:152-189): centred value truncated to int64 */
void orc_crt_compose_i64(const uint64_t* in, size_t npoly, int L, size_t N, const uint64_t* moduli, int W,
                         int64_t* out);
/* OpenMP threads of the parallel entry points (bench cpu_baseline) */
void orc_set_threads(int n);
int orc_max_threads(void);
/* compose_big_pair_to_complex_by_delta (HE.cu:1007-1027), per value: out[i] = +-big/delta. */
void orc_big_to_f64(const uint64_t* mag, const uint8_t* neg, size_t count, int W, double delta,
                    double* out, size_t out_stride);
/* quantize_coeff_to_rns_kernel (batched_encoder.cu:125-152) = RNS decompose:
 * in[i*in_stride] for i in [npoly*N) -> out [npoly][L][N]:  x = llround(z*delta); x mod q. */
void orc_rns_decompose(const double* in, size_t in_stride, size_t npoly, size_t N, int L,
                       const uint64_t* moduli, double delta, uint64_t* out);
void orc_rns_decompose_1t(const double* in, size_t in_stride, size_t npoly, size_t N, int L,
                          const uint64_t* moduli, double delta, uint64_t* out);

/* ---------------- FP64 encoder pieces (encoder.cu, HE.cu, batched_encoder.cu) ---------- */
/* Encoder::init_complex_matrices (encoder.cu:425-444): V, V^T, Vinv, Vinv^T (n*n complex each). */
void orc_encoder_matrices(int n, double* V, double* VT, double* Vinv, double* VinvT);
/* mat_mul_kernel_complex (encoder.cu:318-326): C = A*B. */
void orc_cmatmul(const double* A, const double* B, double* C, int n);
/* init_wdft_tables (HE.cu:275-310): V[w][r], Vinv_T[w][r] = V^-1[r][w]; complex Gauss-Jordan. */
int  orc_wdft_tables(double* V, double* Vinv_T);
/* w_idft_kernel (batched_encoder.cu:104-123): out[r][pos] = sum_w in[w][pos]*invT[w][r]. */
void orc_w_idft(const double* in, double* out, const double* Vinv_T, int n2, int phi);
/* wdft_forward_complex_kernel (HE.cu:1147-1172): out[w][pos] = sum_r in[r][pos]*V[w][r]. */
void orc_wdft_forward(const double* in, double* out, const double* V, int n2, int phi);

/* ---------------- samplers / ring ops (HE.cu:509-713, 1330-1368) ----------------------- */
void orc_ternary_secret(uint64_t* s, int phi, int L, int n, const uint64_t* moduli);
void orc_uniform_random(uint64_t* a, int phi, int L, int n, const uint64_t* moduli);
void orc_gaussian_noise(uint64_t* e, int phi, int L, int n, const uint64_t* moduli);
void orc_matrix_to_poly(const uint64_t* in, uint64_t* out, int n, int L, int phi);
void orc_poly_to_matrix(const uint64_t* in, uint64_t* out, int n, int L, int phi);

/* ---------------- end-to-end reference pipelines (reference geometry) ------------------ */
/* Context for the pipelines below: tables for (n, L, moduli, delta). */
typedef struct orc_he orc_he;
orc_he* orc_he_create(int n, int L, const uint64_t* moduli, double delta, int gauss);
void    orc_he_destroy(orc_he* h);
/* BatchedEncoder::encode_to_wntt_eval (batched_encoder.cu:161-228): msg [phi][n2] complex ->
 * out_re/out_im matrix-major [phi][L][n2]. */
void orc_he_encode(orc_he* h, const double* msg, uint64_t* out_re, uint64_t* out_im);
/* generate_secret_key (HE.cu:1272-1307): sk [phi][L][n] in X-NTT(phantom) domain. */
void orc_he_keygen(orc_he* h, uint64_t* sk);
/* encrypt_pair (HE.cu:1455-1552): ct = [b | a] each matrix-major [phi][L][n2]. */
void orc_he_encrypt_pair(orc_he* h, const uint64_t* m_re, const uint64_t* m_im, const uint64_t* sk,
                         uint64_t* ct_re, uint64_t* ct_im);
/* decrypt_to_eval (HE.cu:1553-1601): poly-major m = b + INTT(NTT(a) * s). */
void orc_he_decrypt_to_eval(orc_he* h, const uint64_t* ct, const uint64_t* sk, uint64_t* out_poly);
/* decode_eval_pair_to_complex (HE.cu:1619-1689): poly-major eval pair -> msg [phi][n2] complex. */
void orc_he_decode(orc_he* h, const uint64_t* eval_re, const uint64_t* eval_im, double* msg);
/* Intermediates for stage-by-stage parity. */
void orc_he_decode_stages(orc_he* h, const uint64_t* eval_re, const uint64_t* eval_im,
                          uint64_t* coeff_re, uint64_t* coeff_im, uint64_t* mag_re, uint8_t* neg_re,
                          uint64_t* mag_im, uint8_t* neg_im, double* coeff_cx, double* eval_cx, double* msg);
int     orc_he_words(orc_he* h);
const uint64_t* orc_he_V(orc_he* h);
const uint64_t* orc_he_VinvT(orc_he* h);

/* ---------------- trace GEMM (batched_trace.cu:37-197, trace.cu:30-161) ----------------- */
/* Layout [batch][L][n][n] per real / imaginary plane; limb l uses moduli[l]. */
void orc_trace_map_bprime(const uint64_t* Br, const uint64_t* Bi, uint64_t* Bpr, uint64_t* Bpi, int n, int L,
                          size_t batch, const uint64_t* moduli);
void orc_trace_gemm(const uint64_t* Ar, const uint64_t* Ai, const uint64_t* Br, const uint64_t* Bi, uint64_t* Cr,
                    uint64_t* Ci, int n, int L, size_t batch, const uint64_t* moduli);
void orc_trace_rescale(uint64_t* Cr, uint64_t* Ci, int n, int L, size_t batch, const uint64_t* moduli,
                       const uint64_t* inv);

/* ---------------- synthetic inputs ----------------
 * Not a reference function: the deterministic input generator shared by tests/golden/make_digests.py
 * and the full-shape GPU parity tests, so both sides see identical inputs.  Element i of a
 * [npoly][L][N] batch (i counted from poly `poly0`) is splitmix64(seed + i) mod q_l; message i is
 * splitmix64(seed + i) mapped to a double in [-1, 1) (53 random bits). */
uint64_t orc_splitmix64(uint64_t x);
void orc_fill_residues(uint64_t* out, size_t npoly, int L, size_t N, const uint64_t* moduli, uint64_t seed,
                       size_t poly0);
void orc_fill_messages(double* out, size_t count, uint64_t seed, size_t idx0);

#ifdef __cplusplus
}
#endif
#endif
