// matrix_fhe_api.hpp -- the reference's include/core host API, re-provided on the MI355X backend.
//
// A caller of Shaibk/Matrix-FHE-GPU's include/core/{config.h, ntt_core.cuh, HE.cuh, encoder.cuh,
// batched_encoder.cuh} keeps its source; the forwarding headers of the same names in this
// directory include this file.  Everything here is implemented in
// matrix-fhe-gpu_amd/csrc/core_api.cpp as thin C++ over the C ABI (include/mfhe.h).
//
// Type mapping: cudaStream_t -> hipStream_t, cuDoubleComplex -> hipDoubleComplex (both double2).
// Behavioural differences:
//   * errors throw matrix_fhe::BackendError instead of exit(1) (HE.cu:411-433, ntt_core.cu:53-67);
//   * table setup is per (n, limbs) context, built once; no static first-caller keying;
//   * batched single launches replace per-poly / per-lane launch loops;
//   * the GPU kernels declared as __global__ in encoder.cuh (dequantize_exact_kernel,
//     crt_compose_centerlift_kernel, mat_mul_kernel_complex) are replaced by host entry points
//     (crt_compose_centerlift below, mfhe_crt_compose_f64, mfhe_xy_dft); kernel symbols are not part of
//     this surface.
#pragma once
#include <hip/hip_complex.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <array>
#include <stdexcept>
#include <string>

class DNTTTable;  // phantom surface, include/phantom/phantom_api.hpp
struct mfhe_ctx;
struct mfhe_comm;

namespace matrix_fhe {

using ::mfhe_ctx;

// ---- parameters (reference include/core/config.h:7-52) ----
constexpr int LOG_N = 16;
constexpr int HE_N = 1 << LOG_N;
constexpr int MATRIX_N = 64;
constexpr int BATCH_SIZE = 512;      // phi(771)
constexpr int BATCH_PRIME_P = 771;
constexpr int PACK_N = MATRIX_N * BATCH_SIZE;
constexpr int POLY_N = PACK_N;
constexpr int RNS_NUM_LIMBS = 11;
constexpr int P_NUM_LIMBS = 3;
constexpr double SCALING_FACTOR = 34359738368.0;  // 2^35
constexpr uint64_t RNS_MODULI[RNS_NUM_LIMBS] = {
    17592186435073ULL, 17182765057ULL, 17184541441ULL, 17186120449ULL, 17186515201ULL, 17186909953ULL,
    17188883713ULL,    17190462721ULL, 17190857473ULL, 17191844353ULL, 17192831233ULL};
constexpr uint64_t P_MODULI[P_NUM_LIMBS] = {18014398515156481ULL, 549757491457ULL, 549759662593ULL};

struct BackendError : std::runtime_error {
    int code;
    BackendError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// ---- NTT layer (reference ntt_core.cuh) ----
struct NTTTable {
    uint64_t* d_psi_powers;        // omega^i, omega = psi4n^4 (ntt_core.cu:110)
    uint64_t* d_psi_inv_powers;    // omega^-i
    uint64_t* d_twist_powers;      // psi4n^i
    uint64_t* d_twist_inv_powers;  // psi4n^-i
    uint64_t* d_n_inv;             // n^-1 per limb
    int modulus_count;
    int n;
};
void init_ntt_tables_manual(int n, int limbs);
void init_ntt_moduli_manual(const uint64_t* h_moduli);
const NTTTable& get_manual_ntt_table();
void init_gl_perm_tables(int n);
void init_gl_twist_tables(int n, int limbs);
const uint32_t* get_gl_perm();
const uint32_t* get_gl_inv_perm();
void apply_gl_perm(const uint64_t* in, uint64_t* out, int limbs, int batch_count, int n, bool inverse,
                   hipStream_t stream = 0);
void xy_ntt_forward_phantom(uint64_t* data, int limbs, int batch_count, int n, hipStream_t stream = 0);
void xy_ntt_backward_phantom(uint64_t* data, int limbs, int batch_count, int n, hipStream_t stream = 0);
void xy_ntt_forward_gl(uint64_t* data, uint64_t* tmp, int limbs, int batch_count, int n, hipStream_t stream = 0);
void xy_ntt_backward_gl(uint64_t* data, uint64_t* tmp, int limbs, int batch_count, int n, hipStream_t stream = 0);
void custom_ntt_forward(uint64_t* data, int limbs, int batch_count, int n, hipStream_t stream = 0);
void custom_ntt_backward(uint64_t* data, int limbs, int batch_count, int n, hipStream_t stream = 0);

// ---- HE backend (reference HE.cuh) ----
struct RLWECiphertext {
    uint64_t* data;   // [b | a], each matrix-major [phi][limbs][n*n]
    int num_limbs;
    bool is_ntt;
    RLWECiphertext() : data(nullptr), num_limbs(0), is_ntt(false) {}
};
struct SecretKey {
    uint64_t* data;   // [phi][limbs][n], X-NTT domain
    int num_limbs;
};
void copy_device_moduli(uint64_t* h_out, int count);
void init_he_backend();
const DNTTTable& get_ntt_table();
const DNTTTable& get_xy_ntt_table();
void wntt_forward_matrix(const uint64_t* in, uint64_t* out, int n, int limbs, int phi, hipStream_t stream = 0);
void wntt_inverse_matrix(const uint64_t* in_eval, uint64_t* out_coeff, int n, int limbs, int phi,
                         hipStream_t stream = 0);
void wntt_forward_centered(const int64_t* in_coeff_centered, int64_t* out_eval_centered, int n, int phi,
                           hipStream_t stream = 0);
void wntt_inverse_centered(const int64_t* in_eval_centered, int64_t* out_coeff_centered, int n, int phi,
                           hipStream_t stream = 0);
void wdft_forward_centered_pair(const int64_t* in_re_centered, const int64_t* in_im_centered, double* out_re_eval,
                                double* out_im_eval, int n, int phi, hipStream_t stream = 0);
void wdft_inverse_pair(const double* in_re_eval, const double* in_im_eval, double* out_re_coeff,
                       double* out_im_coeff, int n, int phi, hipStream_t stream = 0);
void allocate_ciphertext(RLWECiphertext& ct, int limbs);
void free_ciphertext(RLWECiphertext& ct);
void generate_secret_key(SecretKey& sk, int limbs);
void encrypt(const uint64_t* message_coeffs, const SecretKey& sk, RLWECiphertext& ct);
void encrypt_pair(const uint64_t* msg_re, const uint64_t* msg_im, const SecretKey& sk, RLWECiphertext& ct_re,
                  RLWECiphertext& ct_im);
void decrypt_and_decode(const RLWECiphertext& ct_re, const RLWECiphertext& ct_im, const SecretKey& sk,
                        hipDoubleComplex* output_msg);
void decrypt_to_eval_matrix(const RLWECiphertext& ct, const SecretKey& sk, uint64_t* out_eval_matrix);
void add_ciphertexts(const RLWECiphertext& ct1, const RLWECiphertext& ct2, RLWECiphertext& res);
void multiply_ciphertexts_raw(const RLWECiphertext& ct1, const RLWECiphertext& ct2, uint64_t* d0, uint64_t* d1,
                              uint64_t* d2);

// ---- encoders (reference encoder.cuh, batched_encoder.cuh) ----
void crt_compose_centerlift_big(const uint64_t* d_in_rns, uint64_t* d_out_mag, uint8_t* d_out_neg, int n2, int limbs,
                                hipStream_t stream = 0);
// host entry for the __global__ crt_compose_centerlift_kernel (encoder.cu:152-189): the centred value truncated to
// int64 (low magnitude word, sign applied with wrap), <<<ceil(n2/256), 256>>> over one lane's [limbs][n2]
void crt_compose_centerlift(const uint64_t* d_in_rns, int64_t* d_out_centered, int n2, int limbs,
                            hipStream_t stream = 0);

class Encoder {
   public:
    int n;
    hipDoubleComplex* d_V_cx;
    hipDoubleComplex* d_V_cx_T;
    hipDoubleComplex* d_V_inv_cx;
    hipDoubleComplex* d_V_inv_cx_T;
    explicit Encoder(int n);
    ~Encoder();
    Encoder(const Encoder&) = delete;
    Encoder& operator=(const Encoder&) = delete;
    // one lane: quantize P = Vinv M Vinv^T into RNS [limb][n*n] (encoder.cu:446-458)
    void encode(const hipDoubleComplex* d_msg, uint64_t* d_real_rns, uint64_t* d_imag_rns);
    // one lane: exact CRT dequantize then V E V^T (encoder.cu:470-490)
    void decode_lane_from_rns_eval(const uint64_t* d_real_rns, const uint64_t* d_imag_rns, hipDoubleComplex* d_msg);
    void decode_from_eval_complex(const hipDoubleComplex* d_eval, hipDoubleComplex* d_msg);
    void idft2(const hipDoubleComplex* d_eval_xy, hipDoubleComplex* d_coeff_xy);
};

class BatchedEncoder {
   public:
    explicit BatchedEncoder(int n);
    void encode_to_wntt_eval(const hipDoubleComplex* d_msg_batch, uint64_t* d_out_re, uint64_t* d_out_im,
                             hipStream_t stream = 0);
    void unpack_eval_p17(const uint64_t* d_in_re, const uint64_t* d_in_im, uint64_t* d_eval_re, uint64_t* d_eval_im,
                         hipStream_t stream = 0);
    int n() const { return n_; }
    int n2() const { return n2_; }

   private:
    int n_, n2_;
};

// ---- trace GEMM (reference include/core/trace.cuh, include/core/batched_trace.cuh) ----
// Planes [batch][limbs][n][n]; moduli RNS_MODULI.  As in the reference, trace_gemm_batched /
// trace_gemm_ABpT_rns run over all RNS_NUM_LIMBS limbs whatever rns_limbs says (batched_trace.cu:113-116,
// trace.cu:90), map_B_to_Bprime_Xinv_twist and rescale_by_delta_rns likewise (trace.cu:45,137), and the
// rescales multiply limbs >= 3 by 0 (batched_trace.cu:179, trace.cu:151-154).
void map_B_to_Bprime_Xinv_twist(const uint64_t* B_real, const uint64_t* B_imag, uint64_t* Bp_real,
                                uint64_t* Bp_imag, int n, int rns_limbs);
void trace_gemm_ABpT_rns(const uint64_t* A_real, const uint64_t* A_imag, const uint64_t* Bp_real,
                         const uint64_t* Bp_imag, uint64_t* C_real, uint64_t* C_imag, int n, int rns_limbs);
void rescale_by_delta_rns(uint64_t* C_real, uint64_t* C_imag, int n, int rns_limbs, uint64_t inv0, uint64_t inv1,
                          uint64_t inv2);
void map_B_to_Bprime_batched(const uint64_t* B_real, const uint64_t* B_imag, uint64_t* Bp_real, uint64_t* Bp_imag,
                             int n, int rns_limbs, int batch_size);
void trace_gemm_batched(const uint64_t* A_real, const uint64_t* A_imag, const uint64_t* Bp_real,
                        const uint64_t* Bp_imag, uint64_t* C_real, uint64_t* C_imag, int n, int rns_limbs,
                        int batch_size);
void rescale_by_delta_batched(uint64_t* C_real, uint64_t* C_imag, int n, int rns_limbs, int batch_size,
                              uint64_t inv0, uint64_t inv1, uint64_t inv2);

// ---- multi-GPU residue sharding (extension: the reference is single-GPU) ----
// Decode's per-lane compose loop (HE.cu:1653-1668 -> crt_compose_centerlift_big) over limbs sharded across
// GPUs: rank g of G holds limbs [g*limbs/G, (g+1)*limbs/G) of every lane as [lanes][limbs/G][n2] (the
// matrix-major shard of the W-INTT output).  One RCCL communicator per process/GPU.
class ResidueComm {
   public:
    static constexpr int kIdBytes = 128;
    // rank 0 draws the id; the caller hands the same bytes to every rank (MPI, a file, a socket...)
    static std::array<uint8_t, kIdBytes> unique_id();
    ResidueComm(const std::array<uint8_t, kIdBytes>& id, int nranks, int rank);   // collective
    ~ResidueComm();
    ResidueComm(const ResidueComm&) = delete;
    ResidueComm& operator=(const ResidueComm&) = delete;
    int size() const { return nranks_; }
    int rank() const { return rank_; }
    ::mfhe_comm* handle() const { return comm_; }

   private:
    ::mfhe_comm* comm_ = nullptr;
    int nranks_ = 1, rank_ = 0;
};
// Exchange (all-gather, or all-to-all when `alltoall`) + compose of this rank's lane slice
// [g*lanes/G, (g+1)*lanes/G) to centred value / SCALING_FACTOR: d_out [lanes/G][n2] f64, bit-identical to the
// single-GPU compose of the unsharded residues.  Moduli RNS_MODULI[0..limbs).
void crt_recombine_sharded(ResidueComm& comm, const uint64_t* d_shard, double* d_out, int n2, int limbs, int lanes,
                           bool alltoall = false, hipStream_t stream = 0);

// Residue-sharded HE pipeline (BASELINE C4): this rank's limbs [g*limbs_total/G, (g+1)*limbs_total/G) of
// RNS_MODULI[0..limbs_total).  Keys, encoded messages and ciphertexts of a shard carry num_limbs =
// limbs_total/G and are exactly those limbs of the unsharded ones (the uniform sampler of encrypt_pair is
// seeded with the global limb index, HE.cu:564-578).  decrypt_and_decode runs the W-INTT on the shard, the
// RCCL recombine of this rank's lanes (the per-lane compose loop of HE.cu:1653-1668), an all-gather of the
// composed lanes and the W-DFT + XY-DFT: every rank receives the whole [BATCH_SIZE][n*n] message, identical
// to decrypt_and_decode (HE.cu:1691-1708) of the unsharded ciphertexts.
class ResidueShard {
   public:
    ResidueShard(ResidueComm& comm, int limbs_total);
    ~ResidueShard();
    ResidueShard(const ResidueShard&) = delete;
    ResidueShard& operator=(const ResidueShard&) = delete;
    int limb_base() const { return base_; }
    int limbs() const { return lg_; }
    int limbs_total() const { return total_; }
    void generate_secret_key(SecretKey& sk) const;
    void allocate_ciphertext(RLWECiphertext& ct) const;
    // BatchedEncoder::encode_to_wntt_eval on the shard's limbs: d_msg [BATCH_SIZE][n*n] -> [BATCH_SIZE][limbs()][n*n]
    void encode_to_wntt_eval(const hipDoubleComplex* d_msg_batch, uint64_t* d_out_re, uint64_t* d_out_im) const;
    void encrypt_pair(const uint64_t* msg_re, const uint64_t* msg_im, const SecretKey& sk, RLWECiphertext& ct_re,
                      RLWECiphertext& ct_im) const;
    void decrypt_and_decode(const RLWECiphertext& ct_re, const RLWECiphertext& ct_im, const SecretKey& sk,
                            hipDoubleComplex* output_msg, bool alltoall = false, hipStream_t stream = 0) const;
    ::mfhe_ctx* context() const { return ctx_; }

   private:
    ResidueComm& comm_;
    int total_ = 0, lg_ = 0, base_ = 0;
    ::mfhe_ctx* ctx_ = nullptr;   // the shard's moduli, W-CRT tables, limb-shard sampler
    ::mfhe_ctx* all_ = nullptr;   // all limbs_total moduli (CRT tables of the recombine), cached
};

// The C-ABI context (include/mfhe.h) behind this API for a given (n, limbs): moduli RNS_MODULI[0..limbs),
// delta = SCALING_FACTOR, phantom + GL (+ W-CRT when with_wcrt) tables.  Built once, cached.
struct mfhe_ctx* backend_context(int n, int limbs, bool with_wcrt = false);

}  // namespace matrix_fhe
