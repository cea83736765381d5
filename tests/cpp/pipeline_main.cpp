// End-to-end pipeline driver: the reference's src/main.cu:31-157 flow (encode -> keygen -> encrypt ->
// decrypt+decode at n = 64, phi = 512, L = 11, check max |err| < 1e-4) through the include/core API,
// with a per-stage wall-clock breakdown.  Exit 0 on success.
#include <chrono>
#include <cmath>

#include "HE.cuh"
#include "batched_encoder.cuh"
#include "config.h"
#include "test_util.hpp"

using namespace matrix_fhe;
using clk = std::chrono::steady_clock;

static double ms_since(clk::time_point t0) {
    HIP_OK(hipDeviceSynchronize());
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
    const int n = MATRIX_N, PHI = BATCH_SIZE, L = RNS_NUM_LIMBS, n2 = n * n;
    const size_t cnt = (size_t)PHI * n2, words = (size_t)PHI * L * n2;
    std::printf("=== pipeline: n=%d phi=%d L=%d (%zu complex slots) ===\n", n, PHI, L, cnt);
    auto t0 = clk::now();
    init_he_backend();
    SecretKey sk;
    generate_secret_key(sk, L);
    std::printf("init + keygen: %.1f ms (tables built once per process)\n", ms_since(t0));

    std::vector<hipDoubleComplex> h_in(cnt);
    for (int ell = 0; ell < PHI; ++ell)  // main.cu:62-69 input pattern
        for (int i = 0; i < n2; ++i)
            h_in[(size_t)ell * n2 + i] = make_hipDoubleComplex(ell + i * 0.00001, ell - i * 0.00001);
    hipDoubleComplex* d_in = h2d(h_in);
    uint64_t *pre = dev_alloc<uint64_t>(words), *pim = dev_alloc<uint64_t>(words);
    hipDoubleComplex* d_out = dev_alloc<hipDoubleComplex>(cnt);
    BatchedEncoder enc(n);
    RLWECiphertext ct_re, ct_im;
    allocate_ciphertext(ct_re, L);
    allocate_ciphertext(ct_im, L);

    double te = 0, tc = 0, td = 0;
    for (int r = 0; r <= reps; ++r) {  // rep 0 warms up
        t0 = clk::now();
        enc.encode_to_wntt_eval(d_in, pre, pim);
        const double a = ms_since(t0);
        t0 = clk::now();
        encrypt_pair(pre, pim, sk, ct_re, ct_im);
        const double b = ms_since(t0);
        t0 = clk::now();
        decrypt_and_decode(ct_re, ct_im, sk, d_out);
        const double c = ms_since(t0);
        if (r) te += a, tc += b, td += c;
    }
    if (reps > 0)
        std::printf("per pipeline (mean of %d): encode %.2f ms, encrypt_pair %.2f ms, decrypt_and_decode %.2f ms\n",
                    reps, te / reps, tc / reps, td / reps);
    auto h_out = d2h(d_out, cnt);
    double max_err = 0;
    size_t at = 0;
    for (size_t i = 0; i < cnt; ++i) {
        const double e = std::hypot(h_out[i].x - h_in[i].x, h_out[i].y - h_in[i].y);
        if (e > max_err) max_err = e, at = i;
    }
    std::printf("Global Max Error: %.6e (lane %zu, index %zu)\n", max_err, at / n2, at % n2);
    free_ciphertext(ct_re);
    free_ciphertext(ct_im);
    hipFree(d_in); hipFree(pre); hipFree(pim); hipFree(d_out); hipFree(sk.data);
    const bool ok = max_err < 1e-4;
    std::printf(ok ? ">>> [SUCCESS] pipeline verified\n" : ">>> [FAILURE] error too high\n");
    return ok ? 0 : 1;
}
