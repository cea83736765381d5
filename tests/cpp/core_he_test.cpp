// HE / encoder layer through the reference's own API names (HE.cuh, encoder.cuh, batched_encoder.cuh).
// Restates the checks of test_encode_decode_loop.cu / test_wcrt_roundtrip.cu / test_encode_decode_wcrt.cu
// plus the ciphertext ops of HE.cu:1710-1740, verified on the host.
#include <cmath>
#include <complex>

#include "HE.cuh"
#include "batched_encoder.cuh"
#include "config.h"
#include "batched_trace.cuh"
#include "encoder.cuh"
#include "trace.cuh"
#include "test_util.hpp"

using namespace matrix_fhe;

int main() {
    const int n = MATRIX_N, n2 = n * n, L = RNS_NUM_LIMBS, PHI = BATCH_SIZE;
    uint64_t seed = 0x4D46484500000001ull;
    auto urand = [&](void) { return (double)(splitmix(seed) >> 11) * 0x1.0p-53; };
    init_he_backend();

    // ---- Encoder lane round trip (encoder.cu:446-501) ----
    std::printf("[encoder lane]\n");
    {
        Encoder enc(n);
        std::vector<hipDoubleComplex> m(n2);
        for (auto& v : m) v = make_hipDoubleComplex(2 * urand() - 1, 2 * urand() - 1);
        hipDoubleComplex* dm = h2d(m);
        uint64_t *re = dev_alloc<uint64_t>((size_t)L * n2), *im = dev_alloc<uint64_t>((size_t)L * n2);
        enc.encode(dm, re, im);
        auto hre = d2h(re, (size_t)L * n2);
        for (int l = 0; l < L; ++l) EXPECT(hre[(size_t)l * n2 + 5] < RNS_MODULI[l], "residue range");
        hipDoubleComplex* out = dev_alloc<hipDoubleComplex>(n2);
        enc.decode_lane_from_rns_eval(re, im, out);
        auto ho = d2h(out, n2);
        double err = 0;
        for (int i = 0; i < n2; ++i) err = std::max(err, std::hypot(ho[i].x - m[i].x, ho[i].y - m[i].y));
        std::printf("  max err %.3e\n", err);
        EXPECT(err < 1e-6, "lane decode(encode(m)) err %.3e", err);
        // idft2 then decode_from_eval_complex is the identity
        enc.idft2(dm, out);
        hipDoubleComplex* back = dev_alloc<hipDoubleComplex>(n2);
        enc.decode_from_eval_complex(out, back);
        auto hb = d2h(back, n2);
        err = 0;
        for (int i = 0; i < n2; ++i) err = std::max(err, std::hypot(hb[i].x - m[i].x, hb[i].y - m[i].y));
        EXPECT(err < 1e-10, "xy dft(idft) err %.3e", err);
        hipFree(dm); hipFree(re); hipFree(im); hipFree(out); hipFree(back);
    }

    // ---- crt_compose_centerlift_big (encoder.cu:191-245): centred values incl. > 64 bits ----
    std::printf("[crt compose]\n");
    {
        const int cnt = 6;
        const __int128 vals[cnt] = {0, 1, -1, (__int128)123456789 << 70, -((__int128)987654321 << 64) - 17,
                                    ((__int128)1 << 100) + 5};
        std::vector<uint64_t> rns((size_t)L * cnt);
        for (int l = 0; l < L; ++l)
            for (int i = 0; i < cnt; ++i) {
                __int128 r = vals[i] % (__int128)RNS_MODULI[l];
                if (r < 0) r += RNS_MODULI[l];
                rns[(size_t)l * cnt + i] = (uint64_t)r;
            }
        uint64_t* din = h2d(rns);
        uint64_t* mag = dev_alloc<uint64_t>(7 * cnt);
        uint8_t* neg = dev_alloc<uint8_t>(cnt);
        crt_compose_centerlift_big(din, mag, neg, cnt, L);
        auto hm = d2h(mag, 7 * cnt);
        auto hn = d2h(neg, cnt);
        for (int i = 0; i < cnt; ++i) {
            const unsigned __int128 a = (unsigned __int128)(vals[i] < 0 ? -vals[i] : vals[i]);
            EXPECT(hm[7 * i] == (uint64_t)a && hm[7 * i + 1] == (uint64_t)(a >> 64), "mag %d", i);
            for (int w = 2; w < 7; ++w) EXPECT(hm[7 * i + w] == 0, "mag %d word %d", i, w);
            EXPECT(hn[i] == (vals[i] < 0), "sign %d", i);
        }
        hipFree(din); hipFree(mag); hipFree(neg);
    }

    // ---- sharded recombine through a 1-rank RCCL communicator == single-GPU compose (extension) ----
    std::printf("[crt recombine, 1-rank RCCL]\n");
    {
        const int lanes = 4, cnt = 64;
        std::vector<uint64_t> rns((size_t)lanes * L * cnt);
        uint64_t s2 = 99;
        for (int w = 0; w < lanes; ++w)
            for (int i = 0; i < cnt; ++i) {
                const int64_t v = (int64_t)(splitmix(s2) >> 20) - (1ll << 43);
                for (int l = 0; l < L; ++l) {
                    int64_t r = v % (int64_t)RNS_MODULI[l];
                    rns[((size_t)w * L + l) * cnt + i] = (uint64_t)(r < 0 ? r + (int64_t)RNS_MODULI[l] : r);
                }
            }
        uint64_t* din = h2d(rns);
        double* out = dev_alloc<double>((size_t)lanes * cnt);
        ResidueComm comm(ResidueComm::unique_id(), 1, 0);
        for (int a2a = 0; a2a < 2; ++a2a) {
            crt_recombine_sharded(comm, din, out, cnt, L, lanes, a2a != 0);
            auto ho = d2h(out, (size_t)lanes * cnt);
            s2 = 99;
            for (size_t i = 0; i < ho.size(); ++i) {
                const int64_t v = (int64_t)(splitmix(s2) >> 20) - (1ll << 43);
                EXPECT(ho[i] == (double)v / SCALING_FACTOR, "recombine value %zu (alltoall %d)", i, a2a);
            }
        }
        hipFree(din); hipFree(out);
    }

    // ---- W-CRT forward / inverse exact round trip (HE.cu:437-452) ----
    std::printf("[wcrt]\n");
    const size_t words = (size_t)PHI * L * n2;
    std::vector<uint64_t> x(words);
    for (size_t i = 0; i < words; ++i) x[i] = splitmix(seed) % RNS_MODULI[(i / n2) % L];
    uint64_t *dx = h2d(x), *dev = dev_alloc<uint64_t>(words), *dback = dev_alloc<uint64_t>(words);
    wntt_forward_matrix(dx, dev, n, L, PHI);
    wntt_inverse_matrix(dev, dback, n, L, PHI);
    EXPECT(d2h(dback, words) == x, "wntt inverse(forward(x)) == x");

    // ---- ciphertext add / tensor (HE.cu:631-669,1710-1740) on matrix-major [b | a] ----
    std::printf("[ct ops]\n");
    {
        RLWECiphertext c1, c2, r;
        allocate_ciphertext(c1, L);
        allocate_ciphertext(c2, L);
        allocate_ciphertext(r, L);
        std::vector<uint64_t> h1(2 * words), h2(2 * words);
        for (size_t i = 0; i < 2 * words; ++i) {
            const uint64_t q = RNS_MODULI[((i % words) / n2) % L];
            h1[i] = splitmix(seed) % q;
            h2[i] = splitmix(seed) % q;
        }
        HIP_OK(hipMemcpy(c1.data, h1.data(), 2 * words * 8, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(c2.data, h2.data(), 2 * words * 8, hipMemcpyHostToDevice));
        add_ciphertexts(c1, c2, r);
        auto hr = d2h(r.data, 2 * words);
        uint64_t *d0 = dev_alloc<uint64_t>(words), *d1 = dev_alloc<uint64_t>(words), *d2 = dev_alloc<uint64_t>(words);
        multiply_ciphertexts_raw(c1, c2, d0, d1, d2);
        auto v0 = d2h(d0, words), v1 = d2h(d1, words), v2 = d2h(d2, words);
        size_t bad = 0;
        for (size_t i = 0; i < words; i += 97) {
            const uint64_t q = RNS_MODULI[(i / n2) % L];
            const uint64_t b1 = h1[i], a1 = h1[words + i], b2 = h2[i], a2 = h2[words + i];
            bad += hr[i] != (b1 + b2) % q;
            bad += hr[words + i] != (a1 + a2) % q;
            bad += v0[i] != mulmod(b1, b2, q);
            bad += v1[i] != (mulmod(b1, a2, q) + mulmod(a1, b2, q)) % q;
            bad += v2[i] != mulmod(a1, a2, q);
        }
        EXPECT(bad == 0, "ct add / tensor mismatches %zu", bad);
        free_ciphertext(c1); free_ciphertext(c2); free_ciphertext(r);
        hipFree(d0); hipFree(d1); hipFree(d2);
    }

    // ---- encrypt -> add -> decrypt: decode is linear, so dec(ct(m1) + ct(m2)) ~ m1 + m2 ----
    std::printf("[encrypt + add + decrypt]\n");
    {
        const size_t cnt = (size_t)PHI * n2;
        std::vector<hipDoubleComplex> m1(cnt), m2(cnt);
        for (size_t i = 0; i < cnt; ++i) {
            m1[i] = make_hipDoubleComplex(urand() - 0.5, urand() - 0.5);
            m2[i] = make_hipDoubleComplex(urand() - 0.5, urand() - 0.5);
        }
        hipDoubleComplex *dm1 = h2d(m1), *dm2 = h2d(m2), *dout = dev_alloc<hipDoubleComplex>(cnt);
        uint64_t *e1r = dev_alloc<uint64_t>(words), *e1i = dev_alloc<uint64_t>(words);
        uint64_t *e2r = dev_alloc<uint64_t>(words), *e2i = dev_alloc<uint64_t>(words);
        BatchedEncoder be(n);
        be.encode_to_wntt_eval(dm1, e1r, e1i);
        be.encode_to_wntt_eval(dm2, e2r, e2i);
        SecretKey sk;
        generate_secret_key(sk, L);
        RLWECiphertext c1r, c1i, c2r, c2i;
        for (auto* c : {&c1r, &c1i, &c2r, &c2i}) allocate_ciphertext(*c, L);
        encrypt_pair(e1r, e1i, sk, c1r, c1i);
        encrypt_pair(e2r, e2i, sk, c2r, c2i);
        add_ciphertexts(c1r, c2r, c1r);
        add_ciphertexts(c1i, c2i, c1i);
        decrypt_and_decode(c1r, c1i, sk, dout);
        auto ho = d2h(dout, cnt);
        double err = 0;
        for (size_t i = 0; i < cnt; ++i)
            err = std::max(err, std::hypot(ho[i].x - m1[i].x - m2[i].x, ho[i].y - m1[i].y - m2[i].y));
        std::printf("  max err %.3e\n", err);
        EXPECT(err < 1e-3, "homomorphic add err %.3e", err);

        // residue-sharded pipeline through a 1-rank RCCL communicator: every stage equals the unsharded one
        std::printf("[residue shard, 1-rank RCCL]\n");
        {
            ResidueComm comm(ResidueComm::unique_id(), 1, 0);
            ResidueShard sh(comm, L);
            EXPECT(sh.limb_base() == 0 && sh.limbs() == L && sh.limbs_total() == L, "shard geometry");
            SecretKey ssk;
            sh.generate_secret_key(ssk);
            EXPECT(d2h(ssk.data, (size_t)PHI * L * n) == d2h(sk.data, (size_t)PHI * L * n), "shard keygen");
            uint64_t *s1r = dev_alloc<uint64_t>(words), *s1i = dev_alloc<uint64_t>(words);
            sh.encode_to_wntt_eval(dm1, s1r, s1i);
            EXPECT(d2h(s1r, words) == d2h(e1r, words) && d2h(s1i, words) == d2h(e1i, words), "shard encode");
            RLWECiphertext sr, si;
            sh.allocate_ciphertext(sr);
            sh.allocate_ciphertext(si);
            sh.encrypt_pair(s1r, s1i, ssk, sr, si);
            RLWECiphertext ur, ui;
            allocate_ciphertext(ur, L);
            allocate_ciphertext(ui, L);
            encrypt_pair(e1r, e1i, sk, ur, ui);
            EXPECT(d2h(sr.data, 2 * words) == d2h(ur.data, 2 * words), "shard encrypt_pair (re)");
            EXPECT(d2h(si.data, 2 * words) == d2h(ui.data, 2 * words), "shard encrypt_pair (im)");
            decrypt_and_decode(ur, ui, sk, dout);
            const auto ref = d2h(dout, cnt);
            hipDoubleComplex* dsh = dev_alloc<hipDoubleComplex>(cnt);
            for (int a2a = 0; a2a < 2; ++a2a) {
                sh.decrypt_and_decode(sr, si, ssk, dsh, a2a != 0);
                const auto got = d2h(dsh, cnt);
                size_t bad = 0;
                for (size_t i = 0; i < cnt; ++i) bad += got[i].x != ref[i].x || got[i].y != ref[i].y;
                EXPECT(bad == 0, "sharded decrypt_and_decode != unsharded (%zu values, alltoall %d)", bad, a2a);
            }
            bool threw = false;
            try { ResidueShard bad_shard(comm, 0); } catch (const BackendError&) { threw = true; }
            EXPECT(threw, "limbs_total 0 must throw");
            for (auto* c : {&sr, &si, &ur, &ui}) free_ciphertext(*c);
            hipFree(ssk.data); hipFree(s1r); hipFree(s1i); hipFree(dsh);
        }
        for (auto* c : {&c1r, &c1i, &c2r, &c2i}) free_ciphertext(*c);
        hipFree(sk.data); hipFree(dm1); hipFree(dm2); hipFree(dout);
        hipFree(e1r); hipFree(e1i); hipFree(e2r); hipFree(e2i);
    }

    // ---- batched trace GEMM (batched_trace.cu:37-197): map B -> B', C = n A B'^T, rescale ----
    std::printf("[trace gemm]\n");
    {
        const int batch = 2;
        const size_t tw = (size_t)batch * L * n2;
        std::vector<uint64_t> hA[2], hB[2];
        for (int c = 0; c < 2; ++c) {
            hA[c].resize(tw);
            hB[c].resize(tw);
            for (size_t i = 0; i < tw; ++i) {
                const uint64_t q = RNS_MODULI[(i / n2) % L];
                hA[c][i] = splitmix(seed) % q;
                hB[c][i] = splitmix(seed) % q;
            }
        }
        uint64_t *ar = h2d(hA[0]), *ai = h2d(hA[1]), *br = h2d(hB[0]), *bi = h2d(hB[1]);
        uint64_t *bpr = dev_alloc<uint64_t>(tw), *bpi = dev_alloc<uint64_t>(tw);
        uint64_t *cr = dev_alloc<uint64_t>(tw), *ci = dev_alloc<uint64_t>(tw);
        map_B_to_Bprime_batched(br, bi, bpr, bpi, n, L, batch);
        trace_gemm_batched(ar, ai, bpr, bpi, cr, ci, n, L, batch);
        auto gr = d2h(cr, tw), gi = d2h(ci, tw);
        const uint64_t inv0 = 3, inv1 = 5, inv2 = 7;
        rescale_by_delta_batched(cr, ci, n, L, batch, inv0, inv1, inv2);
        auto sr = d2h(cr, tw), si = d2h(ci, tw);
        size_t bad = 0;
        for (size_t o = 0; o < tw; o += 131) {
            const size_t mat = o / n2, pos = o % n2, row = pos / n, col = pos % n, l = mat % L;
            const uint64_t q = RNS_MODULI[l];
            uint64_t accr = 0, acci = 0;
            for (int t = 0; t < n; ++t) {   // B'[col][t] from B: row j = (n - col) mod n, conj, times -i if j != 0
                const size_t j = (n - col) % n, src = mat * n2 + j * n + t;
                const uint64_t b_r = hB[0][src], b_i = hB[1][src];
                const uint64_t nbr = b_r ? q - b_r : 0, nbi = b_i ? q - b_i : 0;
                const uint64_t pr = j == 0 ? b_r : nbi, pi = j == 0 ? nbi : nbr;
                const uint64_t a_r = hA[0][mat * n2 + row * n + t], a_i = hA[1][mat * n2 + row * n + t];
                accr = (accr + mulmod(a_r, pr, q) + q - mulmod(a_i, pi, q)) % q;
                acci = (acci + mulmod(a_r, pi, q) + mulmod(a_i, pr, q)) % q;
            }
            accr = mulmod(accr, n % q, q);
            acci = mulmod(acci, n % q, q);
            bad += gr[o] != accr || gi[o] != acci;
            const uint64_t inv = l == 0 ? inv0 : l == 1 ? inv1 : l == 2 ? inv2 : 0;   // limbs >= 3: times 0
            bad += sr[o] != mulmod(accr, inv, q) || si[o] != mulmod(acci, inv, q);
        }
        EXPECT(bad == 0, "trace gemm / rescale mismatches %zu", bad);
        for (auto* p : {ar, ai, br, bi, bpr, bpi, cr, ci}) hipFree(p);
    }

    bool threw = false;
    try { wntt_forward_matrix(dx, dev, n, L, 256); } catch (const BackendError&) { threw = true; }
    EXPECT(threw, "phi != 512 must throw");
    hipFree(dx); hipFree(dev); hipFree(dback);
    std::printf(g_failures ? ">>> [FAIL] %d checks failed\n" : ">>> [PASS] core HE API\n", g_failures);
    return g_failures ? 1 : 0;
}
