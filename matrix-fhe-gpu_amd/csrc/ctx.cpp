// ctx.cpp -- mfhe_ctx creation: parameter validation and device table build.
//
// Table definitions (restating the reference's host-side setup):
//   phantom NTT  -- phantom::arith::NTT(log_n, q) (PhantomContext at HE.cu:327-336)
//   GL / cyclic  -- init_ntt_tables_manual + init_gl_twist_tables (ntt_core.cu:75-148, 175-198),
//                   re-expressed for our CT network: root psi' = beta^2, twists beta^-j / beta^-2j
//   GL perm      -- init_gl_perm_tables (ntt_core.cu:150-173)
//   wide CRT     -- Encoder::Encoder CRT tables (encoder.cu:341-421), generalised to W words
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <complex>
#include <mutex>
#include <thread>
#include <cstring>
#include <string>
#include <vector>

#include "host_math.hpp"
#include "gemm.hpp"
#include "mfhe_ctx.hpp"

namespace mfhe {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_error(hipError_t e, const char* what) {
    return set_error(MFHE_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
static int dalloc(mfhe_ctx* c, T** p, size_t n) {
    void* ptr = nullptr;
    hipError_t e = hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess) return hip_error(e, "hipMalloc");
    c->allocs.push_back(ptr);
    *p = (T*)ptr;
    return MFHE_OK;
}

template <class T>
static int upload(mfhe_ctx* c, T** p, const std::vector<T>& h) {
    int rc = dalloc(c, p, h.size());
    if (rc) return rc;
    MFHE_HIP(hipMemcpy(*p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return MFHE_OK;
}

static double centred(uint64_t w, uint64_t q) { return (w > q / 2) ? -(double)(q - w) : (double)w; }

// Phantom-format table for root `psi` (order 2N): tw[brev(i)] = psi^i; itw[brev(i)] = psi^-i, itw[1] *= n^-1.
static void build_ct_tables(uint64_t q, uint64_t psi, int logN, uint64_t* tw, uint64_t* itw, uint64_t* ninv) {
    const uint32_t n = 1u << logN;
    const uint64_t psi_inv = hm::invmod(psi, q);
    uint64_t p = 1, pi = 1;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r = hm::brev(i, logN);
        tw[r] = p;
        itw[r] = pi;
        p = hm::mulmod(p, psi, q);
        pi = hm::mulmod(pi, psi_inv, q);
    }
    *ninv = hm::invmod(n % q, q);
    if (n > 1) itw[1] = hm::mulmod(itw[1], *ninv, q);
}

struct HostTabs {
    std::vector<uint64_t> tw, tws, itw, itws, ninv, ninvs;
    std::vector<double> twf, itwf, ninvf;   // centred w (the FP64 quotient uses (v*w)/q)
};

static void add_limb_tables(HostTabs& h, uint64_t q, uint64_t psi, int logN, bool f64) {
    const size_t n = (size_t)1 << logN;
    std::vector<uint64_t> tw(n), itw(n);
    uint64_t ninv = 0;
    build_ct_tables(q, psi, logN, tw.data(), itw.data(), &ninv);
    for (size_t i = 0; i < n; ++i) {
        h.tw.push_back(tw[i]);
        h.tws.push_back(hm::shoup(tw[i], q));
        h.itw.push_back(itw[i]);
        h.itws.push_back(hm::shoup(itw[i], q));
        if (f64) {
            double a = centred(tw[i], q), b = centred(itw[i], q);
            h.twf.push_back(a);
            h.itwf.push_back(b);
        }
    }
    h.ninv.push_back(ninv);
    h.ninvs.push_back(hm::shoup(ninv, q));
    if (f64) {
        double a = centred(ninv, q);
        h.ninvf.push_back(a);
    }
}

static int upload_tabs(mfhe_ctx* c, HostTabs& h, NttTablesU& u, NttTablesF& f) {
    int rc;
    if ((rc = upload(c, &u.tw, h.tw)) || (rc = upload(c, &u.tws, h.tws)) || (rc = upload(c, &u.itw, h.itw)) ||
        (rc = upload(c, &u.itws, h.itws)) || (rc = upload(c, &u.ninv, h.ninv)) || (rc = upload(c, &u.ninvs, h.ninvs)))
        return rc;
    if (!h.twf.empty()) {
        if ((rc = upload(c, &f.tw, h.twf)) || (rc = upload(c, &f.itw, h.itwf)) || (rc = upload(c, &f.ninv, h.ninvf)))
            return rc;
    }
    return MFHE_OK;
}

// powers table: out[j] = r^j, u64 (+shoup) and centred F64
static void powers(uint64_t q, uint64_t r, size_t n, bool f64, std::vector<uint64_t>& w, std::vector<uint64_t>& ws,
                   std::vector<double>& wf) {
    uint64_t c = 1;
    for (size_t j = 0; j < n; ++j) {
        w.push_back(c);
        ws.push_back(hm::shoup(c, q));
        if (f64) {
            double a = centred(c, q);
            wf.push_back(a);
        }
        c = hm::mulmod(c, r, q);
    }
}

static int build_crt(mfhe_ctx* c, int min_words) {
    const int L = c->L;
    std::vector<uint64_t> Q(64, 0);
    Q[0] = 1;
    for (int i = 0; i < L; ++i) hm::big_mul_u64(Q.data(), c->moduli[i], Q.data(), 64);
    const int W = std::max(min_words, std::max(1, (hm::bitlen(Q) + 1 + 63) / 64));
    if (W > 32) return set_error(MFHE_EUNSUPPORTED, "wide CRT needs more than 32 words (product of moduli > 2^2047)");
    c->W = W;
    Q.resize(W);
    std::vector<uint64_t> Qh(W), M((size_t)L * W), inv((size_t)L * 2), mu((size_t)L * 2);
    std::vector<double> qinv(L);
    std::vector<uint64_t> r64(L);
    uint64_t carry = 0;
    for (int i = W - 1; i >= 0; --i) {
        Qh[i] = (Q[i] >> 1) | (carry << 63);
        carry = Q[i] & 1;
    }
    for (int k = 0; k < L; ++k) {
        const uint64_t q = c->moduli[k];
        hm::u128 rem = 0;
        for (int i = W - 1; i >= 0; --i) {
            hm::u128 cur = (rem << 64) | Q[i];
            M[(size_t)k * W + i] = (uint64_t)(cur / q);
            rem = cur % q;
        }
        hm::u128 r2 = 0;
        for (int i = W - 1; i >= 0; --i) r2 = ((r2 << 64) | M[(size_t)k * W + i]) % q;
        const uint64_t iv = hm::invmod((uint64_t)r2, q);
        inv[2 * k] = iv;
        inv[2 * k + 1] = hm::shoup(iv, q);
        qinv[k] = 1.0 / (double)q;
        mu[2 * k] = q;
        mu[2 * k + 1] = (uint64_t)((((hm::u128)1) << 64) / q);
        r64[k] = (uint64_t)((((hm::u128)1) << 64) % q);
    }
    int rc;
    c->crt_qbig = std::any_of(Qh.begin() + 1, Qh.end(), [](uint64_t w) { return w != 0; });
    // FP64 fast-path constants: every q < 2^50 (exact FP64 mulmod) and odd (divisibility test)
    c->d_crt_lf = nullptr;
    if (c->f64_ok && std::all_of(c->moduli.begin(), c->moduli.end(), [](uint64_t q) { return (q & 1) != 0; })) {
        std::vector<CrtLimbF> lf(L);
        for (int k = 0; k < L; ++k) {
            const uint64_t q = c->moduli[k];
            uint64_t qi = q;   // Newton: q^-1 mod 2^64 (q odd), 5 steps from 3 correct bits
            for (int it = 0; it < 5; ++it) qi *= 2 - q * qi;
            lf[k] = CrtLimbF{q, (double)q, (double)inv[2 * k], qinv[k], M[(size_t)k * W], qi, ~0ull / q, 0};
        }
        if ((rc = upload(c, &c->d_crt_lf, lf))) return rc;
    }
    if ((rc = upload(c, &c->d_crt_M, M)) || (rc = upload(c, &c->d_crt_inv, inv)) ||
        (rc = upload(c, &c->d_crt_qinv, qinv)) || (rc = upload(c, &c->d_crt_Q, Q)) ||
        (rc = upload(c, &c->d_crt_Qhalf, Qh)) || (rc = upload(c, &c->d_rns_mu, mu)) ||
        (rc = upload(c, &c->d_r64, r64)))
        return rc;
    return MFHE_OK;
}

// balanced base-256 digits every x in [0, q) needs: the smallest d with q - 1 <= 127 (256^d - 1) / 255
static int wcrt_digits(uint64_t q) {
    int d = 1;
    for (hm::u128 top = 127; d < 9 && (hm::u128)(q - 1) > top; ++d) top = top * 256 + 127;
    return d;
}

// W-axis tables: init_wntt_tables (HE.cu:237-273), init_wdft_tables (HE.cu:275-310),
// Encoder::init_complex_matrices (encoder.cu:425-444).
static int build_wcrt(mfhe_ctx* c) {
    const int PHI = mfhe_ctx::PHI, L = c->L;
    uint16_t exp[512];
    hm::wcrt_exponents(exp);
    std::vector<uint64_t> V((size_t)L * PHI * PHI), Vi((size_t)L * PHI * PHI);
    std::vector<int> bad(L, 0);
    std::vector<std::thread> th;
    for (int l = 0; l < L; ++l)
        th.emplace_back([&, l] {
            const uint64_t q = c->moduli[l];
            const uint64_t eta = hm::find_eta771(q);
            if (!eta) { bad[l] = 1; return; }
            std::vector<uint64_t> xs(PHI), inv;
            for (int w = 0; w < PHI; ++w) {
                const uint64_t root = hm::powmod(eta, exp[w], q);
                xs[w] = root;
                uint64_t cur = 1;
                for (int r = 0; r < PHI; ++r) {
                    V[((size_t)l * PHI + w) * PHI + r] = cur;
                    cur = hm::mulmod(cur, root, q);
                }
            }
            if (!hm::vandermonde_inverse_mod(xs, q, inv)) { bad[l] = 1; return; }
            std::copy(inv.begin(), inv.end(), Vi.begin() + (size_t)l * PHI * PHI);
        });
    for (auto& t : th) t.join();
    for (int l = 0; l < L; ++l)
        if (bad[l]) return set_error(MFHE_EUNSUPPORTED, "W-CRT table construction failed (no order-771 root)");
    // complex W-DFT: V[w][r] = root_w^r by repeated multiplication, as HE.cu:282-290.  Depends on nothing
    // but phi, so the (0.5 s) complex Gauss-Jordan inverse is computed once per process.
    static std::mutex wd_mu;
    static std::vector<double> wd_cache, wdi_cache;
    std::lock_guard<std::mutex> lk(wd_mu);
    if (wd_cache.empty()) {
        std::vector<double> wd((size_t)PHI * PHI * 2), wdi;
        const double p = 771.0, two_pi = 6.283185307179586476925286766559;
        for (int w = 0; w < PHI; ++w) {
            const double ang = two_pi * (double)exp[w] / p;
            const std::complex<double> root(std::cos(ang), std::sin(ang));
            std::complex<double> cur(1.0, 0.0);
            for (int r = 0; r < PHI; ++r) {
                wd[((size_t)w * PHI + r) * 2] = cur.real();
                wd[((size_t)w * PHI + r) * 2 + 1] = cur.imag();
                cur *= root;
            }
        }
        std::vector<double> a = wd;
        if (!hm::complex_inverse_gj(a, PHI, wdi)) return set_error(MFHE_EUNSUPPORTED, "W-DFT matrix singular");
        wd_cache.swap(wd);
        wdi_cache.swap(wdi);
    }
    const std::vector<double>& wd = wd_cache;
    const std::vector<double>& wdi = wdi_cache;
    std::vector<double2> wdv((size_t)PHI * PHI), wdvi((size_t)PHI * PHI);
    std::memcpy(wdv.data(), wd.data(), wd.size() * 8);
    std::memcpy(wdvi.data(), wdi.data(), wdi.size() * 8);
    int rc;
    if ((rc = upload(c, &c->d_wV, V)) || (rc = upload(c, &c->d_wVinv, Vi)) || (rc = upload(c, &c->d_wdV, wdv)) ||
        (rc = upload(c, &c->d_wdVinv, wdvi)))
        return rc;
    {
        // factored W-DFT tables (the complex counterpart of the factored W-CRT below; tools/wcrt_factor_check.py):
        // entries from exact integer exponents, so each is cos / sin of one angle (no repeated-product drift)
        auto cis = [](long num, long den) {
            const double two_pi = 6.283185307179586476925286766559;
            const long e = ((num % den) + den) % den;
            return make_double2(std::cos(two_pi * (double)e / (double)den), std::sin(two_pi * (double)e / (double)den));
        };
        std::vector<double2> zc(256 * 256), zic(256 * 256), lam(12), xp(512);
        for (int i = 0; i < 256; ++i)
            for (int k = 0; k < 256; ++k) {
                const long e = ((long)(i + 1) * (k + 1)) % 257;
                zc[(size_t)i * 256 + k] = cis(e, 257);
                zic[(size_t)i * 256 + k] = cis(-e, 257);
            }
        double2 kap[2][3];
        for (int ap = 0; ap < 2; ++ap)
            for (int t = 0; t < 3; ++t) {
                const double2 w = cis(-(long)((ap + 1) * t), 3);
                kap[ap][t] = make_double2(w.x / 771.0, w.y / 771.0);
            }
        auto sub = [](double2 x, double2 y) { return make_double2(x.x - y.x, x.y - y.y); };
        for (int ap = 0; ap < 2; ++ap)
            for (int t = 0; t < 3; ++t) {
                lam[(0 * 2 + ap) * 3 + t] = sub(kap[ap][t], kap[ap][(t + 1) % 3]);
                lam[(1 * 2 + ap) * 3 + t] = sub(kap[ap][(t + 2) % 3], kap[ap][(t + 1) % 3]);
            }
        for (int s = 0; s < 2; ++s)
            for (int k = 0; k < 256; ++k) xp[(size_t)s * 256 + k] = cis(-(long)(255 + s) * (k + 1), 257);
        std::vector<int> num(515, 0), ph(513, 0);   // Phi_771 = (x^514 + x^257 + 1) / (x^2 + x + 1)
        num[0] = num[257] = num[514] = 1;
        for (int d = 514; d >= 2; --d)
            if (num[d]) {
                const int cf = num[d];
                ph[d - 2] = cf;
                num[d] -= cf;
                num[d - 1] -= cf;
                num[d - 2] -= cf;
            }
        std::vector<int8_t> phi(ph.begin(), ph.end());
        // Rader (r06): for b, j != 0 write j = g^n, b = g^-m (g = 3, a primitive root of 257); then
        // sum_j zeta^(bj) F[j] = (a * bk)[m], the cyclic convolution of a[n] = F[g^n] and bk[k] = zeta^(g^-k), taken
        // as IFFT_256(FFT_256(a) FFT_256(bk)): the kernel gets FFT_256(bk) / 256 (long double sums)
        std::vector<int16_t> gp(512);
        {
            long x = 1;
            for (int n = 0; n < 256; ++n) {
                gp[n] = (int16_t)x;
                x = x * 3 % 257;
            }
            long inv3 = 1;
            for (int e = 0; e < 255; ++e) inv3 = inv3 * 3 % 257;   // 3^255 = 3^-1 mod 257
            long y = 1;
            for (int m = 0; m < 256; ++m) {
                gp[256 + m] = (int16_t)y;
                y = y * inv3 % 257;
            }
        }
        std::vector<double2> rad(512);   // [0]: bk = zeta^(g^-k) (forward); [1]: its conjugate (inverse, zeta^-1)
        {
            const long double tp = 6.283185307179586476925286766559L;
            std::vector<long double> br(256), bi(256), cr(256), ci(256);
            for (int k = 0; k < 256; ++k) {
                br[k] = cosl(tp * (long double)gp[256 + k] / 257.0L);
                bi[k] = sinl(tp * (long double)gp[256 + k] / 257.0L);
                cr[k] = cosl(-tp * (long double)k / 256.0L);
                ci[k] = sinl(-tp * (long double)k / 256.0L);
            }
            for (int dir = 0; dir < 2; ++dir)
                for (int k = 0; k < 256; ++k) {
                    long double sr = 0, si = 0;
                    for (int n = 0; n < 256; ++n) {
                        const int e = (n * k) % 256;
                        const long double xr = br[n], xi = dir ? -bi[n] : bi[n];
                        sr += xr * cr[e] - xi * ci[e];
                        si += xr * ci[e] + xi * cr[e];
                    }
                    rad[(size_t)dir * 256 + k] = make_double2((double)(sr / 256.0L), (double)(si / 256.0L));
                }
        }
        if ((rc = upload(c, &c->d_wdZ, zc)) || (rc = upload(c, &c->d_wdZi, zic)) || (rc = upload(c, &c->d_wdlam, lam)) ||
            (rc = upload(c, &c->d_wdxp, xp)) || (rc = upload(c, &c->d_wdphi, phi)) || (rc = upload(c, &c->d_wdrad, rad)) ||
            (rc = upload(c, &c->d_wdgp, gp)))
            return rc;
    }
    // i8 MFMA operand planes (gemm.hip): D balanced base-256 digits of every V / V^-1 entry, and
    // 256^s mod q for the epilogue.  Needs 2^27 < q (|acc_s| < q) and q < 2^59 (D <= 8).
    bool big = true;
    for (uint64_t q : c->moduli) big = big && q > (1ull << 27);
    int D = 5;
    for (uint64_t q : c->moduli) D = std::max(D, wcrt_digits(q));
    if (big && D <= 8) {
        const size_t plane = (size_t)PHI * PHI;
        std::vector<int8_t> vd((size_t)L * D * plane), vid((size_t)L * D * plane);
        std::vector<uint64_t> rt((size_t)L * (2 * D - 1) * 2);
        for (int l = 0; l < L; ++l) {
            int8_t d[8];
            for (size_t e = 0; e < plane; ++e) {
                // plane layout [k/32][row][k%32] (gemm.hip "k-panel-major"): row = w, k = r of V[w][r]
                const size_t w = e / PHI, r = e % PHI, o = ((r >> 5) * PHI + w) * 32 + (r & 31);
                balanced_digits(V[(size_t)l * plane + e], D, d);
                for (int i = 0; i < D; ++i) vd[((size_t)l * D + i) * plane + o] = d[i];
                balanced_digits(Vi[(size_t)l * plane + e], D, d);
                for (int i = 0; i < D; ++i) vid[((size_t)l * D + i) * plane + o] = d[i];
            }
            const uint64_t q = c->moduli[l];
            uint64_t p256 = 1;
            for (int s = 0; s < 2 * D - 1; ++s) {
                rt[((size_t)l * (2 * D - 1) + s) * 2] = p256;
                rt[((size_t)l * (2 * D - 1) + s) * 2 + 1] = hm::shoup(p256, q);
                p256 = hm::mulmod(p256, 256 % q, q);
            }
        }
        if ((rc = upload(c, &c->d_wVdig, vd)) || (rc = upload(c, &c->d_wVidig, vid)) || (rc = upload(c, &c->d_wrtab, rt)))
            return rc;
        c->wD = D;
        // per-limb digit count: every value in [0, q) has zero balanced digits from d_l on, so limb l's
        // products with those planes vanish and its GEMM runs at d_l^2 instead of D^2 MFMAs
        c->wDl.resize(L);
        for (int l = 0; l < L; ++l) {
            c->wDl[l] = std::min(D, wcrt_digits(c->moduli[l]));
        }
        // FP64 epilogue constants (every q < 2^50): q, 1/q and centred 2^32, 2^64, 2^96 mod q
        if (c->f64_ok) {
            std::vector<double> ep((size_t)L * 8, 0.0);
            for (int l = 0; l < L; ++l) {
                const uint64_t q = c->moduli[l];
                const uint64_t p32 = (uint64_t)((((hm::u128)1) << 32) % q);
                const uint64_t p64 = hm::mulmod(p32, p32, q), p96 = hm::mulmod(p64, p32, q);
                ep[(size_t)l * 8 + 0] = (double)q;
                ep[(size_t)l * 8 + 1] = 1.0 / (double)q;
                ep[(size_t)l * 8 + 2] = centred(p32, q);
                ep[(size_t)l * 8 + 3] = centred(p64, q);
                ep[(size_t)l * 8 + 4] = centred(p96, q);
            }
            if ((rc = upload(c, &c->d_wepi, ep))) return rc;
            // factored forward (gemm.hip, 771 = 3 x 257): zeta = eta^3 of order 257, omega = eta^257 of order 3
            if (D <= 6) {
                constexpr int FK = 256;
                std::vector<int8_t> zd((size_t)L * D * FK * FK);
                std::vector<double> fo((size_t)L * 16, 0.0);
                for (int l = 0; l < L; ++l) {
                    const uint64_t q = c->moduli[l], eta = hm::find_eta771(q);
                    const uint64_t zeta = hm::powmod(eta, 3, q), omega = hm::powmod(eta, 257, q);
                    int8_t d[8];
                    for (int i = 0; i < FK; ++i) {
                        const uint64_t zi = hm::powmod(zeta, (uint64_t)i + 1, q);
                        uint64_t cur = zi;
                        for (int k = 0; k < FK; ++k, cur = hm::mulmod(cur, zi, q)) {
                            balanced_digits(cur, D, d);
                            const size_t o = ((size_t)(k >> 5) * FK + i) * 32 + (k & 31);
                            for (int j = 0; j < D; ++j) zd[((size_t)l * D + j) * FK * FK + o] = d[j];
                        }
                    }
                    fo[(size_t)l * 16 + 0] = (double)q;
                    fo[(size_t)l * 16 + 1] = 1.0 / (double)q;
                    for (int ap = 0; ap < 2; ++ap)
                        for (int r1 = 0; r1 < 3; ++r1) {
                            fo[(size_t)l * 16 + 2 + 3 * ap + r1] = centred(hm::powmod(omega, (uint64_t)(ap + 1) * r1, q), q);
                            fo[(size_t)l * 16 + 8 + 3 * ap + r1] =
                                centred(hm::powmod(omega, (uint64_t)(ap + 1) * ((r1 + 2) % 3), q), q);
                        }
                }
                if ((rc = upload(c, &c->d_wZdig, zd)) || (rc = upload(c, &c->d_wfold, fo))) return rc;
                // factored inverse (gemm.hip mfma_digitize_ifold_kernel / epilogue): the 771-point interpolation
                // with zeros at the non-units, reduced mod Phi_771 (tools/wcrt_factor_check.py).  Zi[i][k] =
                // zeta^-((i+1)(k+1)); kappa[a][t] = 771^-1 omega^(-a t); lam1[a][t] = kappa[a][t] - kappa[a][t+1],
                // lam2[a][t] = kappa[a][t+2] - kappa[a][t+1] (t mod 3); z[l][0 / 1][k] = zeta^(-255 / -256 (k+1)).
                std::vector<int8_t> zid((size_t)L * D * FK * FK);
                std::vector<double> ifo((size_t)L * 16, 0.0), iz((size_t)L * 48, 0.0);
                for (int l = 0; l < L; ++l) {
                    const uint64_t q = c->moduli[l], eta = hm::find_eta771(q);
                    const uint64_t zinv = hm::powmod(hm::powmod(eta, 3, q), 256, q), omega = hm::powmod(eta, 257, q);
                    const uint64_t inv771 = hm::powmod(771 % q, q - 2, q);
                    int8_t d[8];
                    for (int i = 0; i < FK; ++i) {
                        const uint64_t zi = hm::powmod(zinv, (uint64_t)i + 1, q);
                        uint64_t cur = zi;
                        for (int k = 0; k < FK; ++k, cur = hm::mulmod(cur, zi, q)) {
                            balanced_digits(cur, D, d);
                            const size_t o = ((size_t)(k >> 5) * FK + i) * 32 + (k & 31);
                            for (int j = 0; j < D; ++j) zid[((size_t)l * D + j) * FK * FK + o] = d[j];
                        }
                    }
                    uint64_t kap[2][3];
                    for (int ap = 0; ap < 2; ++ap)
                        for (int t = 0; t < 3; ++t)
                            kap[ap][t] = hm::mulmod(inv771, hm::powmod(omega, (uint64_t)((3 - ((ap + 1) * t) % 3) % 3), q), q);
                    auto sub = [q](uint64_t x, uint64_t y) { return x >= y ? x - y : x + q - y; };
                    ifo[(size_t)l * 16 + 0] = (double)q;
                    ifo[(size_t)l * 16 + 1] = 1.0 / (double)q;
                    for (int ap = 0; ap < 2; ++ap)
                        for (int t = 0; t < 3; ++t) {
                            ifo[(size_t)l * 16 + 2 + 3 * ap + t] = centred(sub(kap[ap][t], kap[ap][(t + 1) % 3]), q);
                            ifo[(size_t)l * 16 + 8 + 3 * ap + t] = centred(sub(kap[ap][(t + 2) % 3], kap[ap][(t + 1) % 3]), q);
                        }
                    for (int s = 0; s < 2; ++s) {   // x_s = zeta^-(255 + s): x_s, then x_s^(16 j + 1), j < 16
                        const uint64_t xs = hm::powmod(zinv, 255 + (uint64_t)s, q);
                        iz[(size_t)l * 48 + s] = centred(xs, q);
                        for (int j = 0; j < 16; ++j)
                            iz[(size_t)l * 48 + 16 + 16 * s + j] = centred(hm::powmod(xs, 16 * (uint64_t)j + 1, q), q);
                    }
                }
                // Phi_771 = (x^514 + x^257 + 1) / (x^2 + x + 1), coefficients in {-1, 0, 1}; phi[j + 1] = coefficient j
                std::vector<int> num(515, 0), ph(513, 0);
                num[0] = num[257] = num[514] = 1;
                for (int d = 514; d >= 2; --d)
                    if (num[d]) {
                        const int cf = num[d];
                        ph[d - 2] = cf;
                        num[d] -= cf;
                        num[d - 1] -= cf;
                        num[d - 2] -= cf;
                    }
                auto pc = [&](int j) { return (uint8_t)((j < 0 ? 0 : ph[j]) + 1); };
                std::vector<uint8_t> phi(320, 0);
                for (int r2 = 0; r2 <= 256; ++r2)
                    phi[r2 ? r2 - 1 : 256] = (uint8_t)(pc(r2) | pc(r2 - 1) << 2 | pc(r2 + 257) << 4 | pc(r2 + 256) << 6);
                if ((rc = upload(c, &c->d_wZidig, zid)) || (rc = upload(c, &c->d_wifold, ifo)) ||
                    (rc = upload(c, &c->d_wiz, iz)) || (rc = upload(c, &c->d_wphi, phi)))
                    return rc;
            }
        }
    }
    return MFHE_OK;
}

// XY encoder matrices: Encoder::init_complex_matrices (encoder.cu:425-444); n x n complex, built on first
// use (they only make sense for the matrix dimension n = N of the X/Y axes, so N is capped at 2^10).
int ensure_xy(mfhe_ctx* c) {
    if (c->d_encV) return MFHE_OK;
    if (c->N > 1024) return set_error(MFHE_EUNSUPPORTED, "XY encoder matrices need n <= 1024");
    const int n = (int)c->N;
    std::vector<double2> eV((size_t)n * n), eVT((size_t)n * n), eVi((size_t)n * n), eViT((size_t)n * n);
    {
        const double PI = 3.141592653589793;
        auto cmul = [](double2 a, double2 b) { return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); };
        for (int j = 0; j < n; ++j) {
            uint64_t e = 1, b5 = 5;
            int p = j;
            while (p > 0) { if (p & 1) e = (e * b5) % (uint64_t)(4 * n); b5 = (b5 * b5) % (uint64_t)(4 * n); p >>= 1; }
            const double ang = 2.0 * PI * (double)e / (4.0 * n);
            const double2 z = make_double2(std::cos(ang), std::sin(ang)), zi = make_double2(z.x, -z.y);
            const double2 sc = make_double2(1.0 / n, 0.0);
            double2 cc = make_double2(1, 0), ci = make_double2(1, 0);
            for (int k = 0; k < n; ++k) {
                eV[(size_t)j * n + k] = cc;
                eVi[(size_t)k * n + j] = cmul(ci, sc);
                cc = cmul(cc, z);
                ci = cmul(ci, zi);
            }
        }
        for (int r = 0; r < n; ++r)
            for (int cc2 = 0; cc2 < n; ++cc2) {
                eVT[(size_t)cc2 * n + r] = eV[(size_t)r * n + cc2];
                eViT[(size_t)cc2 * n + r] = eVi[(size_t)r * n + cc2];
            }
    }
    int rc;
    if ((rc = upload(c, &c->d_encV, eV)) || (rc = upload(c, &c->d_encVT, eVT)) || (rc = upload(c, &c->d_encVi, eVi)) ||
        (rc = upload(c, &c->d_encViT, eViT)))
        return rc;
    return MFHE_OK;
}

static int ctx_create_impl(const uint64_t* moduli, int L, int logN, int conv, double delta, mfhe_ctx** out) {
    if (!out) return set_error(MFHE_EINVAL, "mfhe_ctx_create: out is null");
    *out = nullptr;
    if (!moduli || L < 1 || L > 256) return set_error(MFHE_EINVAL, "mfhe_ctx_create: need 1 <= L <= 256 moduli");
    if (logN < 1 || logN > 17) return set_error(MFHE_EINVAL, "mfhe_ctx_create: log_n must be in [1, 17]");
    if (!(delta > 0.0) || !std::isfinite(delta)) return set_error(MFHE_EINVAL, "mfhe_ctx_create: delta must be > 0");
    const uint64_t N = 1ull << logN;
    for (int i = 0; i < L; ++i) {
        const uint64_t q = moduli[i];
        if (q < 3 || q >= (1ull << 62) || !hm::is_prime(q))
            return set_error(MFHE_EINVAL, "mfhe_ctx_create: modulus " + std::to_string(q) + " is not a prime < 2^62");
        for (int j = 0; j < i; ++j)
            if (moduli[j] == q) return set_error(MFHE_EINVAL, "mfhe_ctx_create: moduli must be distinct");
        if ((conv & MFHE_CONV_PHANTOM) && (q - 1) % (2 * N) != 0)
            return set_error(MFHE_EUNSUPPORTED, "modulus " + std::to_string(q) + " has no primitive 2N-th root");
        if ((conv & MFHE_CONV_GL) && (q - 1) % (4 * N) != 0)
            return set_error(MFHE_EUNSUPPORTED, "modulus " + std::to_string(q) + " has no primitive 4N-th root (GL)");
        if ((conv & MFHE_CONV_WCRT) && (q - 1) % 771 != 0)
            return set_error(MFHE_EUNSUPPORTED, "modulus " + std::to_string(q) + " has no 771-th root (W-CRT)");
        if ((conv & MFHE_CONV_WCRT) && q >= (1ull << 59))
            return set_error(MFHE_EUNSUPPORTED, "W-CRT needs moduli < 2^59 (512-term u128 accumulation)");
    }
    mfhe_ctx* c = new mfhe_ctx();
    c->L = L;
    c->logN = logN;
    c->N = N;
    c->conv = conv;
    c->delta = delta;
    c->moduli.assign(moduli, moduli + L);
    c->f64_ok = std::all_of(c->moduli.begin(), c->moduli.end(), [](uint64_t q) { return q < (1ull << 50); });
    c->arith = c->f64_ok ? MFHE_ARITH_F64 : MFHE_ARITH_U64;
    c->u60_ok = std::all_of(c->moduli.begin(), c->moduli.end(), [](uint64_t q) { return q < (1ull << 60); });
    hipError_t he = hipGetDevice(&c->device);
    int rc = MFHE_OK;
    if (he != hipSuccess) rc = hip_error(he, "hipGetDevice");
    if (!rc && (he = hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, c->device)) != hipSuccess)
        rc = hip_error(he, "hipDeviceGetAttribute");

    auto fail = [&](int code) {
        for (void* p : c->allocs) (void)hipFree(p);
        delete c;
        return code;
    };
    if (rc) return fail(rc);

    // per-limb constants
    std::vector<LimbConst> lcs(L);
    std::vector<uint64_t> dmod((size_t)L * 3);
    for (int i = 0; i < L; ++i) {
        const uint64_t q = moduli[i];
        lcs[i].q = q;
        lcs[i].qf = (double)q;
        lcs[i].qinv = 1.0 / (double)q;
        lcs[i].pad = 0;
        const hm::u128 two64 = ((hm::u128)1) << 64;
        dmod[3 * i] = q;
        dmod[3 * i + 2] = (uint64_t)(two64 / q);                          // high word of floor(2^128/q)
        dmod[3 * i + 1] = (uint64_t)(((two64 % q) << 64) / q);           // low word
    }
    if ((rc = upload(c, &c->d_limbs, lcs)) || (rc = upload(c, &c->d_dmod, dmod))) return fail(rc);

    if (conv & MFHE_CONV_PHANTOM) {
        HostTabs h;
        for (int i = 0; i < L; ++i) {
            const uint64_t psi = hm::minimal_primitive_root(2 * N, moduli[i]);
            if (!psi) return fail(set_error(MFHE_EUNSUPPORTED, "no primitive 2N-th root"));
            add_limb_tables(h, moduli[i], psi, logN, c->f64_ok);
        }
        if ((rc = upload_tabs(c, h, c->ph_u, c->ph_f))) return fail(rc);
    }
    if (conv & MFHE_CONV_GL) {
        HostTabs h;
        std::vector<uint64_t> gpre, gpres, gpost, gposts, cpre, cpres, cpost, cposts;
        std::vector<double> gpref, gpostf, cpref, cpostf;
        for (int i = 0; i < L; ++i) {
            const uint64_t q = moduli[i];
            const uint64_t beta = hm::first_psi4n(q, N);
            if (!beta) return fail(set_error(MFHE_EUNSUPPORTED, "no psi4n (GL)"));
            const uint64_t psi2 = hm::mulmod(beta, beta, q);   // primitive 2N-th root of the network
            add_limb_tables(h, q, psi2, logN, c->f64_ok);
            const uint64_t bi = hm::invmod(beta, q);
            powers(q, bi, N, c->f64_ok, gpre, gpres, gpref);                     // beta^-j
            powers(q, beta, N, c->f64_ok, gpost, gposts, gpostf);                // beta^j
            powers(q, hm::mulmod(bi, bi, q), N, c->f64_ok, cpre, cpres, cpref);  // beta^-2j
            powers(q, psi2, N, c->f64_ok, cpost, cposts, cpostf);                // beta^2j
        }
        if ((rc = upload_tabs(c, h, c->gl_u, c->gl_f))) return fail(rc);
        if ((rc = upload(c, &c->gl_pre_u, gpre)) || (rc = upload(c, &c->gl_pre_us, gpres)) ||
            (rc = upload(c, &c->gl_post_u, gpost)) || (rc = upload(c, &c->gl_post_us, gposts)) ||
            (rc = upload(c, &c->cyc_pre_u, cpre)) || (rc = upload(c, &c->cyc_pre_us, cpres)) ||
            (rc = upload(c, &c->cyc_post_u, cpost)) || (rc = upload(c, &c->cyc_post_us, cposts)))
            return fail(rc);
        if (c->f64_ok) {
            if ((rc = upload(c, &c->gl_pre_f, gpref)) || (rc = upload(c, &c->gl_post_f, gpostf)) ||
                (rc = upload(c, &c->cyc_pre_f, cpref)) || (rc = upload(c, &c->cyc_post_f, cpostf)))
                return fail(rc);
        }
        // init_gl_perm_tables (ntt_core.cu:150-173)
        std::vector<uint32_t> perm(N), iperm(N);
        const uint32_t m = 4u * (uint32_t)N;
        uint32_t e = 1 % m;
        for (uint32_t j = 0; j < N; ++j) {
            const uint32_t tgt = hm::brev((e - 1) / 4, logN);
            perm[j] = tgt;
            iperm[tgt] = j;
            e = (uint32_t)((uint64_t)e * 5u % m);
        }
        if ((rc = upload(c, &c->gl_perm, perm)) || (rc = upload(c, &c->gl_inv_perm, iperm))) return fail(rc);
    }
    if ((rc = build_crt(c, 1))) return fail(rc);
    if ((conv & MFHE_CONV_WCRT) && (rc = build_wcrt(c))) return fail(rc);
    *out = c;
    return MFHE_OK;
}

}  // namespace mfhe

using namespace mfhe;

extern "C" int mfhe_ctx_create(const uint64_t* moduli, int L, int log_n, int conventions, double delta,
                               mfhe_ctx** out) {
    try {
        return ctx_create_impl(moduli, L, log_n, conventions, delta, out);
    } catch (const std::exception& e) {
        return set_error(MFHE_ENOMEM, std::string("mfhe_ctx_create: ") + e.what());
    }
}

extern "C" int mfhe_ctx_destroy(mfhe_ctx* c) {
    if (!c) return MFHE_OK;
    if (c->ws) (void)hipFree(c->ws);
    if (c->gemm_ws) (void)hipFree(c->gemm_ws);
    if (c->gemm_ws2) (void)hipFree(c->gemm_ws2);
    if (c->he_side) (void)hipStreamDestroy(c->he_side);
    if (c->he_fork) (void)hipEventDestroy(c->he_fork);
    if (c->he_join) (void)hipEventDestroy(c->he_join);
    if (c->wd_ws) (void)hipFree(c->wd_ws);
    for (void* p : c->allocs) (void)hipFree(p);
    delete c;
    return MFHE_OK;
}

extern "C" int mfhe_ctx_get_info(const mfhe_ctx* c, mfhe_ctx_info* info) {
    if (!c || !info) return set_error(MFHE_EINVAL, "mfhe_ctx_get_info: null argument");
    info->num_limbs = c->L;
    info->log_n = c->logN;
    info->crt_words = c->W;
    info->arith = c->arith;
    info->conventions = c->conv;
    info->phi = (c->conv & MFHE_CONV_WCRT) ? 512 : 0;
    info->delta = c->delta;
    return MFHE_OK;
}

extern "C" int mfhe_ctx_set_arith(mfhe_ctx* c, int arith) {
    if (!c) return set_error(MFHE_EINVAL, "mfhe_ctx_set_arith: null ctx");
    if (arith == MFHE_ARITH_AUTO) arith = c->f64_ok ? MFHE_ARITH_F64 : MFHE_ARITH_U64;
    if (arith == MFHE_ARITH_F64 && !c->f64_ok)
        return set_error(MFHE_EUNSUPPORTED, "F64 arithmetic needs every modulus < 2^50");
    if (arith != MFHE_ARITH_F64 && arith != MFHE_ARITH_U64) return set_error(MFHE_EINVAL, "bad arith");
    c->arith = arith;
    return MFHE_OK;
}

extern "C" int mfhe_ctx_set_limb_shard(mfhe_ctx* c, int limb_base, int limbs_total) {
    if (!c) return set_error(MFHE_EINVAL, "mfhe_ctx_set_limb_shard: null ctx");
    if (limbs_total == 0) limbs_total = c->L;
    if (limb_base < 0 || limbs_total < c->L || limb_base + c->L > limbs_total)
        return set_error(MFHE_EINVAL, "mfhe_ctx_set_limb_shard: [limb_base, limb_base + L) must lie in [0, limbs_total)");
    c->limb_base = limb_base;
    c->limbs_total = limbs_total;
    return MFHE_OK;
}

extern "C" int mfhe_ctx_set_option(mfhe_ctx* c, int opt, int64_t v) {
    if (!c) return set_error(MFHE_EINVAL, "mfhe_ctx_set_option: null ctx");
    switch (opt) {
        case MFHE_OPT_NTT_CHUNK_BYTES:
            if (v < 0) return set_error(MFHE_EINVAL, "chunk bytes must be >= 0");
            c->ntt_chunk_bytes = v;
            return MFHE_OK;
        case MFHE_OPT_NTT_PLAN:
            // 5 (the one-launch N = 2^16 forward with an in-L2 hand-off, r05) was removed in r06: latency-bound at the one
            // wave per SIMD its LDS allows and slower than the two passes (profiles/r06_xl2_sq_pmc.txt)
            if (v < 0 || v > 3) return set_error(MFHE_EINVAL, "plan must be 0, 1, 2 or 3");
            c->ntt_plan = (int)v;
            return MFHE_OK;
        case MFHE_OPT_NTT_WG_PER_CU:
            if (v < 0 || v > 16) return set_error(MFHE_EINVAL, "workgroups per CU must be in [0, 16]");
            c->ntt_wg_per_cu = (int)v;
            return MFHE_OK;
        case MFHE_OPT_NTT_PREFETCH:
            if (v < 0 || v > 2) return set_error(MFHE_EINVAL, "prefetch must be 0, 1 or 2");
            c->ntt_prefetch = (int)v;
            return MFHE_OK;
        case MFHE_OPT_NTT_PACK:
            if (v < 0 || v > 1) return set_error(MFHE_EINVAL, "pack must be 0 or 1");
            c->ntt_pack = (int)v;
            return MFHE_OK;
        case MFHE_OPT_NTT_FUSED:
            // the one-launch L2 hand-off NTT was removed in r04 (slower than the two-pass plan, and its hand-off
            // was never proven): 0 is accepted, anything else is not
            if (v != 0) return set_error(MFHE_EUNSUPPORTED, "the fused NTT was removed (DESIGN.md §3.1); only 0 is accepted");
            return MFHE_OK;
        case MFHE_OPT_WCRT_MFMA:
            if (v < 0 || v > 3) return set_error(MFHE_EINVAL, "wcrt mfma must be 0, 1, 2 or 3");
            c->wcrt_mfma = (int)v;
            return MFHE_OK;
        case MFHE_OPT_WCRT_PIPE:
            if (v < 0 || v > 3) return set_error(MFHE_EINVAL, "wcrt pipe must be 0, 1, 2 or 3");
            c->wcrt_pipe = (int)v;
            return MFHE_OK;
        case MFHE_OPT_CGEMM_MFMA:
            if (v < 0 || v > 3) return set_error(MFHE_EINVAL, "cgemm mfma must be 0 .. 3");
            c->cgemm_mfma = (int)v;
            return MFHE_OK;
        case MFHE_OPT_HE_FUSED:
            if (v < 0 || v > 1) return set_error(MFHE_EINVAL, "he fused must be 0 or 1");
            c->he_fused = (int)v;
            return MFHE_OK;
        case MFHE_OPT_TRACE_SPLIT:
            if (v < 0 || v > 2) return set_error(MFHE_EINVAL, "trace split must be 0, 1 or 2");
            c->trace_split = (int)v;
            return MFHE_OK;
        case MFHE_OPT_ENC_E_SMALL:
            if (v < 0 || v > 1) return set_error(MFHE_EINVAL, "enc e small must be 0 or 1");
            c->enc_e_small = (int)v;
            return MFHE_OK;
        case MFHE_OPT_ENC_A_DIRECT:
            if (v < 0 || v > 1) return set_error(MFHE_EINVAL, "enc a direct must be 0 or 1");
            c->enc_a_direct = (int)v;
            return MFHE_OK;
        case MFHE_OPT_DEC_MM:   // the decrypt's ring product on the matrix cores (r05): measured 2.4x slower, removed in r06
            if (v != 0) return set_error(MFHE_EINVAL, "MFHE_OPT_DEC_MM was removed in r06: only 0 is accepted");
            return MFHE_OK;
        case MFHE_OPT_HE_STREAMS:
            if (v < 0 || v > 3) return set_error(MFHE_EINVAL, "he streams must be 0, 1, 2 or 3");
            c->he_streams = (int)v;
            return MFHE_OK;
        case MFHE_OPT_NTT_U60:
            if (v < 0 || v > 1) return set_error(MFHE_EINVAL, "ntt u60 must be 0 or 1");
            c->ntt_u60 = (int)v;
            return MFHE_OK;
        case MFHE_OPT_CRT_WORDS:
            if (v < 1 || v > 32) return set_error(MFHE_EINVAL, "crt words must be in [1, 32]");
            if (v <= c->W) return MFHE_OK;
            return build_crt(c, (int)v);   // old tables stay in c->allocs until destroy
        default: return set_error(MFHE_EINVAL, "unknown option");
    }
}

extern "C" int mfhe_gl_perm_tables(const mfhe_ctx* c, const uint32_t** perm, const uint32_t** iperm) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (!(c->conv & MFHE_CONV_GL)) return set_error(MFHE_ENOTREADY, "no GL tables");
    if (perm) *perm = c->gl_perm;
    if (iperm) *iperm = c->gl_inv_perm;
    return MFHE_OK;
}

extern "C" int mfhe_xy_tables(const mfhe_ctx* c, const double** V, const double** VT, const double** Vi,
                              const double** ViT) {
    if (!c) return set_error(MFHE_EINVAL, "null ctx");
    if (int rc = ensure_xy(const_cast<mfhe_ctx*>(c))) return rc;   // lazily built tables, logically const
    if (V) *V = (const double*)c->d_encV;
    if (VT) *VT = (const double*)c->d_encVT;
    if (Vi) *Vi = (const double*)c->d_encVi;
    if (ViT) *ViT = (const double*)c->d_encViT;
    return MFHE_OK;
}

extern "C" int mfhe_ctx_get_option(const mfhe_ctx* c, int opt, int64_t* v) {
    if (!c || !v) return set_error(MFHE_EINVAL, "mfhe_ctx_get_option: null argument");
    switch (opt) {
        case MFHE_OPT_NTT_CHUNK_BYTES: *v = c->ntt_chunk_bytes; return MFHE_OK;
        case MFHE_OPT_NTT_PLAN: *v = c->ntt_plan; return MFHE_OK;
        case MFHE_OPT_NTT_PLAN_EFFECTIVE:
            *v = mfhe::ntt_phantom_plan(c->arith == MFHE_ARITH_F64, c->logN, c->ntt_plan, true);
            return MFHE_OK;
        case MFHE_OPT_NTT_WG_PER_CU: *v = c->ntt_wg_per_cu; return MFHE_OK;
        case MFHE_OPT_NTT_PREFETCH: *v = c->ntt_prefetch; return MFHE_OK;
        case MFHE_OPT_NTT_FUSED: *v = 0; return MFHE_OK;
        case MFHE_OPT_NTT_PACK: *v = c->ntt_pack; return MFHE_OK;
        case MFHE_OPT_WCRT_PIPE: *v = c->wcrt_pipe; return MFHE_OK;
        case MFHE_OPT_WCRT_MFMA: *v = c->d_wVdig ? c->wcrt_mfma : 0; return MFHE_OK;
        case MFHE_OPT_CGEMM_MFMA: *v = c->cgemm_mfma; return MFHE_OK;
        case MFHE_OPT_HE_FUSED: *v = c->he_fused; return MFHE_OK;
        case MFHE_OPT_TRACE_SPLIT: *v = c->trace_split; return MFHE_OK;
        case MFHE_OPT_CRT_WORDS: *v = c->W; return MFHE_OK;
        case MFHE_OPT_NTT_U60: *v = c->ntt_u60 && c->u60_ok; return MFHE_OK;
        case MFHE_OPT_HE_STREAMS: *v = c->he_streams; return MFHE_OK;
        case MFHE_OPT_ENC_A_DIRECT: *v = c->enc_a_direct; return MFHE_OK;
        case MFHE_OPT_ENC_E_SMALL: *v = c->enc_e_small; return MFHE_OK;
        case MFHE_OPT_DEC_MM: *v = 0; return MFHE_OK;
        default: return set_error(MFHE_EINVAL, "unknown option");
    }
}

extern "C" int mfhe_ctx_get_moduli(const mfhe_ctx* c, uint64_t* out, int count) {
    if (!c || !out || count < c->L) return set_error(MFHE_EINVAL, "mfhe_ctx_get_moduli: bad argument");
    std::memcpy(out, c->moduli.data(), (size_t)c->L * 8);
    return MFHE_OK;
}

extern "C" const char* mfhe_last_error(void) { return g_last_error.c_str(); }
extern "C" const char* mfhe_version(void) { return "mfhe-mi355x 0.1 (gfx950)"; }
