// host_math.cpp -- see host_math.hpp.
#include "host_math.hpp"

#include <algorithm>
#include <complex>
#include <thread>

namespace mfhe {
namespace hm {

bool is_prime(uint64_t n) {
    if (n < 2) return false;
    static const uint64_t small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (uint64_t p : small) {
        if (n == p) return true;
        if (n % p == 0) return false;
    }
    uint64_t d = n - 1;
    int s = 0;
    while ((d & 1) == 0) { d >>= 1; ++s; }
    for (uint64_t a : small) {
        uint64_t x = powmod(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool composite = true;
        for (int r = 1; r < s; ++r) {
            x = mulmod(x, x, n);
            if (x == n - 1) { composite = false; break; }
        }
        if (composite) return false;
    }
    return true;
}

// SEAL try_minimal_primitive_root: any primitive root g, then min over g^(2i+1), i < degree/2.
uint64_t minimal_primitive_root(uint64_t degree, uint64_t q) {
    if (degree < 2 || (q - 1) % degree != 0) return 0;
    uint64_t g = 0;
    for (uint64_t x = 2; x < q && x < (1ull << 32); ++x) {
        uint64_t c = powmod(x, (q - 1) / degree, q);
        if (powmod(c, degree / 2, q) == q - 1) { g = c; break; }
    }
    if (!g) return 0;
    uint64_t best = g, g2 = mulmod(g, g, q), cur = g;
    for (uint64_t i = 0; i < degree / 2; ++i) {
        if (cur < best) best = cur;
        cur = mulmod(cur, g2, q);
    }
    return best;
}

uint64_t first_psi4n(uint64_t q, uint64_t n) {
    const uint64_t order = 4 * n;
    if ((q - 1) % order != 0) return 0;
    for (uint64_t root = 2; root <= 100000; ++root) {
        uint64_t g = powmod(root, (q - 1) / order, q);
        if (powmod(g, 2 * n, q) == q - 1) return g;
    }
    return 0;
}

uint64_t find_eta771(uint64_t q) {
    const uint64_t p = 771;
    if ((q - 1) % p != 0) return 0;
    const uint64_t e = (q - 1) / p;
    for (uint64_t g = 2; g < q; ++g) {
        uint64_t eta = powmod(g, e, q);
        if (eta == 1) continue;
        if (powmod(eta, p / 3, q) == 1) continue;
        if (powmod(eta, p / 257, q) == 1) continue;
        return eta;
    }
    return 0;
}

void wcrt_exponents(uint16_t* exp512) {
    int idx = 0;
    for (int a = 1; a <= 2; ++a)
        for (int b = 1; b <= 256; ++b) exp512[idx++] = (uint16_t)((a * 257 + b * 3) % 771);
}

bool vandermonde_inverse_mod(const std::vector<uint64_t>& x, uint64_t q, std::vector<uint64_t>& inv) {
    const int dim = (int)x.size();
    inv.assign((size_t)dim * dim, 0);
    std::vector<uint64_t> P((size_t)dim + 1, 0);   // P(X) = prod (X - x_j)
    P[0] = 1;
    for (int j = 0; j < dim; ++j) {
        const uint64_t nx = (q - x[j]) % q;
        for (int k = j + 1; k >= 1; --k) P[k] = addmod(P[k - 1], mulmod(P[k], nx, q), q);
        P[0] = mulmod(P[0], nx, q);
    }
    bool ok = true;
    std::vector<uint64_t> b(dim);
    for (int w = 0; w < dim; ++w) {   // synthetic division P / (X - x_w), then P'(x_w)
        b[dim - 1] = P[dim];
        for (int k = dim - 1; k >= 1; --k) b[k - 1] = addmod(mulmod(x[w], b[k], q), P[k], q);
        uint64_t den = 0;
        for (int k = dim - 1; k >= 0; --k) den = addmod(mulmod(den, x[w], q), b[k], q);
        if (den == 0) { ok = false; continue; }
        const uint64_t di = invmod(den, q);
        for (int r = 0; r < dim; ++r) inv[(size_t)r * dim + w] = mulmod(b[r], di, q);
    }
    return ok;
}

bool complex_inverse_gj(std::vector<double>& a_ri, int dim, std::vector<double>& inv_ri) {
    using C = std::complex<double>;
    C* a = reinterpret_cast<C*>(a_ri.data());
    inv_ri.assign((size_t)dim * dim * 2, 0.0);
    C* inv = reinterpret_cast<C*>(inv_ri.data());
    for (int i = 0; i < dim; ++i) inv[(size_t)i * dim + i] = 1.0;
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    for (int i = 0; i < dim; ++i) {
        int piv = i;
        double best = std::abs(a[(size_t)i * dim + i]);
        for (int r = i + 1; r < dim; ++r) {
            const double cand = std::abs(a[(size_t)r * dim + i]);
            if (cand > best) { best = cand; piv = r; }
        }
        if (best < 1e-18) return false;
        if (piv != i)
            for (int j = 0; j < dim; ++j) {
                std::swap(a[(size_t)i * dim + j], a[(size_t)piv * dim + j]);
                std::swap(inv[(size_t)i * dim + j], inv[(size_t)piv * dim + j]);
            }
        const C pv = a[(size_t)i * dim + i];
        for (int j = 0; j < dim; ++j) { a[(size_t)i * dim + j] /= pv; inv[(size_t)i * dim + j] /= pv; }
        auto work = [&](int r0, int r1) {
            for (int r = r0; r < r1; ++r) {
                if (r == i) continue;
                const C f = a[(size_t)r * dim + i];
                if (std::abs(f) < 1e-18) continue;
                for (int c = 0; c < dim; ++c) {
                    a[(size_t)r * dim + c] -= f * a[(size_t)i * dim + c];
                    inv[(size_t)r * dim + c] -= f * inv[(size_t)i * dim + c];
                }
            }
        };
        std::vector<std::thread> th;
        const int chunk = (dim + (int)nth - 1) / (int)nth;
        for (unsigned t = 0; t < nth; ++t) {
            const int r0 = (int)t * chunk, r1 = std::min(dim, r0 + chunk);
            if (r0 < r1) th.emplace_back(work, r0, r1);
        }
        for (auto& t : th) t.join();
    }
    return true;
}

void big_mul_u64(const uint64_t* a, uint64_t m, uint64_t* out, int W) {
    u128 carry = 0;
    for (int i = 0; i < W; ++i) {
        u128 p = (u128)a[i] * m + carry;
        out[i] = (uint64_t)p;
        carry = p >> 64;
    }
}

int bitlen(const std::vector<uint64_t>& a) {
    for (int i = (int)a.size() - 1; i >= 0; --i)
        if (a[i]) return i * 64 + 64 - __builtin_clzll(a[i]);
    return 0;
}

}  // namespace hm
}  // namespace mfhe
