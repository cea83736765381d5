// host_math.cpp -- see host_math.hpp.
#include "host_math.hpp"

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
