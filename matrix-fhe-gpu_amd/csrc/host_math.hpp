// host_math.hpp -- host-side number theory for building device tables.
//
// Mirrors the table construction the reference does on the host:
//   * phantom::arith::NTT tables: psi = minimal primitive
//     2n-th root (SEAL try_minimal_primitive_root), tw[brev(i)] = psi^i,
//     itw[brev(i)] = psi^-i with itw[1] *= n^-1, Shoup companions.
//   * GL tables (ntt_core.cu:49-70,75-148,175-198): psi4n = first g^((q-1)/4n)
//     with g^(2n) == -1 (g = 2,3,...).
//   * W-CRT eta (HE.cu:119-133) and CRT constants (encoder.cu:341-421).
#pragma once
#include <cstdint>
#include <vector>

namespace mfhe {
namespace hm {

using u128 = unsigned __int128;

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) { uint64_t s = a + b; return s >= q ? s - q : s; }
inline uint64_t submod(uint64_t a, uint64_t b, uint64_t q) { return a >= b ? a - b : a + q - b; }
inline uint64_t powmod(uint64_t a, uint64_t e, uint64_t q) {
    uint64_t r = 1 % q;
    a %= q;
    while (e) {
        if (e & 1) r = mulmod(r, a, q);
        a = mulmod(a, a, q);
        e >>= 1;
    }
    return r;
}
inline uint64_t invmod(uint64_t a, uint64_t q) { return powmod(a, q - 2, q); }
inline uint64_t shoup(uint64_t w, uint64_t q) { return (uint64_t)(((u128)w << 64) / q); }
inline uint32_t brev(uint32_t x, int bits) {
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) { r = (r << 1) | (x & 1u); x >>= 1; }
    return r;
}

bool is_prime(uint64_t n);
// smallest primitive `degree`-th root of unity mod q (SEAL semantics); 0 if none
uint64_t minimal_primitive_root(uint64_t degree, uint64_t q);
// reference get_psi (ntt_core.cu:49-70); 0 if none
uint64_t first_psi4n(uint64_t q, uint64_t n);
// reference h_find_eta (HE.cu:119-133); 0 if none
uint64_t find_eta771(uint64_t q);

// exp[] order of the 512 W lanes (HE.cu:72-105 == batched_encoder.cu:276-282): a*257 + b*3 mod 771
void wcrt_exponents(uint16_t* exp512);
// Exact inverse of the Vandermonde matrix V[w][r] = x_w^r mod q (dim x dim, row-major out[r][w]) by
// Lagrange interpolation, O(dim^2).  Equal to the reference's Gauss-Jordan inverse (HE.cu:135-185),
// the inverse being unique.  Returns false if two points coincide.
bool vandermonde_inverse_mod(const std::vector<uint64_t>& x, uint64_t q, std::vector<uint64_t>& inv);
// Complex Gauss-Jordan with partial pivoting (matrix_inverse_complex, HE.cu:187-235); row-major, in place.
bool complex_inverse_gj(std::vector<double>& a_ri, int dim, std::vector<double>& inv_ri);

// multiprecision helpers, little-endian words
void big_mul_u64(const uint64_t* a, uint64_t m, uint64_t* out, int W);
int bitlen(const std::vector<uint64_t>& a);

}  // namespace hm
}  // namespace mfhe
