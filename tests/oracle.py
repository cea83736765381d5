"""ctypes bindings for oracle/liboracle.so -- the CPU restatement of the reference hot path.

Test infrastructure only (the checker, never the thing measured or shipped).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
ORACLE_SO = ORACLE_DIR / "liboracle.so"


def _load():
    src = ORACLE_DIR / "mfhe_oracle.c"
    if not ORACLE_SO.exists() or ORACLE_SO.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, capture_output=True)
    return ctypes.CDLL(str(ORACLE_SO))


L = _load()
u64 = ctypes.c_uint64
vp = ctypes.c_void_p
sz = ctypes.c_size_t
ci = ctypes.c_int


def _s(name, args, res=None):
    f = getattr(L, name)
    f.argtypes = args
    f.restype = res
    return f


_s("orc_mulmod", [u64, u64, u64], u64)
_s("orc_powmod", [u64, u64, u64], u64)
_s("orc_invmod", [u64, u64], u64)
_s("orc_is_prime", [u64], ci)
_s("orc_gen_primes", [ci, u64, ci, vp], ci)
_s("orc_minimal_primitive_root", [u64, u64], u64)
_s("orc_get_psi4n", [u64, ci], u64)
_s("orc_find_eta", [u64], u64)
_s("orc_phantom_tables", [ci, u64, vp, vp, vp, vp, vp, vp])
for n in ("orc_phantom_fwd", "orc_phantom_inv", "orc_phantom_fwd_1t"):
    _s(n, [vp, sz, ci, ci, vp])
for n in ("orc_custom_ntt_fwd", "orc_custom_ntt_bwd", "orc_gl_ntt_fwd", "orc_gl_ntt_bwd"):
    _s(n, [vp, sz, ci, ci, vp])
_s("orc_gl_perm_table", [ci, vp, vp])
_s("orc_gl_perm", [vp, vp, sz, ci, ci, ci])
_s("orc_wcrt_exp", [vp])
_s("orc_wcrt_tables", [u64, vp, vp, ci], ci)
_s("orc_wntt_forward_matrix", [vp, vp, ci, ci, ci, vp, vp])
_s("orc_wntt_inverse_matrix", [vp, vp, ci, ci, ci, vp, vp])
_s("orc_wntt_forward_vector", [vp, vp, ci, ci, ci, vp, vp])
_s("orc_wntt_forward_centered", [vp, vp, ci, ci, ci, vp, vp, ci])
_s("orc_wntt_inverse_centered", [vp, vp, ci, ci, vp, vp])
_s("orc_crt_min_words", [vp, ci], ci)
_s("orc_crt_tables", [vp, ci, ci, vp, vp, vp, vp], ci)
for n in ("orc_crt_compose", "orc_crt_compose_1t"):
    _s(n, [vp, sz, ci, sz, vp, ci, vp, vp])
_s("orc_crt_compose_i64", [vp, sz, ci, sz, vp, ci, vp])
_s("orc_set_threads", [ci])
_s("orc_max_threads", [], ci)
_s("orc_big_to_f64", [vp, vp, sz, ci, ctypes.c_double, vp, sz])
for n in ("orc_rns_decompose", "orc_rns_decompose_1t"):
    _s(n, [vp, sz, sz, sz, ci, vp, ctypes.c_double, vp])
_s("orc_encoder_matrices", [ci, vp, vp, vp, vp])
_s("orc_cmatmul", [vp, vp, vp, ci])
_s("orc_wdft_tables", [vp, vp], ci)
_s("orc_w_idft", [vp, vp, vp, ci, ci])
_s("orc_wdft_forward", [vp, vp, vp, ci, ci])
for n in ("orc_ternary_secret", "orc_uniform_random", "orc_gaussian_noise"):
    _s(n, [vp, ci, ci, ci, vp])
_s("orc_matrix_to_poly", [vp, vp, ci, ci, ci])
_s("orc_poly_to_matrix", [vp, vp, ci, ci, ci])
_s("orc_he_create", [ci, ci, vp, ctypes.c_double, ci], vp)
_s("orc_he_destroy", [vp])
_s("orc_he_encode", [vp, vp, vp, vp])
_s("orc_he_keygen", [vp, vp])
_s("orc_he_encrypt_pair", [vp, vp, vp, vp, vp, vp])
_s("orc_he_decrypt_to_eval", [vp, vp, vp, vp])
_s("orc_he_decode", [vp, vp, vp, vp])
_s("orc_he_decode_stages", [vp] + [vp] * 13)
_s("orc_he_words", [vp], ci)
_s("orc_he_V", [vp], vp)
_s("orc_he_VinvT", [vp], vp)
_s("orc_trace_map_bprime", [vp, vp, vp, vp, ci, ci, sz, vp])
_s("orc_trace_gemm", [vp, vp, vp, vp, vp, vp, ci, ci, sz, vp])
_s("orc_trace_rescale", [vp, vp, ci, ci, sz, vp, vp])
_s("orc_splitmix64", [u64], u64)
_s("orc_fill_residues", [vp, sz, ci, sz, vp, u64, sz])
_s("orc_fill_messages", [vp, sz, u64, sz])


def fill_residues(npoly: int, L_: int, N: int, moduli, seed: int, poly0: int = 0) -> np.ndarray:
    """Deterministic synthetic residues [npoly][L][N] (orc_fill_residues; SURVEY.md §8(d) seeds)."""
    out = np.empty(npoly * L_ * N, np.uint64)
    L.orc_fill_residues(P(out), npoly, L_, N, P(U64(moduli)), seed, poly0)
    return out


def fill_messages(count: int, seed: int, idx0: int = 0) -> np.ndarray:
    """Deterministic messages in [-1, 1) (orc_fill_messages)."""
    out = np.empty(count, np.float64)
    L.orc_fill_messages(P(out), count, seed, idx0)
    return out


def P(a: np.ndarray):
    return a.ctypes.data_as(vp)


def U64(x) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=np.uint64)


# ------------- convenience wrappers -------------
def gen_primes(bits: int, m: int, count: int) -> list[int]:
    out = np.zeros(count, dtype=np.uint64)
    n = L.orc_gen_primes(bits, m, count, P(out))
    assert n == count, f"only {n} primes found"
    return [int(x) for x in out]


def phantom_fwd(data: np.ndarray, L_: int, log_n: int, moduli) -> np.ndarray:
    d = U64(data).copy()
    m = U64(moduli)
    L.orc_phantom_fwd(P(d), d.size // (L_ << log_n), L_, log_n, P(m))
    return d


def phantom_inv(data: np.ndarray, L_: int, log_n: int, moduli) -> np.ndarray:
    d = U64(data).copy()
    m = U64(moduli)
    L.orc_phantom_inv(P(d), d.size // (L_ << log_n), L_, log_n, P(m))
    return d


def phantom_tables(log_n: int, q: int):
    n = 1 << log_n
    tw, tws, itw, itws = (np.zeros(n, np.uint64) for _ in range(4))
    ninv, ninvs = np.zeros(1, np.uint64), np.zeros(1, np.uint64)
    L.orc_phantom_tables(log_n, q, P(tw), P(tws), P(itw), P(itws), P(ninv), P(ninvs))
    return tw, tws, itw, itws, int(ninv[0]), int(ninvs[0])


def _custom(fn, data, L_, n, moduli):
    d = U64(data).copy()
    m = U64(moduli)
    fn(P(d), d.size // (L_ * n), L_, n, P(m))
    return d


def custom_fwd(d, L_, n, m): return _custom(L.orc_custom_ntt_fwd, d, L_, n, m)
def custom_bwd(d, L_, n, m): return _custom(L.orc_custom_ntt_bwd, d, L_, n, m)
def gl_fwd(d, L_, n, m): return _custom(L.orc_gl_ntt_fwd, d, L_, n, m)
def gl_bwd(d, L_, n, m): return _custom(L.orc_gl_ntt_bwd, d, L_, n, m)


def gl_perm(data, L_, n, inverse=False):
    d = U64(data)
    out = np.zeros_like(d)
    L.orc_gl_perm(P(d), P(out), d.size // (L_ * n), L_, n, int(inverse))
    return out


def crt_words(moduli) -> int:
    m = U64(moduli)
    return L.orc_crt_min_words(P(m), len(moduli))


def crt_compose(data, npoly, L_, N, moduli, W=None):
    d = U64(data)
    m = U64(moduli)
    W = W or crt_words(moduli)
    mag = np.zeros(npoly * N * W, np.uint64)
    neg = np.zeros(npoly * N, np.uint8)
    L.orc_crt_compose(P(d), npoly, L_, N, P(m), W, P(mag), P(neg))
    return mag.reshape(npoly * N, W), neg


def crt_compose_i64(data, npoly, L_, N, moduli, W=None):
    """encoder.cu:152-189: centred CRT value truncated to int64 (low magnitude word, sign with wrap)."""
    d = U64(data)
    m = U64(moduli)
    W = W or crt_words(moduli)
    out = np.zeros(npoly * N, np.int64)
    L.orc_crt_compose_i64(P(d), npoly, L_, N, P(m), W, P(out))
    return out


def big_to_f64(mag, neg, W, delta):
    mag = U64(mag)
    neg = np.ascontiguousarray(neg, np.uint8)
    cnt = neg.size
    out = np.zeros(cnt, np.float64)
    L.orc_big_to_f64(P(mag), P(neg), cnt, W, delta, P(out), 1)
    return out


def rns_decompose(vals, npoly, N, moduli, delta, stride=1):
    v = np.ascontiguousarray(vals, np.float64)
    m = U64(moduli)
    out = np.zeros(npoly * len(moduli) * N, np.uint64)
    L.orc_rns_decompose(P(v), stride, npoly, N, len(moduli), P(m), delta, P(out))
    return out


def wcrt_exp() -> np.ndarray:
    e = np.zeros(512, np.uint16)
    L.orc_wcrt_exp(P(e))
    return e


def wcrt_tables(q: int, gauss: bool = False):
    V = np.zeros(512 * 512, np.uint64)
    Vi = np.zeros(512 * 512, np.uint64)
    rc = L.orc_wcrt_tables(q, P(V), P(Vi), int(gauss))
    assert rc == 0
    return V, Vi


# ---- trace GEMM, [batch][L][n][n] planes (batched_trace.cu) ----
def trace_map_bprime(br, bi, n, L_, batch, moduli):
    br, bi = U64(br), U64(bi)
    opr, opi = np.zeros_like(br), np.zeros_like(bi)
    L.orc_trace_map_bprime(P(br), P(bi), P(opr), P(opi), n, L_, batch, P(U64(moduli)))
    return opr, opi


def trace_gemm(ar, ai, br, bi, n, L_, batch, moduli):
    ar, ai, br, bi = U64(ar), U64(ai), U64(br), U64(bi)
    cr, ci_ = np.zeros_like(ar), np.zeros_like(ai)
    L.orc_trace_gemm(P(ar), P(ai), P(br), P(bi), P(cr), P(ci_), n, L_, batch, P(U64(moduli)))
    return cr, ci_


def trace_rescale(cr, ci_, n, L_, batch, moduli, inv):
    cr, ci_ = U64(cr).copy(), U64(ci_).copy()
    L.orc_trace_rescale(P(cr), P(ci_), n, L_, batch, P(U64(moduli)), P(U64(inv)))
    return cr, ci_


class HE:
    """orc_he pipeline context (reference geometry)."""

    def __init__(self, n, moduli, delta, gauss=False):
        self.n, self.moduli, self.delta = n, list(moduli), delta
        self.L = len(moduli)
        self._m = U64(moduli)
        self.h = L.orc_he_create(n, self.L, P(self._m), delta, int(gauss))
        assert self.h, "orc_he_create failed"
        self.W = L.orc_he_words(self.h)
        self.phi = 512

    def __del__(self):
        if getattr(self, "h", None):
            L.orc_he_destroy(self.h)
            self.h = None

    @property
    def words(self):
        return self.phi * self.L * self.n * self.n

    def encode(self, msg):
        msg = np.ascontiguousarray(msg, np.complex128)
        re_ = np.zeros(self.words, np.uint64)
        im_ = np.zeros(self.words, np.uint64)
        L.orc_he_encode(self.h, P(msg), P(re_), P(im_))
        return re_, im_

    def keygen(self):
        sk = np.zeros(self.phi * self.L * self.n, np.uint64)
        L.orc_he_keygen(self.h, P(sk))
        return sk

    def encrypt_pair(self, m_re, m_im, sk):
        cre = np.zeros(2 * self.words, np.uint64)
        cim = np.zeros(2 * self.words, np.uint64)
        L.orc_he_encrypt_pair(self.h, P(U64(m_re)), P(U64(m_im)), P(U64(sk)), P(cre), P(cim))
        return cre, cim

    def decrypt_to_eval(self, ct, sk):
        out = np.zeros(self.words, np.uint64)
        L.orc_he_decrypt_to_eval(self.h, P(U64(ct)), P(U64(sk)), P(out))
        return out

    def decode(self, ev_re, ev_im):
        msg = np.zeros(self.phi * self.n * self.n, np.complex128)
        L.orc_he_decode(self.h, P(U64(ev_re)), P(U64(ev_im)), P(msg))
        return msg
