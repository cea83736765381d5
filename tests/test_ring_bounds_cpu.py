"""CPU restatement of the fused X-axis ring product's FP64 schedule (matrix-fhe-gpu_amd/csrc/ring_row.hpp,
ring_mul_row64_lds; r06: one centred reduction after the fourth forward stage, X left unreduced on every other
inverse stage), op for op in IEEE double with the FMAs evaluated exactly, so that:

* every mulmod meets its precondition |v w / q| < 2^51 (the magic-constant rounding) and every add stays exact
  (|x| < 2^53), for q just below 2^50 (the largest modulus the FP64 path takes) and for a 2^40 modulus, on random
  and on all-(q - 1) / alternating inputs with random centred twiddles;
* the canonical outputs equal the same butterfly network evaluated in exact integers mod q.

The twiddles are random centred values (the bounds depend only on |w| <= q/2), so this checks the schedule, not
the tables; the GPU tests (tests/test_he_gpu.py) check the tables and the kernels."""
from fractions import Fraction

import numpy as np
import pytest

MAGIC = 6755399441055744.0   # 1.5 * 2^52, ntt_arith.hpp ArithF64::kMagic
LIMIT = float(2 ** 51)


class F64:
    """ArithF64 (ntt_arith.hpp) in Python floats with exact FMAs; records the largest |v w / q| and |x| it sees."""

    def __init__(self, q: int):
        self.q = float(q)
        self.qi = q
        self.qinv = 1.0 / float(q)
        self.max_ratio = 0.0
        self.max_abs = 0.0

    @staticmethod
    def fma(a: float, b: float, c: float) -> float:
        return float(Fraction(a) * Fraction(b) + Fraction(c))   # one rounding, as v_fma_f64

    def _seen(self, *xs):
        for x in xs:
            self.max_abs = max(self.max_abs, abs(x))
            assert abs(x) < 2.0 ** 53 and x == int(x), x

    def round_int(self, a: float, b: float) -> float:
        self.max_ratio = max(self.max_ratio, abs(Fraction(a) * Fraction(b)))
        assert abs(Fraction(a) * Fraction(b)) < LIMIT
        return self.fma(a, b, MAGIC) - MAGIC

    def mulmod(self, v: float, w: float) -> float:
        self._seen(v)
        hi = v * w
        lo = self.fma(v, w, -hi)
        k = self.round_int(hi, self.qinv)
        r = self.fma(-k, self.q, hi) + lo
        self._seen(r)
        return r

    def reduce(self, x: float) -> float:
        self._seen(x)
        return self.fma(-self.round_int(x, self.qinv), self.q, x)

    def canon(self, x: float) -> int:
        r = self.reduce(x)
        r = r + self.q if r < 0.0 else r
        return int(r)


def ring_row64(x, sv, tw, itw, ninv, ar, exact=False, q=None):
    """ring_mul_row64_lds for the 16 lanes of one row at once: lane j holds coefficients j + 16 m (layout A) and
    the butterflies act on register pairs exactly as the kernel's (the transposes only move values).  exact=True
    runs the same network in integers mod q (no schedule)."""
    lanes = [[x[j + 16 * m] for m in range(4)] for j in range(16)]
    if exact:
        mm = lambda v, w: (v * w) % q      # noqa: E731
        red = lambda v: v % q              # noqa: E731
    else:
        mm, red = ar.mulmod, ar.reduce

    def ct(r, i0, i1, w):
        t = mm(r[i1], w)
        r[i0], r[i1] = r[i0] + t, r[i0] - t

    def gs(r, i0, i1, w, last, lazy=False):
        u, v = r[i0], r[i1]
        r[i0] = mm(u + v, ninv) if last else (u + v if lazy else red(u + v))
        r[i1] = mm(u - v, w)

    def relayout(src, dst):   # value of coefficient e moves from layout src to layout dst
        val = {}
        for j in range(16):
            for m in range(4):
                val[src(j, m)] = lanes[j][m]
        for j in range(16):
            for m in range(4):
                lanes[j][m] = val[dst(j, m)]

    A = lambda j, m: j + 16 * m                          # noqa: E731
    B = lambda j, m: 16 * (j >> 2) + (j & 3) + 4 * m     # noqa: E731
    C = lambda j, m: 4 * j + m                           # noqa: E731
    for j in range(16):
        r = lanes[j]
        ct(r, 0, 2, tw[1]); ct(r, 1, 3, tw[1]); ct(r, 0, 1, tw[2]); ct(r, 2, 3, tw[3])
    relayout(A, B)
    for j in range(16):
        r, b = lanes[j], j >> 2
        ct(r, 0, 2, tw[4 + b]); ct(r, 1, 3, tw[4 + b]); ct(r, 0, 1, tw[8 + 2 * b]); ct(r, 2, 3, tw[9 + 2 * b])
        for m in range(4):
            r[m] = red(r[m])
    relayout(B, C)
    for j in range(16):
        r = lanes[j]
        ct(r, 0, 2, tw[16 + j]); ct(r, 1, 3, tw[16 + j]); ct(r, 0, 1, tw[32 + 2 * j]); ct(r, 2, 3, tw[33 + 2 * j])
        for m in range(4):
            r[m] = mm(r[m], sv[4 * j + m])
        gs(r, 0, 1, itw[32 + 2 * j], False, True); gs(r, 2, 3, itw[33 + 2 * j], False, True)
        gs(r, 0, 2, itw[16 + j], False); gs(r, 1, 3, itw[16 + j], False)
    relayout(C, B)
    for j in range(16):
        r, b = lanes[j], j >> 2
        gs(r, 0, 1, itw[8 + 2 * b], False, True); gs(r, 2, 3, itw[9 + 2 * b], False, True)
        gs(r, 0, 2, itw[4 + b], False); gs(r, 1, 3, itw[4 + b], False)
    relayout(B, A)
    for j in range(16):
        r = lanes[j]
        gs(r, 0, 1, itw[2], False, True); gs(r, 2, 3, itw[3], False, True)
        gs(r, 0, 2, itw[1], True); gs(r, 1, 3, itw[1], True)
    out = [0] * 64
    for j in range(16):
        for m in range(4):
            v = lanes[j][m]
            out[j + 16 * m] = (v % q) if exact else ar.canon(v)
    return out


@pytest.mark.parametrize("q", [(1 << 50) - 27, (1 << 40) - 87])
@pytest.mark.parametrize("pattern", ["random", "q-1", "alternating"])
def test_ring_row64_schedule_bounds_and_exactness(q, pattern):
    rng = np.random.default_rng(q % 1000 + len(pattern))
    ar = F64(q)
    half = q // 2
    for row in range(6):
        tw = [float(int(v) - half) for v in rng.integers(0, q, 64)]
        itw = [float(int(v) - half) for v in rng.integers(0, q, 64)]
        sv = [float(int(v) - half) for v in rng.integers(0, q, 64)]
        ninv = float(int(rng.integers(0, q)) - half)
        if pattern == "random":
            x = [int(v) for v in rng.integers(0, q, 64)]
        elif pattern == "q-1":
            x = [q - 1] * 64
        else:
            x = [(q - 1) if i % 2 else 0 for i in range(64)]
        got = ring_row64([float(v) for v in x], sv, tw, itw, ninv, ar)
        want = ring_row64(x, [int(v) % q for v in sv], [int(v) % q for v in tw], [int(v) % q for v in itw],
                          int(ninv) % q, None, exact=True, q=q)
        assert got == want
    assert ar.max_ratio < LIMIT
    assert ar.max_abs < 2.0 ** 53
