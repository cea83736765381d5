"""Test helper: primes of a given bit size in a residue class (deterministic Miller-Rabin, no GPU, no oracle)."""


_BASES = (2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37)


def _is_prime(n: int) -> bool:
    """Deterministic Miller-Rabin for n < 2^64 (the 12 prime bases cover 64 bits)."""
    if n < 2:
        return False
    for p in _BASES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for a in _BASES:
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def primes_of_size(bits: int, m: int, count: int) -> list[int]:
    """Up to `count` distinct primes of exactly `bits` bits with q = 1 mod m: the largest first, then the smallest
    (alternating), so a context holds both ends of the size class. Empty if none exists."""
    lo, hi = 1 << (bits - 1), (1 << bits) - 1
    top = ((hi - 1) // m) * m + 1
    bot = ((lo - 1 + m - 1) // m) * m + 1
    big, small = [], []
    c = top
    while c >= lo and len(big) < count and top - c < 4000 * m:
        if _is_prime(c):
            big.append(c)
        c -= m
    c = bot
    while c <= hi and len(small) < count and c - bot < 4000 * m:
        if _is_prime(c):
            small.append(c)
        c += m
    out = []
    for a, b in zip(big + [None] * count, small + [None] * count):
        for v in (a, b):
            if v is not None and v not in out and len(out) < count:
                out.append(v)
    return out
