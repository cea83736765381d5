"""Full-shape parity configurations (BASELINE.json configs C2, C3, C4-shard, C5-shard) and their digests.

Test infrastructure.  The BASELINE shapes are too large to commit as vectors (C3 is 4 GiB per buffer,
the C5 shard 16 GiB), so the CPU oracle's outputs are committed as SHA-256 digests instead
("SHA-256 digests of full outputs for the larger configs"):

  per-poly digest  d_p = SHA-256(bytes of polynomial p's output, little-endian, all limbs / words)
  top digest       D   = SHA-256(d_0 || d_1 || ... || d_{npoly-1})

so a mismatch on the GPU names the polynomial that differs, and hashing parallelises over threads.
Inputs come from the oracle's deterministic generator (orc_fill_residues / orc_fill_messages,
splitmix64 of seed + element index) with the SURVEY.md §8(d) seeds 0x4D46484500000000 + config id.
Moduli: the largest L primes q < 2^bits with q = 1 mod 4N (oracle gen_primes, same as bench.py).

`make_digests.py` writes digests.npz from the oracle; tests/test_fullshape_gpu.py recomputes them from
the HIP path through the C ABI; tests/test_fullshape_cpu.py re-derives sample polynomials on the CPU.
"""
from __future__ import annotations

import hashlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

SEED0 = 0x4D46484500000000
DELTA = 2.0 ** 35

# name -> shape.  ctx moduli = gen_primes(bits, 4N, L); the NTT runs on limbs [start, start + nl).
NTT_CONFIGS = {
    # BASELINE configs[1]: N = 2^14, 4 RNS moduli, batch 256, forward + inverse
    "c2": dict(log_n=14, L=4, bits=50, batch=256, start=0, nl=4, seed=SEED0 + 2, kinds=("fwd", "inv")),
    # configs[2]: N = 2^16, 8 moduli, batch 1024 (the bench's headline shape and moduli)
    "c3": dict(log_n=16, L=8, bits=50, batch=1024, start=0, nl=8, seed=SEED0 + 3, kinds=("fwd", "inv")),
    # the same shape with 60-bit primes: the U64 (Harvey/Shoup) arithmetic path
    "c3u60": dict(log_n=16, L=8, bits=60, batch=1024, start=0, nl=8, seed=SEED0 + 0x33, kinds=("fwd", "inv")),
    # configs[3] residue shard: N = 2^16, 16 moduli, batch 1024; GPU 1 of 4 owns limbs 4..7
    "c4shard": dict(log_n=16, L=16, bits=50, batch=1024, start=4, nl=4, seed=SEED0 + 4, kinds=("fwd", "inv")),
    # configs[4] residue shard: N = 2^17, 32 moduli, batch 4096; GPU 1 of 8 owns limbs 4..7
    "c5shard": dict(log_n=17, L=32, bits=50, batch=4096, start=4, nl=4, seed=SEED0 + 5, kinds=("fwd",)),
}

# configs[2] encode -> NTT -> INTT -> decode with CRT, generic length-N batch:
# messages m (seed + 0x100) -> RNS decompose (delta 2^35) -> forward NTT -> inverse NTT -> compose -> f64.
# Digests: "decomp" (residues), "decomp_fwd" (NTT of the residues), "compose_f64" (the round trip's
# decoded doubles), and "compose_int" (wide CRT magnitudes + signs of the uniform C3 input residues,
# which exercise the full bigint path, not the small-value fast path).
C3_PIPE = dict(cfg="c3", msg_seed=SEED0 + 3 + 0x100, delta=DELTA)
CHUNK_POLYS = {14: 256, 16: 64, 17: 32}


def moduli_for(cfg: dict) -> list[int]:
    import oracle as O
    return O.gen_primes(cfg["bits"], 1 << (cfg["log_n"] + 2), cfg["L"])


def shard_moduli(cfg: dict) -> list[int]:
    m = moduli_for(cfg)
    return m[cfg["start"]: cfg["start"] + cfg["nl"]]


def poly_digests(buf: np.ndarray, npoly: int, extra: np.ndarray | None = None, threads: int = 16) -> np.ndarray:
    """[npoly][32] uint8 SHA-256 of each polynomial's bytes (buf split into npoly equal slices; `extra`,
    if given, is split the same way and its slice is hashed after the main slice)."""
    b = np.ascontiguousarray(buf).reshape(-1).view(np.uint8)
    per = b.size // npoly
    assert per * npoly == b.size
    e = None if extra is None else np.ascontiguousarray(extra).reshape(-1).view(np.uint8)
    pe = 0 if e is None else e.size // npoly

    def one(p):
        h = hashlib.sha256(memoryview(b[p * per:(p + 1) * per]))
        if e is not None:
            h.update(memoryview(e[p * pe:(p + 1) * pe]))
        return np.frombuffer(h.digest(), np.uint8)

    with ThreadPoolExecutor(threads) as ex:
        return np.stack(list(ex.map(one, range(npoly))))


def top_digest(per_poly: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(per_poly, dtype=np.uint8).tobytes()).hexdigest()


def first_mismatch(got: np.ndarray, want: np.ndarray) -> int | None:
    bad = np.nonzero((got != want).any(axis=1))[0]
    return None if bad.size == 0 else int(bad[0])
