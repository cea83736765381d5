"""CPU check of the N = 2^14 single-pass kernel's data layouts (matrix-fhe-gpu_amd/csrc/ntt_single14.hpp).

The kernel moves the 128 KiB polynomial between four register layouts through an unpadded LDS buffer whose slots
are XOR-swizzled.  Restated here in Python from the header's comments and checked exhaustively:
  * every layout maps (thread, register) one-to-one onto the 2^14 elements, and its register bits are the bits the
    kernel's stages pair (forward L0: b13..b10, L1: b9..b6, L2: b5..b3 (+ b2), L3: b2..b0 (+ b3));
  * the swizzle is a bijection on [0, 2^14);
  * every exchange access is free of LDS bank conflicts: ds_write_b64 serves 16-lane groups (slots must differ
    mod 16), ds_read_b64 32-lane groups (slots must differ mod 32) (/opt/skills/guides/MI355X_MICROARCH.md, LDS);
  * the twiddle product rule: tw[k] = tw[k & 2047] * tw[k & ~2047] for psi^brev14(k) tables.
"""
import numpy as np


def swz(j):
    h = ((j >> 5) & 1) | (((j >> 6) & 1) << 2) | (((j >> 7) & 1) << 3) | (((j >> 8) & 1) * 18)
    return j ^ h


def jidx(lay, t, k):
    lane, wave = t & 63, t >> 6
    if lay == 0:
        return (k << 10) | t
    if lay == 1:
        return (wave << 10) | (k << 6) | lane
    if lay == 2:
        return (wave << 10) | ((lane >> 2) << 6) | (k << 2) | (lane & 3)
    return (wave << 10) | ((lane >> 5) << 9) | ((lane & 15) << 5) | (((lane >> 4) & 1) << 4) | k


T = np.arange(1024)
KBASE = {0: 10, 1: 6, 2: 2, 3: 0}


def test_layouts_are_bijections_with_the_stage_bits_in_registers():
    for lay in range(4):
        allj = np.concatenate([jidx(lay, T, k) for k in range(16)])
        assert np.array_equal(np.sort(allj), np.arange(1 << 14)), lay
        # register k's bit i is element bit KBASE + i, the same for every thread
        for k in range(16):
            for i in range(4):
                a = jidx(lay, T, k & ~(1 << i))
                b = jidx(lay, T, k | (1 << i))
                assert np.all(b - a == 1 << (KBASE[lay] + i)), (lay, k, i)
    assert np.array_equal(np.sort(swz(np.arange(1 << 14))), np.arange(1 << 14))


def test_exchange_accesses_are_bank_conflict_free():
    for lay in range(4):
        for wave in range(16):
            t = wave * 64 + np.arange(64)
            for k in range(16):
                slot = swz(jidx(lay, t, k))
                for g in range(4):      # ds_write_b64: 4 groups of 16 lanes, 32 banks of 4 B
                    s = slot[16 * g:16 * g + 16] % 16
                    assert len(set(s.tolist())) == 16, ("write", lay, wave, k, g)
                for g in range(2):      # ds_read_b64: 2 groups of 32 lanes, 64 banks of 4 B
                    s = slot[32 * g:32 * g + 32] % 32
                    assert len(set(s.tolist())) == 32, ("read", lay, wave, k, g)


def test_twiddle_product_rule(orc):
    """tw[k] = psi^brev14(k) (ctx.cpp build_ct_tables), so tw[k] = tw[k & 2047] tw[k & ~2047] mod q -- the
    kernel's stage-11..13 twiddles; the inverse table likewise once itw[1]'s folded n^-1 is taken out."""
    q = orc.gen_primes(50, 1 << 16, 1)[0]
    psi = next(pow(g, (q - 1) // (1 << 15), q) for g in range(2, 200)
               if pow(pow(g, (q - 1) // (1 << 15), q), 1 << 14, q) == q - 1)

    def brev(x, bits=14):
        return int(format(x, f"0{bits}b")[::-1], 2)
    tw = [pow(psi, brev(k), q) for k in range(1 << 14)]
    for k in list(range(2048, 1 << 14, 37)) + [2048, 4096, 8191, 16383]:
        assert tw[k] == tw[k & 2047] * tw[k & ~2047] % q, k


def tbits(lay):
    m = 0x1F
    for t in range(1024):
        m |= jidx(lay, t, 0)
    return m


def test_exchange_addresses_split_into_thread_xor_and_immediate():
    """s14_slot: swz(j(t, k)) == (S(t) ^ (C(k) & TB)) + (C(k) & ~TB) with S(t) = swz(j(t, 0)), C(k) = swz(j(0, k));
    the XOR part (in bytes) stays below the buffer's 256-B alignment; L1..L3 keep every wave on its own 1024-element
    block (the wave-local exchanges need no s_barrier)."""
    for lay in range(4):
        tb = tbits(lay)
        S = swz(jidx(lay, T, 0))
        for k in range(16):
            c = int(swz(jidx(lay, 0, k)))
            assert ((c & tb) << 3) < 256, (lay, k)
            assert np.array_equal((S ^ (c & tb)) + (c & ~tb), swz(jidx(lay, T, k))), (lay, k)
            if lay:
                assert np.array_equal(swz(jidx(lay, T, k)) >> 10, T >> 6), (lay, k)


def test_twiddle_index_split():
    """s14_tw: 2^s + (j >> (14 - s)) == 2^s | (jk >> sh) | (jt >> sh) with disjoint parts, so the & 2047 / >> 11 split
    of stages 11..13 distributes over the two parts."""
    for lay in range(4):
        jt = jidx(lay, T, 0)
        for s in range(14):
            sh = 14 - s
            for k in range(16):
                jk = int(jidx(lay, 0, k))
                ck = (1 << s) | (jk >> sh)
                vt = jt >> sh
                assert not np.any(vt & ck)
                idx = (1 << s) + (jidx(lay, T, k) >> sh)
                assert np.array_equal(idx, vt + ck)
                assert np.array_equal(idx & 2047, (vt & 2047) + (ck & 2047))
                assert np.array_equal(idx >> 11, (vt >> 11) + (ck >> 11))
