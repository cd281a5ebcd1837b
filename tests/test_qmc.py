"""QMC sequences of the oracle (mcqmc.h, scr_halton.h, faure tables) checked
against independent Python restatements."""
import ctypes as C

import numpy as np
import pytest

from oracle.oracle import lib

PRIMES = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89, 97,
          101, 103, 107, 109, 113, 127, 131, 137, 139, 149, 151, 157, 163, 167, 173, 179, 181, 191, 193, 197, 199,
          211, 223, 227]


def faure_perm(b):
    """Faure's permutation of 0..b-1 (standard recursive construction)."""
    if b == 2:
        return [0, 1]
    if b % 2 == 0:
        h = faure_perm(b // 2)
        return [2 * v for v in h] + [2 * v + 1 for v in h]
    c = (b - 1) // 2
    prev = faure_perm(b - 1)
    out = [v + 1 if v >= c else v for v in prev]
    return out[:c] + [c] + out[c:]


def test_faure_tables():
    for dim in range(50):
        base = 3 if dim < 2 else PRIMES[dim - 1]
        n = 1 if dim == 0 else (2 if dim == 1 else base)
        out = (C.c_int * max(n, 3))()
        lib().orc_faure(dim, out)
        ref = faure_perm(base)
        assert list(out[:n]) == ref[:n]
        if dim >= 2:
            assert sorted(ref) == list(range(base))


def fnv(v):
    h = 0x811C9DC5
    for i in range(4):
        h ^= (v >> (8 * i)) & 0xFF
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


def ri_vdc(bits, r):
    b = int("{:032b}".format(bits)[::-1], 2)
    return np.float32(min(max((b ^ r) * 2.0 ** -32, 0.0), 1.0))


def ri_lp(i, r):
    v = 1 << 31
    while i:
        if i & 1:
            r ^= v
        i >>= 1
        v |= v >> 1
    return np.float32(min(max(r * 2.0 ** -32, 0.0), 1.0))


@pytest.mark.parametrize("seed", [1, 2])
def test_radical_inverses_and_hash(seed):
    rng = np.random.default_rng(seed)
    for v in rng.integers(0, 2 ** 32, 200, dtype=np.uint64):
        v = int(v)
        assert lib().orc_fnv(v) == fnv(v)
        assert np.float32(lib().orc_ri_vdc(v, 0)) == ri_vdc(v, 0)
        assert np.float32(lib().orc_ri_lp(v & 0xFFFF, 0)) == ri_lp(v & 0xFFFF, 0)


def test_scrambled_halton_is_a_radical_inverse_in_base():
    # scrHalton(dim, n), scr_halton.h:47-69: digits of n in base prims[dim]
    # through Faure's permutation, with n advanced as (unsigned)(n * invPrim)
    # in double and invPrim = 1/p printed with 9 decimals (scr_halton.h:34-43)
    # -- so e.g. n = p gives 0 (then clamped to 1e-36), as in the reference.
    for dim in (2, 3, 7, 11, 20):
        base = PRIMES[dim - 1]
        perm = faure_perm(base)
        inv = float("%.9f" % (1.0 / base))
        for n in (1, 2, base - 1, base, base * base + 3, 123457):
            val, dn, factor, k = 0.0, float(n), inv, n
            while k > 0:
                val += perm[k % base] * factor
                dn *= inv
                k = int(dn)
                factor *= inv
            val = min(max(val, 1e-36), 1.0)
            assert lib().orc_scrhalton(dim, n) == val


def test_halton_sequence_monotone_fractions():
    out = (C.c_float * 64)()
    lib().orc_halton_seq(2, 0, 64, out)
    # base-2 radical inverse of 1..64
    ref = [int("{:b}".format(i)[::-1], 2) / 2 ** len("{:b}".format(i)) for i in range(1, 65)]
    assert np.allclose(np.array(out[:]), ref, atol=1e-6)
