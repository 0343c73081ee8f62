"""The split-input Shoup product of the 60-bit primes' butterflies (csrc/hec_device.h shoup_split_lazy), restated
with Python integers and checked against exact modular products: t = Y w mod q lies in [0, 2q) for every Y < 4q,
and the two 32-bit quotient factors it needs come out of the Shoup factor wq = floor(w 2^64 / q) that the twiddle
tables already hold.  Host-only (the kernels' bits are covered by the GPU parity suite under HEC_SPLIT_BFLY)."""
import random

import pytest

M64 = (1 << 64) - 1
M32 = (1 << 32) - 1

# 2^60 - 262143 (SEAL's first 60-bit prime for N = 2^15, tools/micro_bfly.hip) and other odd moduli just below 2^60
# (the bounds hold for any odd q < 2^60)
PRIMES = [1152921504606584833, (1 << 60) - 1, (1 << 60) - (1 << 32) + 1, (1 << 59) + 65537]


def split_lazy(Y, w, wq, a, q):
    """shoup_split_lazy on u64 / u32 words: Y = y1 2^31 + y0, Y w == y1 a + y0 w (mod q), a = w 2^31 mod q."""
    y0, y1 = Y & 0x7FFFFFFF, Y >> 31
    assert y1 < (1 << 32)
    ap, wp = (wq >> 1) & M32, wq >> 32
    qs = y1 * ap + y0 * wp
    assert qs <= M64  # the quotient sum fits the 64-bit multiply-add chain
    qh = qs >> 32
    lo = (y0 * (w & M32) + y1 * (a & M32)) & M64
    hi = (y0 * (w >> 32) + y1 * (a >> 32)) & M32
    return (lo + (hi << 32) - ((qh * (q & M32) + (((qh * (q >> 32)) & M32) << 32)) & M64)) & M64


@pytest.mark.parametrize("q", PRIMES)
def test_split_shoup_range_and_residue(q):
    assert q < (1 << 60)  # the engine rejects wider moduli (coeff_modulus check), which the bounds below need
    rng = random.Random(q)
    edge = [0, 1, q - 1, q, 2 * q - 1, 4 * q - 1]
    for _ in range(4000):
        w = rng.choice([0, 1, q - 1, rng.randrange(q)])
        Y = rng.choice(edge + [rng.randrange(4 * q)])
        wq = (w << 64) // q
        a = (w << 31) % q
        # the quotient factors are bits of wq
        assert ((a << 32) // q) == ((wq >> 1) & M32)
        assert ((w << 32) // q) == (wq >> 32)
        t = split_lazy(Y, w, wq, a, q)
        assert t < 2 * q
        assert t % q == (Y * w) % q


@pytest.mark.parametrize("q", PRIMES[:2])
def test_split_shoup_butterflies_match_plain_shoup(q):
    """Harvey CT / GS butterflies built on either product give the same canonical outputs."""
    rng = random.Random(7 * q)
    two_q = 2 * q

    def shoup_lazy(Y, w, wq):
        return (Y * w - ((Y * wq) >> 64) * q) & M64

    for _ in range(2000):
        w = rng.randrange(q)
        wq = (w << 64) // q
        a = (w << 31) % q
        X, Y = rng.randrange(4 * q), rng.randrange(4 * q)
        x = X - two_q if X >= two_q else X
        t1, t2 = shoup_lazy(Y, w, wq), split_lazy(Y, w, wq, a, q)
        assert (x + t1) % q == (x + t2) % q and (x - t1 + two_q) % q == (x - t2 + two_q) % q
        assert x + t2 < 4 * q and x - t2 + two_q < 4 * q
