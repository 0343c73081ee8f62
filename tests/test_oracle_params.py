"""Oracle pinning: parameter setup (SURVEY §8(a) a11, §8(c) 'Conventions pinned by static reading of
build/demo').  The prime tables below are SEAL 4.1's CoeffModulus::Create output for the BASELINE
configs as statically read from the reference's build/demo disassembly."""
import random

import pytest

from _helpers import ks_count

# SURVEY §8 parameter table (cfg1 = the reference demo, matrix_operations.cpp:1050)
CFG1 = [0xffffffffffe8001, 0xfffff4c001, 0xfffffdc001, 0xfffffffffffc001]
CFG2_FIRST, CFG2_P = 0xfffffffff840001, 0xffffffffffc0001
CFG2_40 = (0xffff690001, 0xffffe80001)  # first and last of the ascending 40-bit primes


def test_create_coeff_modulus_cfg1(orc):
    assert orc.Oracle.create_coeff_modulus(1 << 13, [60, 40, 40, 60]) == CFG1


def test_create_coeff_modulus_cfg2(orc):
    m = orc.Oracle.create_coeff_modulus(1 << 15, [60] + [40] * 9 + [60])
    assert m[0] == CFG2_FIRST and m[-1] == CFG2_P
    assert m[1] == CFG2_40[0] and m[9] == CFG2_40[1]
    assert m[1:10] == sorted(m[1:10])  # .back() of the descending list: ascending 40-bit primes
    assert all(q % (2 << 15) == 1 for q in m)


def test_create_coeff_modulus_cfg5(orc):
    m = orc.Oracle.create_coeff_modulus(1 << 16, [60] + [40] * 15 + [60])
    assert m[0] == CFG2_FIRST and m[-1] == CFG2_P and len(m) == 17
    assert m[1:16] == sorted(m[1:16]) and all(q % (2 << 16) == 1 for q in m)


def test_product_coeff_modulus_matches_oracle(orc, hecdna):
    for N, bits in [(1 << 13, [60, 40, 40, 60]), (1 << 15, [60] + [40] * 9 + [60]), (1 << 11, [50, 36, 36, 50])]:
        assert hecdna.create_coeff_modulus(N, bits) == orc.Oracle.create_coeff_modulus(N, bits)


def test_is_prime_and_barrett(orc):
    L = orc.lib()
    assert L.orc_is_prime(CFG1[0]) == 1 and L.orc_is_prime(CFG1[0] + 2) == 0
    rnd = random.Random(1)
    for q in CFG1 + [CFG2_FIRST]:
        for _ in range(200):
            x = rnd.getrandbits(rnd.choice([64, 100, 120, 127, 128]))
            assert orc.Oracle.barrett128(x & (2**64 - 1), x >> 64, q) == x % q


def test_minimal_primitive_root(orc):
    N = 1 << 10
    m = orc.Oracle.create_coeff_modulus(N, [50, 40, 50])
    o = orc.Oracle(N, m)
    for i, q in enumerate(m):
        psi = o.root(i)
        assert pow(psi, N, q) == q - 1
        # minimal among all primitive 2N-th roots psi^(odd)
        allr = [pow(psi, k, q) for k in range(1, 2 * N, 2)]
        assert psi == min(allr)


def test_galois_elts_and_naf(orc):
    N = 1 << 13
    o = orc.Oracle(N, CFG1)
    elts = o.default_galois_elts()
    assert len(elts) == 25 and elts[0] == 2 * N - 1  # 25 default Galois keys
    assert o.elt_from_step(1) == 3 and o.elt_from_step(2) == 9
    assert o.elt_from_step(-1) == pow(3, N // 2 - 1, 2 * N)
    assert o.elt_from_step(0) == 2 * N - 1
    assert set(elts[1::2]) == {pow(3, 2**i, 2 * N) for i in range(12)}
    assert o.naf(3) == [-1, 4] and o.naf(7) == [-1, 8] and o.naf(-5) == [-1, -4]
    assert o.naf(4095) == [-1, 4096]
    with pytest.raises(orc.OracleError, match="step count too large"):
        o.elt_from_step(N // 2)


def test_keyswitch_counts_match_survey():
    # 156 key switches per cfg1 matvec, 18,204 per cfg3 matvec
    assert ks_count(1 << 13, 64) == 156
    assert ks_count(1 << 15, 4096) == 18204
