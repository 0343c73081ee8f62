"""SEAL 4.1 wire format (client.cpp:113-115, server.cpp:110-122): the engine's C-ABI
reader/writer (csrc/hec_seal_io.cpp) against an independent pure-Python restatement of the layout
(tests/seal_format.py), BLAKE2b against hashlib, and round trips through zlib and zstd.  Host only.
Parity vs SEAL itself is unpinned: no SEAL-written bytes exist under /root/reference."""
import hashlib
import zlib

import numpy as np
import pytest

import seal_format as sf

N = 1 << 11
MOD = [1125899906826241, 68719403009, 68719230977, 1125899906629633]  # 50, 36, 36, 50-bit NTT primes


def rand_ct(size, level, seed=0):
    rng = np.random.default_rng(seed)
    return np.stack([np.stack([rng.integers(0, MOD[i], N, dtype=np.uint64) for i in range(level)])
                     for _ in range(size)])


@pytest.mark.parametrize("n", [0, 1, 63, 127, 128, 129, 255, 256, 1000])
def test_blake2b_matches_hashlib(hecdna, n):
    data = bytes(range(256)) * 4
    assert hecdna.seal_blake2b(data[:n], 64) == hashlib.blake2b(data[:n]).digest()
    assert hecdna.seal_blake2b(data[:n], 32) == hashlib.blake2b(data[:n], digest_size=32).digest()


def test_parms_id_is_blake2b_of_parameter_words(hecdna):
    for lvl in (1, 3, 4):
        assert np.array_equal(hecdna.seal_parms_id(N, MOD[:lvl]), sf.parms_id(N, MOD[:lvl]))


@pytest.mark.parametrize("size,level", [(2, 3), (3, 2), (2, 1)])
def test_ciphertext_save_equals_restatement_and_loads(hecdna, size, level):
    d = rand_ct(size, level, seed=size * 10 + level)
    b = hecdna.seal_ciphertext_save(d, 2.0**40, MOD, compr=hecdna.COMPR_NONE)
    assert b == sf.ciphertext(d, 2.0**40, MOD)
    got, scale, pid, used = hecdna.seal_ciphertext_load(b + b"trailing")
    assert np.array_equal(got, d) and scale == 2.0**40 and used == len(b)
    assert np.array_equal(pid, sf.parms_id(N, MOD[:level]))


def test_ciphertext_compressed_round_trips(hecdna):
    d = rand_ct(2, 3, seed=5)
    zb = hecdna.seal_ciphertext_save(d, 2.0**41, MOD, compr=hecdna.COMPR_ZLIB)
    assert zb[5] == 1 and int.from_bytes(zb[8:16], "little") == len(zb)
    assert zlib.decompress(zb[16:]) == sf.ciphertext(d, 2.0**41, MOD)[16:]          # members inside the stream
    for b in (zb, sf.ciphertext(d, 2.0**41, MOD, compr=1), hecdna.seal_ciphertext_save(d, 2.0**41, MOD)):
        got, scale, _, used = hecdna.seal_ciphertext_load(b)
        assert np.array_equal(got, d) and scale == 2.0**41 and used == len(b)
    zs = hecdna.seal_ciphertext_save(d, 2.0**41, MOD)                                    # zstd, SEAL's default
    assert zs[5] == 2 and zs[8:16] == len(zs).to_bytes(8, "little") and zs[16:20] == b"\x28\xb5\x2f\xfd"


def test_parms_save_load(hecdna):
    b = hecdna.seal_parms_save(N, MOD)
    assert b == sf.parms(N, MOD)
    assert hecdna.seal_parms_load(b + b"xx") == (N, MOD, len(b))


def test_kswitch_keys_save_load(hecdna):
    K, L = len(MOD), len(MOD) - 1
    rng = np.random.default_rng(9)
    keys = [np.stack([np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in MOD])
                                for _ in range(2)]) for _ in range(L)]) for _ in range(2)]
    lists = [None, keys[0], None, keys[1]]                                  # GaloisKeys indices (elt - 1) / 2
    b = hecdna.seal_kswitch_keys_save(N, MOD, lists)
    assert b == sf.kswitch_keys(N, MOD, lists)
    for idx, k in enumerate(lists):
        words, nl, used = hecdna.seal_kswitch_keys_load(b, idx)
        assert nl == 4 and used == len(b)
        assert (words.size == 0) if k is None else np.array_equal(words, k.ravel())


def test_malformed_and_seeded_inputs_follow_seal(hecdna):
    d = rand_ct(2, 3)
    b = bytes(sf.ciphertext(d, 2.0**40, MOD))
    with pytest.raises(hecdna.InvalidArgument, match="loaded SEALHeader is invalid"):
        hecdna.seal_ciphertext_load(b"\x5e\xa2" + b[2:])
    with pytest.raises(hecdna.InvalidArgument, match="truncated"):
        hecdna.seal_ciphertext_load(b[:100])
    seeded = sf.ciphertext(d, 2.0**40, MOD, seeded_c0_only=True)
    with pytest.raises(hecdna.InvalidArgument, match="seeded ciphertext"):
        hecdna.seal_ciphertext_load(seeded)
