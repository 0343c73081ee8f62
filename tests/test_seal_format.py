"""SEAL 4.1 wire format (client.cpp:113-115, server.cpp:110-122): the engine's C-ABI
reader/writer (csrc/hec_seal_io.cpp) against an independent pure-Python restatement of the layout
(tests/seal_format.py), BLAKE2b against hashlib, and round trips through zlib and zstd.  Host only.
Parity vs SEAL itself is unpinned: no SEAL-written bytes exist under /root/reference."""
import hashlib
import os
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
        hecdna.seal_ciphertext_load(seeded)       # no context moduli: SEAL's load needs the context too


# ---- seeded ciphertexts: Ciphertext::expand_seed (SEAL 4.1 Blake2xbPRNG + sample_poly_uniform)
def test_python_blake2b_param_restatement_matches_hashlib():
    """Pin the test restatement's compression to hashlib wherever hashlib can express the parameter block."""
    for n in (0, 5, 128, 300):
        data = bytes(range(256))[: n % 256] * (1 + n // 256)
        data = data[:n]
        assert sf.blake2b_param(data, sf.param_block(64)) == hashlib.blake2b(data).digest()
        key = bytes(range(64))
        assert sf.blake2b_param(data, sf.param_block(64, 64), key) == hashlib.blake2b(data, key=key).digest()
        root = hashlib.blake2b(data, key=key, fanout=1, depth=1, node_offset=4096 << 32).digest()
        assert sf.blake2b_param(data, sf.param_block(64, 64, xof=4096), key) == root  # the BLAKE2Xb root node


@pytest.mark.parametrize("outlen", [1, 63, 64, 65, 200, 4096])
def test_blake2xb_equals_restatement(hecdna, outlen):
    key = bytes((7 * i + 3) & 0xFF for i in range(64))
    data = (5).to_bytes(8, "little")
    assert hecdna.seal_blake2xb(data, key, outlen) == sf.blake2xb(data, key, outlen)
    # a prefix of a longer XOF output is NOT the shorter output (the length is in every node's parameters)
    if outlen > 8:
        assert hecdna.seal_blake2xb(data, key, outlen)[:8] != hecdna.seal_blake2xb(data, key, 8)


@pytest.mark.parametrize("level,compr", [(1, 0), (3, 1), (4, 2)])
def test_seeded_ciphertext_expands_like_seal(hecdna, level, compr):
    """encrypt_symmetric(...).save writes c0 + seed (client.cpp:113-114); Ciphertext::load expands c1."""
    d = rand_ct(2, level, seed=level)
    seed = np.random.default_rng(100 + level).integers(0, 2**63, 8, dtype=np.uint64).tobytes()
    b = sf.ciphertext(d, 2.0**40, MOD, seeded_c0_only=True, seed=seed, compr=min(compr, 1))  # zstd: round trip
    got, scale, pid, used = hecdna.seal_ciphertext_load(b + b"tail", moduli=MOD)
    assert used == len(b) and scale == 2.0**40 and got.shape == (2, level, N)
    assert np.array_equal(got[0], d[0])
    want = sf.expand_seed_c1(seed, MOD[:level], N)
    assert np.array_equal(got[1], want)
    for j in range(level):
        assert int(got[1][j].max()) < MOD[j]
    # the expanded ciphertext saves as an ordinary (unseeded) object and loads back unchanged
    again, _, _, _ = hecdna.seal_ciphertext_load(hecdna.seal_ciphertext_save(got, 2.0**40, MOD, compr))
    assert np.array_equal(again, got)


def test_seeded_ciphertext_rejections(hecdna):
    d = rand_ct(2, 2)
    seed = bytes(range(64))
    with pytest.raises(hecdna.InvalidArgument, match="ciphertext data is invalid"):       # parms_id of 3 primes
        hecdna.seal_ciphertext_load(sf.ciphertext(d, 1.0, MOD, seeded_c0_only=True, seed=seed,
                                                  pid=sf.parms_id(N, MOD[:3])), moduli=MOD)
    with pytest.raises(hecdna.InvalidArgument, match="ciphertext data is invalid"):       # fewer context primes
        hecdna.seal_ciphertext_load(sf.ciphertext(d, 1.0, MOD, seeded_c0_only=True, seed=seed), moduli=MOD[:1])
    with pytest.raises(hecdna.InvalidArgument, match="prng_type"):                        # prng_type::unknown
        hecdna.seal_ciphertext_load(sf.ciphertext(d, 1.0, MOD, seeded_c0_only=True, seed=seed, prng_type=0),
                                    moduli=MOD)


@pytest.mark.parametrize("n,outlen", [(0, 32), (72, 4096), (135, 136), (136, 137), (300, 500)])
def test_shake256_matches_hashlib(hecdna, n, outlen):
    data = bytes((3 * i + 1) & 0xFF for i in range(n))
    assert hecdna.seal_shake256(data, outlen) == hashlib.shake_256(data).digest(outlen)


def test_seeded_ciphertext_shake256_prng(hecdna):
    d = rand_ct(2, 2, seed=9)
    seed = bytes(range(100, 164))
    got, _, _, _ = hecdna.seal_ciphertext_load(sf.ciphertext(d, 1.0, MOD, seeded_c0_only=True, seed=seed,
                                                             prng_type=2), moduli=MOD)
    assert np.array_equal(got[1], sf.expand_seed_c1(seed, MOD[:2], N, prng_type=2))
    assert np.array_equal(got[0], d[0])


def test_prng_rejection_redraws_from_stream_continuation(hecdna):
    """A word is redrawn with probability ((2^64-1) mod q + 2) / 2^64 — about 2^-40 for SEAL's primes, so the
    redraw path is exercised with a modulus whose remainder is large (q = 3 * 2^61 + 1, about 1 in 4 words):
    redraws come from the stream after the bulk draw, in the C++ loader and the restatement alike."""
    q = 3 * (1 << 61) + 1
    n = 256
    c1 = sf.expand_seed_c1(bytes(64), [q], n)
    words = np.frombuffer(sf.Blake2xbStream(bytes(64)).take(n * 8), dtype=np.uint64)
    rejected = words >= np.uint64(((1 << 64) - 1) - ((1 << 64) - 1) % q - 1)
    assert 20 < int(rejected.sum()) < 120
    keep = ~rejected
    assert np.array_equal(c1[0][keep], words[keep] % np.uint64(q))
    d = np.zeros((2, 1, n), dtype=np.uint64)
    got, _, _, _ = hecdna.seal_ciphertext_load(sf.ciphertext(d, 1.0, [q], seeded_c0_only=True), moduli=[q])
    assert np.array_equal(got[1], c1)


def test_kswitch_keys_one_pass_walk(hecdna):
    """hec_seal_kswitch_keys_foreach: the GaloisKeys shape SEAL writes (N lists, a few non-empty) in one pass, raw
    and zstd-compressed, equal to the per-index reader and to the restated layout."""
    import time
    rng = np.random.default_rng(9)
    lists = [None] * N
    idx = [0, 1, 5, 170, 1023, N - 1]
    for i in idx:
        lists[i] = np.stack([rng.integers(0, MOD[k], (3, 2, N), dtype=np.uint64) for k in range(4)], axis=2)
    for compr in (hecdna.COMPR_NONE, hecdna.COMPR_ZSTD):
        b = hecdna.seal_kswitch_keys_save(N, MOD, lists, compr=compr)
        if compr == hecdna.COMPR_NONE:
            assert b == sf.kswitch_keys(N, MOD, lists)
        t0 = time.perf_counter()
        got, nl, used = hecdna.seal_kswitch_keys_lists(b + b"xyz")
        assert time.perf_counter() - t0 < 10
        assert nl == N and used == len(b) and sorted(got) == idx
        for i in idx:
            assert np.array_equal(got[i], lists[i].reshape(-1))
        w, _, _ = hecdna.seal_kswitch_keys_load(b, 170)
        assert np.array_equal(w, got[170])


def test_truncated_dynarray_is_rejected_before_allocation(hecdna):
    """a ciphertext whose DynArray announces more words than its payload holds (server input is untrusted)"""
    d = rand_ct(2, 1, seed=3)
    b = bytearray(sf.ciphertext(d, 2.0**40, MOD))
    inner = 16 + 32 + 1 + 8 * 4 + 8              # outer header, parms_id, ntt flag, size/N/level/scale, correction
    total = int.from_bytes(b[inner + 8:inner + 16], "little")
    cut = 8 * 100                                  # drop 100 words from the inner object, fix both size fields
    b = b[:len(b) - cut]
    b[inner + 8:inner + 16] = (total - cut).to_bytes(8, "little")
    b[8:16] = len(b).to_bytes(8, "little")
    with pytest.raises(hecdna.InvalidArgument, match="truncated"):
        hecdna.seal_ciphertext_load(bytes(b))


@pytest.mark.parametrize("compr", ["zlib", "zstd"])
def test_key_object_decompression_bomb_is_rejected(hecdna, compr):
    """A small compressed KSwitchKeys payload that inflates past the caller's limit is HEC_EINVAL (the bytes come from
    a client socket, server.cpp:110-122), with no allocation beyond about twice the limit; the same object loads
    under a limit that holds it."""
    lists = [np.zeros((3, 2, 4, N), dtype=np.uint64) for _ in range(8)]   # 3 MiB of zeros: ~1000:1 compressible
    mode = hecdna.COMPR_ZLIB if compr == "zlib" else hecdna.COMPR_ZSTD
    b = hecdna.seal_kswitch_keys_save(N, MOD, lists, compr=mode)
    assert len(b) < 64 * 1024
    for fn in (lambda lim: hecdna.seal_kswitch_keys_lists(b, max_bytes=lim),
               lambda lim: hecdna.seal_kswitch_keys_load(b, 3, max_bytes=lim)):
        with pytest.raises(hecdna.InvalidArgument, match="exceeds the size limit"):
            fn(1 << 20)
    got, nl, used = hecdna.seal_kswitch_keys_lists(b, max_bytes=8 << 20)
    assert nl == 8 and used == len(b) and sorted(got) == list(range(8))


def test_nested_compressed_members_share_the_limit(hecdna):
    """A raw KSwitchKeys object whose PublicKeys are each zlib-compressed: every nested payload draws from the one
    limit of the object, so many small bombs cannot multiply it."""
    pid = sf.parms_id(N, MOD)
    k = np.zeros((2, 4, N), dtype=np.uint64)                    # one PublicKey: 128 KiB of words at N = 2^11
    pk = sf.obj(sf.ciphertext(k, 1.0, MOD, pid=pid), compr=1)   # zlib-compressed PublicKey wrapper
    import struct
    m = pid.astype(np.uint64).tobytes() + struct.pack("<QQ", 1, 16) + pk * 16   # 1 list of 16 digits: 2 MiB inflated
    b = sf.obj(m)
    assert len(b) < 64 * 1024
    with pytest.raises(hecdna.InvalidArgument, match="exceeds the size limit"):
        hecdna.seal_kswitch_keys_lists(b, max_bytes=1 << 20)
    got, nl, _ = hecdna.seal_kswitch_keys_lists(b, max_bytes=4 << 20)
    assert nl == 1 and got[0].size == 16 * 2 * 4 * N


def test_foreach_returns_the_visitors_status(hecdna):
    """hec_seal_kswitch_keys_foreach stops the walk and returns the visitor's status unchanged (hecdna.h)"""
    lists = [np.zeros((1, 2, 4, N), dtype=np.uint64), np.ones((1, 2, 4, N), dtype=np.uint64)]
    b = hecdna.seal_kswitch_keys_save(N, MOD, lists)
    for status in (1, 2, 3, 7):
        with pytest.raises(hecdna.HecError) as e:
            hecdna.seal_kswitch_keys_lists(b, visit_status=status)
        assert e.value.code == status and "rejected by the caller" in str(e.value)


def test_context_free_key_limit_covers_cfg5_galois_keys(hecdna):
    """the context-free key loaders' default decompression limit admits SEAL's default GaloisKeys at the
    cfg5 size (N = 2^16, {60, 40 x 15, 60}: 2 log2 N - 1 = 31 lists of 16 PublicKeys of u64[2][17][N], plus at most
    256 B of metadata per PublicKey and the list-length words), the largest key object BASELINE's configs load."""
    N, K = 1 << 16, 17
    L = K - 1
    lists = 2 * 16 - 1
    cfg5 = lists * L * (2 * K * N * 8 + 256) + N * 8 + 4096
    assert cfg5 > 8.8e9
    limit = hecdna.lib().hec_seal_kswitch_keys_default_limit()
    # also bounded by half the host's available memory (the object is inflated in host memory)
    avail = os.sysconf("SC_AVPHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
    assert limit <= 1 << 34 and limit <= max(avail // 2 * 1.05, 1 << 30)
    if avail // 2 >= 1 << 34:
        assert cfg5 <= limit
