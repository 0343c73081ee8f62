"""Test helper: a second, independent restatement of SEAL 4.1's serialization layout in pure Python (struct +
hashlib + zlib), used to check the engine's C++ reader/writer (csrc/hec_seal_io.cpp) byte for byte.

    SEALHeader: <HBBBBHQ  magic 0xA15E, header_size 16, version 4.1, compr_mode, reserved, total size
    DynArray:   header, u64 count, words           Modulus: header, u64 value
    Ciphertext: header, parms_id[4], u8 ntt, u64 size, N, coeff_modulus_size, f64 scale, u64 correction, DynArray
    EncryptionParameters: header, u8 scheme (2 = ckks), u64 N, u64 k, k x Modulus, Modulus (plain = 0)
    PublicKey:  header, Ciphertext             KSwitchKeys: header, parms_id, u64 dim1, dim1 x (u64 dim2, PublicKeys)
    parms_id:   BLAKE2b-256 over the u64 words (scheme, N, moduli..., plain modulus)
No SEAL-written bytes exist under /root/reference, so both restatements are parity-unpinned against SEAL."""
import hashlib
import struct
import zlib

import numpy as np

MAGIC = 0xA15E


def header(total, compr=0):
    return struct.pack("<HBBBBHQ", MAGIC, 16, 4, 1, compr, 0, total)


def obj(members: bytes, compr=0) -> bytes:
    body = zlib.compress(members) if compr == 1 else members
    return header(16 + len(body), compr) + body


def parms_id(N, moduli):
    words = np.array([2, N] + list(moduli) + [0], dtype=np.uint64)
    return np.frombuffer(hashlib.blake2b(words.tobytes(), digest_size=32).digest(), dtype=np.uint64)


def dynarray(words: np.ndarray) -> bytes:
    w = np.ascontiguousarray(words, dtype=np.uint64).ravel()
    return obj(struct.pack("<Q", w.size) + w.tobytes())


def ciphertext(data: np.ndarray, scale, moduli, compr=0, pid=None, seeded_c0_only=False, seed=bytes(64),
               prng_type=1) -> bytes:
    size, level, N = data.shape
    pid = parms_id(N, moduli[:level]) if pid is None else pid
    m = pid.astype(np.uint64).tobytes() + struct.pack("<BQQQdQ", 1, size, N, level, scale, 1)
    m += dynarray(data[0] if seeded_c0_only else data)
    if seeded_c0_only:  # UniformRandomGeneratorInfo: u8 prng type (1 = blake2xb) + 8 x u64 seed
        m += obj(struct.pack("<B", prng_type) + seed)
    return obj(m, compr)


def parms(N, moduli) -> bytes:
    m = struct.pack("<BQQ", 2, N, len(moduli))
    for q in moduli:
        m += obj(struct.pack("<Q", q))
    m += obj(struct.pack("<Q", 0))
    return obj(m)


def kswitch_keys(N, moduli, lists, compr=0) -> bytes:
    pid = parms_id(N, moduli)
    m = pid.astype(np.uint64).tobytes() + struct.pack("<Q", len(lists))
    for k in lists:
        if k is None:
            m += struct.pack("<Q", 0)
            continue
        m += struct.pack("<Q", k.shape[0])
        for j in range(k.shape[0]):
            m += obj(ciphertext(k[j], 1.0, moduli, pid=pid))  # PublicKey wrapping its Ciphertext
    return obj(m, compr)


# ---- seeded ciphertexts (Encryptor::encrypt_symmetric(...).save, src/demos/client.cpp:113-114)
# A pure-Python BLAKE2b compression over an explicit parameter block (RFC 7693), BLAKE2Xb on top of it, SEAL
# 4.1's Blake2xbPRNG stream (4096-byte buffers of BLAKE2Xb(counter, key = seed)) and sample_poly_uniform
# (bulk draw, then per-prime rejection redraws from the stream's continuation).  hashlib cannot build BLAKE2Xb's
# leaf nodes (it refuses depth 0), so the compression is restated here and pinned to hashlib where hashlib can
# express the parameter block (sequential, keyed, and the BLAKE2Xb root node).
_IV = [0x6A09E667F3BCC908, 0xBB67AE8584CAA73B, 0x3C6EF372FE94F82B, 0xA54FF53A5F1D36F1,
       0x510E527FADE682D1, 0x9B05688C2B3E6C1F, 0x1F83D9ABFB41BD6B, 0x5BE0CD19137E2179]
_SIGMA = [[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15], [14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3],
          [11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4], [7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8],
          [9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13], [2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9],
          [12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11], [13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10],
          [6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5], [10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0]]
_M64 = (1 << 64) - 1


def _compress(h, block, t, last):
    m = list(struct.unpack("<16Q", block))
    v = h[:] + _IV[:]
    v[12] ^= t & _M64
    v[13] ^= t >> 64
    if last:
        v[14] ^= _M64
    rot = lambda x, n: ((x >> n) | (x << (64 - n))) & _M64

    def g(a, b, c, d, x, y):
        v[a] = (v[a] + v[b] + x) & _M64; v[d] = rot(v[d] ^ v[a], 32)
        v[c] = (v[c] + v[d]) & _M64;     v[b] = rot(v[b] ^ v[c], 24)
        v[a] = (v[a] + v[b] + y) & _M64; v[d] = rot(v[d] ^ v[a], 16)
        v[c] = (v[c] + v[d]) & _M64;     v[b] = rot(v[b] ^ v[c], 63)
    for r in range(12):
        s = _SIGMA[r % 10]
        g(0, 4, 8, 12, m[s[0]], m[s[1]]); g(1, 5, 9, 13, m[s[2]], m[s[3]])
        g(2, 6, 10, 14, m[s[4]], m[s[5]]); g(3, 7, 11, 15, m[s[6]], m[s[7]])
        g(0, 5, 10, 15, m[s[8]], m[s[9]]); g(1, 6, 11, 12, m[s[10]], m[s[11]])
        g(2, 7, 8, 13, m[s[12]], m[s[13]]); g(3, 4, 9, 14, m[s[14]], m[s[15]])
    return [h[i] ^ v[i] ^ v[i + 8] for i in range(8)]


def param_block(digest, key_len=0, fanout=1, depth=1, leaf=0, node_offset=0, xof=0, node_depth=0, inner=0):
    return struct.pack("<BBBBIIIBB14x16x16x", digest, key_len, fanout, depth, leaf, node_offset, xof, node_depth, inner)


def blake2b_param(data: bytes, param: bytes, key: bytes = b"") -> bytes:
    h = [iv ^ w for iv, w in zip(_IV, struct.unpack("<8Q", param))]
    msg = (key + bytes(128 - len(key)) if key else b"") + data
    t = 0
    while len(msg) > 128:
        t += 128
        h = _compress(h, msg[:128], t, False)
        msg = msg[128:]
    t += len(msg)
    h = _compress(h, msg + bytes(128 - len(msg)), t, True)
    return struct.pack("<8Q", *h)[: param[0]]


def blake2xb(data: bytes, key: bytes, outlen: int) -> bytes:
    root = blake2b_param(data, param_block(64, len(key), xof=outlen), key)
    out, i = b"", 0
    while len(out) < outlen:
        bs = min(64, outlen - len(out))
        out += blake2b_param(root, param_block(bs, 0, 0, 0, leaf=64, node_offset=i, xof=outlen, inner=64))
        i += 1
    return out


class Blake2xbStream:
    """SEAL 4.1 Blake2xbPRNG as a byte stream: buffer k = BLAKE2Xb(u64 k, key = seed, 4096 bytes); with
    prng_type 2, Shake256PRNG: buffer k = SHAKE256(seed || u64 k, 4096 bytes) (hashlib)."""

    def __init__(self, seed: bytes, prng_type=1):
        self.seed, self.counter, self.buf, self.type = seed, 0, b"", prng_type

    def take(self, n: int) -> bytes:
        while len(self.buf) < n:
            ctr = struct.pack("<Q", self.counter)
            self.buf += (blake2xb(ctr, self.seed, 4096) if self.type == 1
                         else hashlib.shake_256(self.seed + ctr).digest(4096))
            self.counter += 1
        out, self.buf = self.buf[:n], self.buf[n:]
        return out


def expand_seed_c1(seed: bytes, moduli, N, prng_type=1) -> np.ndarray:
    """Ciphertext::expand_seed for a version-4 object: sample_poly_uniform over moduli -> u64[level][N]."""
    prng = Blake2xbStream(seed, prng_type)
    words = list(struct.unpack("<%dQ" % (len(moduli) * N), prng.take(8 * len(moduli) * N)))
    out = np.zeros((len(moduli), N), dtype=np.uint64)
    for j, q in enumerate(moduli):
        max_multiple = _M64 - _M64 % q - 1
        for i in range(N):
            v = words[j * N + i]
            while v >= max_multiple:
                v = struct.unpack("<Q", prng.take(8))[0]
            out[j, i] = v % q
    return out
