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


def ciphertext(data: np.ndarray, scale, moduli, compr=0, pid=None, seeded_c0_only=False) -> bytes:
    size, level, N = data.shape
    pid = parms_id(N, moduli[:level]) if pid is None else pid
    m = pid.astype(np.uint64).tobytes() + struct.pack("<BQQQdQ", 1, size, N, level, scale, 1)
    m += dynarray(data[0] if seeded_c0_only else data)
    if seeded_c0_only:  # UniformRandomGeneratorInfo: u8 prng type (1 = blake2xb) + 8 x u64 seed
        m += obj(struct.pack("<B", 1) + bytes(64))
    return obj(m, compr)


def parms(N, moduli) -> bytes:
    m = struct.pack("<BQQ", 2, N, len(moduli))
    for q in moduli:
        m += obj(struct.pack("<Q", q))
    m += obj(struct.pack("<Q", 0))
    return obj(m)


def kswitch_keys(N, moduli, lists) -> bytes:
    pid = parms_id(N, moduli)
    m = pid.astype(np.uint64).tobytes() + struct.pack("<Q", len(lists))
    for k in lists:
        if k is None:
            m += struct.pack("<Q", 0)
            continue
        m += struct.pack("<Q", k.shape[0])
        for j in range(k.shape[0]):
            m += obj(ciphertext(k[j], 1.0, moduli, pid=pid))  # PublicKey wrapping its Ciphertext
    return obj(m)
