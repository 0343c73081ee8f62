"""hecdna — MI355X-native CKKS homomorphic linear-algebra engine (Python plumbing).

The product is the C-ABI in ``include/hecdna.h`` implemented by ``libhecdna.so`` (HIP kernels for
gfx950, built in-tree by ``make`` in this directory).  This module is a thin ctypes binding of that
C-ABI used by the tests, ``bench.py`` and ``__graft_entry__.py``; it mirrors the reference's
operator surface (``he::operators`` / ``he::linalg``, see cpp/ for the C++ façade) but adds no
computation of its own.  Loading fails loudly when the shared library is missing: there is no CPU
fallback.

Data layout (SEAL layout): ciphertext u64[size][level][N] (NTT form), key u64[L][2][K][N].
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HECDNA_LIB") or os.path.join(_HERE, "libhecdna.so")  # override: experiments
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hecdna.h")

_lib = None
u64p = C.POINTER(C.c_uint64)


HEC_OK, HEC_EINVAL, HEC_ELOGIC, HEC_EDEVICE = 0, 1, 2, 3  # include/hecdna.h status codes


class HecError(Exception):
    """Mirrors SEAL's exception classes: code 1 = invalid_argument, 2 = logic_error, 3 = device."""

    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class InvalidArgument(HecError, ValueError):
    pass


class LogicError(HecError, RuntimeError):
    pass


def build(jobs: int = 8):
    subprocess.check_call(["make", "-s", "-C", _HERE, f"-j{jobs}"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build the HIP engine first (make -C {_HERE})")
        L = C.CDLL(LIB_PATH)
        L.hec_last_error.restype = C.c_char_p
        vp = C.c_void_p
        sig = {
            "hec_context_create": [C.c_uint64, u64p, C.c_uint64, C.c_int, C.POINTER(vp)],
            "hec_context_destroy": [vp],
            "hec_context_set_stream": [vp, vp],
            "hec_context_synchronize": [vp],
            "hec_context_set_option": [vp, C.c_char_p, C.c_int64],
            "hec_ciphertext_create": [vp, C.POINTER(vp)],
            "hec_ciphertext_destroy": [vp],
            "hec_ciphertext_upload": [vp, u64p, C.c_uint64, C.c_uint64, C.c_double],
            "hec_ciphertext_download": [vp, u64p],
            "hec_ciphertext_info": [vp, u64p, u64p, C.POINTER(C.c_double)],
            "hec_ciphertext_copy": [vp, vp],
            "hec_ciphertext_export_device": [vp, vp],
            "hec_ciphertext_import_device": [vp, vp, C.c_uint64, C.c_uint64, C.c_double],
            "hec_ciphertext_reduce": [vp, vp],
            "hec_ciphertext_fill_uniform": [vp, C.c_uint64, C.c_uint64, C.c_double, C.c_uint64],
            "hec_plaintext_create": [vp, C.POINTER(vp)],
            "hec_plaintext_destroy": [vp],
            "hec_plaintext_upload": [vp, u64p, C.c_uint64, C.c_double],
            "hec_kswitch_key_upload": [vp, u64p, C.POINTER(vp)],
            "hec_kswitch_key_fill_uniform": [vp, C.c_uint64, C.POINTER(vp)],
            "hec_kswitch_key_destroy": [vp],
            "hec_kswitch_key_download": [vp, u64p],
            "hec_galois_keys_download": [vp, C.c_uint32, u64p],
            "hec_galois_keys_create": [vp, C.POINTER(vp)],
            "hec_galois_keys_add": [vp, C.c_uint32, u64p],
            "hec_galois_keys_add_uniform": [vp, C.c_uint32, C.c_uint64],
            "hec_galois_keys_destroy": [vp],
            "hec_negate_inplace": [vp, vp],
            "hec_add_inplace": [vp, vp, vp],
            "hec_sub_inplace": [vp, vp, vp],
            "hec_add_plain_inplace": [vp, vp, vp],
            "hec_sub_plain_inplace": [vp, vp, vp],
            "hec_multiply_inplace": [vp, vp, vp],
            "hec_multiply_plain_inplace": [vp, vp, vp],
            "hec_square_inplace": [vp, vp],
            "hec_relinearize_inplace": [vp, vp, vp],
            "hec_rescale_to_next_inplace": [vp, vp],
            "hec_mod_switch_to_next_inplace": [vp, vp],
            "hec_rotate_vector_inplace": [vp, vp, C.c_int, vp],
            "hec_apply_galois_inplace": [vp, vp, C.c_uint32, vp],
            "hec_matmul_diag_col": [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp],
            "hec_matmul_diagpt_col": [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp],
            "hec_plaintext_fill_uniform": [vp, C.c_uint64, C.c_double, C.c_uint64],
            "hec_plaintext_download": [vp, u64p],
            "hec_plaintext_info": [vp, u64p, C.POINTER(C.c_double)],
            "hec_encode": [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_uint64, C.c_uint64, C.c_double,
                           C.c_uint64, vp],
            "hec_encode_scalar": [vp, C.c_double, C.c_double, C.c_uint64, vp],
            "hec_matmul_diag_col_partial": [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64, vp, C.c_uint64, vp, vp],
            "hec_matmul_diag_col_partial_set": [vp, vp, C.c_uint64, vp, C.c_uint64, vp, C.c_uint64, vp, vp],
            "hec_matmul_finish": [vp, vp, C.c_uint64, vp, vp],
            "hec_matmul_col_colT": [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp],
            "hec_matrix_matmul": [vp, vp, C.c_uint64, C.c_uint64, C.c_int, vp, C.c_uint64, C.c_uint64, C.c_int,
                                  vp, vp],
            "hec_ntt_forward": [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64],
            "hec_ntt_inverse": [vp, vp, C.c_uint64, C.c_uint64, C.c_uint64],
            "hec_dyadic_multiply": [vp, vp, vp, vp, C.c_uint64, C.c_uint64, C.c_uint64],
            "hec_device_alloc": [vp, C.c_uint64, C.POINTER(vp)],
            "hec_device_free": [vp, vp],
            "hec_memcpy_h2d": [vp, vp, vp, C.c_uint64],
            "hec_memcpy_d2h": [vp, vp, vp, C.c_uint64],
            "hec_time_ntt_forward": [vp, vp, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_double)],
            "hec_profile_enable": [vp, C.c_int],
            "hec_profile_read": [vp, C.c_char_p, C.POINTER(C.c_double), u64p],
            "hec_profile_read_ex": [vp, C.c_char_p, C.POINTER(C.c_double), u64p, C.POINTER(C.c_double), u64p],
            "hec_profile_classes": [vp, C.c_char_p, C.c_uint64],
            "hec_plan_diagonal_shards": [C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_uint32), C.c_uint64,
                                         C.POINTER(C.c_int32)],
            "hec_comm_unique_id": [vp],
            "hec_comm_init": [vp, C.c_int, C.c_int, vp],
            "hec_comm_init_ops": [vp, C.c_int, C.c_int, vp],
            "hec_shard_agree": [vp, C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_double), C.c_uint64, C.c_char_p,
                                C.c_uint64],
            "hec_context_comm": [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)],
            "hec_matmul_diag_col_sharded": [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp],
            "hec_create_coeff_modulus": [C.c_uint64, C.POINTER(C.c_int), C.c_uint64, u64p],
            "hec_seal_blake2b": [vp, C.c_uint64, C.c_uint64, vp],
            "hec_seal_parms_id": [C.c_uint64, u64p, C.c_uint64, u64p],
            "hec_seal_ciphertext_load": [vp, C.c_uint64, u64p, u64p, u64p, C.POINTER(C.c_double), u64p, u64p,
                                         C.c_uint64, u64p],
            "hec_seal_ciphertext_load_ex": [vp, C.c_uint64, u64p, C.c_uint64, u64p, u64p, u64p,
                                            C.POINTER(C.c_double), u64p, u64p, C.c_uint64, u64p],
            "hec_seal_blake2xb": [vp, C.c_uint64, vp, C.c_uint64, C.c_uint64, vp],
            "hec_seal_shake256": [vp, C.c_uint64, C.c_uint64, vp],
            "hec_seal_ciphertext_save": [u64p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double, u64p, C.c_int, vp,
                                         C.c_uint64, u64p],
            "hec_seal_parms_load": [vp, C.c_uint64, u64p, u64p, C.c_uint64, u64p, u64p],
            "hec_seal_parms_save": [C.c_uint64, u64p, C.c_uint64, C.c_int, vp, C.c_uint64, u64p],
            "hec_seal_kswitch_keys_load": [vp, C.c_uint64, C.c_uint64, u64p, u64p, C.c_uint64, u64p, u64p],
            "hec_seal_kswitch_keys_save": [C.c_uint64, u64p, C.c_uint64, C.POINTER(u64p), u64p, C.c_uint64, C.c_int,
                                           vp, C.c_uint64, u64p],
            "hec_seal_kswitch_keys_foreach": [vp, C.c_uint64, KEYLIST_VISIT, vp, u64p, u64p],
            "hec_seal_kswitch_keys_load_ex": [vp, C.c_uint64, C.c_uint64, C.c_uint64, u64p, u64p, C.c_uint64, u64p,
                                              u64p],
            "hec_seal_kswitch_keys_foreach_ex": [vp, C.c_uint64, C.c_uint64, KEYLIST_VISIT, vp, u64p, u64p],
            "hec_ciphertext_load_seal": [vp, vp, C.c_uint64, u64p],
            "hec_ciphertext_save_seal": [vp, C.c_int, vp, C.c_uint64, u64p],
            "hec_kswitch_key_load_seal": [vp, vp, C.c_uint64, C.POINTER(vp), u64p],
            "hec_galois_keys_load_seal": [vp, vp, C.c_uint64, u64p],
            "hec_galois_keys_load_seal_ex": [vp, vp, C.c_uint64, C.c_uint64, u64p],
        }
        for name, args in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = C.c_int
        L.hec_galois_elt_from_step.argtypes = [vp, C.c_int]
        L.hec_galois_elt_from_step.restype = C.c_uint32
        L.hec_default_galois_elts.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.hec_default_galois_elts.restype = C.c_uint64
        L.hec_galois_keys_has.argtypes = [vp, C.c_uint32]
        L.hec_galois_keys_has.restype = C.c_int
        L.hec_profile_classes.restype = C.c_uint64
        L.hec_seal_last_error.restype = C.c_char_p
        L.hec_seal_kswitch_keys_default_limit.restype = C.c_uint64
        L.hec_galois_keys_load_seal_default_lists.argtypes = [vp]
        L.hec_galois_keys_load_seal_default_lists.restype = C.c_uint64
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        msg = lib().hec_last_error().decode()
        if rc == 1:
            raise InvalidArgument(rc, msg)
        if rc == 2:
            raise LogicError(rc, msg)
        raise HecError(rc, msg)


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u64p)


def exported_symbols():
    """Names declared in include/hecdna.h (for the C-ABI export test)."""
    import re
    txt = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(hec_[a-z0-9_]+)\s*\(", txt)))


def plan_diagonal_shards(N, n, world, key_elts):
    """hec_plan_diagonal_shards (host only): per rank the sorted diagonals it owns."""
    keys = (C.c_uint32 * max(1, len(key_elts)))(*key_elts)
    out = (C.c_int32 * n)()
    _check(lib().hec_plan_diagonal_shards(N, n, world, keys, len(key_elts), out))
    plan = [[] for _ in range(world)]
    for j in range(n):
        plan[out[j]].append(j)
    return plan


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    _check(lib().hec_comm_unique_id(buf))
    return buf.raw


COMM_F64_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_uint64, C.c_int)
COMM_U64_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, u64p, C.c_uint64)
REDUCE_MIN, REDUCE_MAX = 0, 1


class CommOps(C.Structure):
    """include/hecdna.h hec_comm_ops"""
    _fields_ = [("user", C.c_void_p), ("allreduce_f64", COMM_F64_FN), ("allreduce_u64_sum", COMM_U64_FN)]


class HostComm:
    """hec_comm_ops over torch.distributed (a backend with MIN / MAX / SUM on CPU tensors: gloo): the sharded
    matvec's collectives on the host, for hec_comm_init_ops and hec_shard_agree.  Keeps the ctypes callbacks alive."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        def f64(_user, buf, count, op):
            try:
                if count:
                    t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,)))
                    dist.all_reduce(t, op=dist.ReduceOp.MIN if op == REDUCE_MIN else dist.ReduceOp.MAX, group=group)
                return 0
            except Exception:  # noqa: BLE001 - reported to the engine as a failed collective
                return 1

        def u64(_user, buf, count):
            try:
                if count:  # residues < 2^60, world <= 8: the int64 sum is exact and non-negative
                    t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(count,)).view(np.int64))
                    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        self._f64, self._u64 = COMM_F64_FN(f64), COMM_U64_FN(u64)
        self.ops = CommOps(None, self._f64, self._u64)


def shard_agree(comm: HostComm, rank: int, status: int, reason: str, scales) -> tuple[int, str]:
    """hec_shard_agree (host only): the sharded matvec's agreement step -> (agreed status, message)."""
    sc = np.ascontiguousarray(scales, dtype=np.float64)
    msg = C.create_string_buffer(512)
    rc = lib().hec_shard_agree(C.byref(comm.ops), rank, status, reason.encode(),
                               sc.ctypes.data_as(C.POINTER(C.c_double)), len(sc), msg, 512)
    return rc, msg.value.decode()


# ------------------------------------------------------------------ SEAL wire format (host side)
COMPR_NONE, COMPR_ZLIB, COMPR_ZSTD = 0, 1, 2


def _seal_check(rc):
    if rc != 0:
        msg = lib().hec_seal_last_error().decode()
        raise (InvalidArgument if rc == 1 else LogicError)(rc, msg)


def _bytes_in(b: bytes):
    return C.c_char_p(b), len(b)


def _sized_out(fn):
    """Call fn(out, cap, written) twice: size query, then into a buffer of that size."""
    n = C.c_uint64()
    _seal_check(fn(None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value)
    _seal_check(fn(buf, n.value, C.byref(n)))
    return buf.raw[: n.value]


def seal_blake2b(data: bytes, outlen=64) -> bytes:
    out = C.create_string_buffer(outlen)
    _seal_check(lib().hec_seal_blake2b(C.c_char_p(data), len(data), outlen, out))
    return out.raw


def seal_parms_id(N, moduli):
    m = np.ascontiguousarray(np.array(moduli, dtype=np.uint64))
    out = np.zeros(4, dtype=np.uint64)
    _seal_check(lib().hec_seal_parms_id(N, _p(m), len(m), _p(out)))
    return out


def seal_ciphertext_save(data: np.ndarray, scale: float, moduli, compr=COMPR_ZSTD) -> bytes:
    """Ciphertext::save of u64[size][level][N] (parms_id of its level from moduli)."""
    d = np.ascontiguousarray(data, dtype=np.uint64)
    m = np.ascontiguousarray(np.array(moduli, dtype=np.uint64))
    size, level, N = d.shape
    return _sized_out(lambda o, c, w: lib().hec_seal_ciphertext_save(_p(d), size, level, N, scale, _p(m), compr, o, c, w))


def seal_blake2xb(data: bytes, key: bytes, outlen: int) -> bytes:
    """BLAKE2Xb XOF output (SEAL's Blake2xbPRNG core)."""
    out = C.create_string_buffer(outlen)
    _seal_check(lib().hec_seal_blake2xb(C.c_char_p(data), len(data), C.c_char_p(key), len(key), outlen, out))
    return out.raw


def seal_shake256(data: bytes, outlen: int) -> bytes:
    """SHAKE256 XOF output (SEAL's Shake256PRNG core)."""
    out = C.create_string_buffer(outlen)
    _seal_check(lib().hec_seal_shake256(C.c_char_p(data), len(data), outlen, out))
    return out.raw


def seal_ciphertext_load(b: bytes, moduli=None):
    """-> (data u64[size][level][N], scale, parms_id, bytes consumed).  With the context's data-level moduli a
    seeded ciphertext (encrypt_symmetric(...).save) is expanded as Ciphertext::expand_seed does."""
    size, level, N, used = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    scale = C.c_double()
    pid = np.zeros(4, dtype=np.uint64)
    m = None if moduli is None else np.ascontiguousarray(np.array(moduli, dtype=np.uint64))
    mp, mc = (None, 0) if m is None else (_p(m), len(m))
    src, n = _bytes_in(b)
    _seal_check(lib().hec_seal_ciphertext_load_ex(src, n, mp, mc, C.byref(size), C.byref(level), C.byref(N),
                                                  C.byref(scale), _p(pid), None, 0, C.byref(used)))
    d = np.zeros((size.value, level.value, N.value), dtype=np.uint64)
    _seal_check(lib().hec_seal_ciphertext_load_ex(src, n, mp, mc, None, None, None, None, None, _p(d), d.size, None))
    return d, scale.value, pid, used.value


def seal_parms_save(N, moduli, compr=COMPR_NONE) -> bytes:
    m = np.ascontiguousarray(np.array(moduli, dtype=np.uint64))
    return _sized_out(lambda o, c, w: lib().hec_seal_parms_save(N, _p(m), len(m), compr, o, c, w))


def seal_parms_load(b: bytes):
    """EncryptionParameters::load -> (N, moduli, bytes consumed)"""
    N, k, used = C.c_uint64(), C.c_uint64(), C.c_uint64()
    src, n = _bytes_in(b)
    out = np.zeros(64, dtype=np.uint64)
    _seal_check(lib().hec_seal_parms_load(src, n, C.byref(N), _p(out), 64, C.byref(k), C.byref(used)))
    return N.value, [int(x) for x in out[: k.value]], used.value


def seal_kswitch_keys_save(N, moduli, key_lists, compr=COMPR_NONE) -> bytes:
    """KSwitchKeys::save: key_lists[i] = u64[L][2][K][N] or None (an empty list)."""
    m = np.ascontiguousarray(np.array(moduli, dtype=np.uint64))
    keep = [None if k is None else np.ascontiguousarray(k, dtype=np.uint64) for k in key_lists]
    ptrs = (u64p * max(1, len(keep)))(*[(_p(k) if k is not None else u64p()) for k in keep])
    digits = np.array([0 if k is None else k.shape[0] for k in keep] or [0], dtype=np.uint64)
    return _sized_out(lambda o, c, w: lib().hec_seal_kswitch_keys_save(N, _p(m), len(m), ptrs, _p(digits), len(keep),
                                                                     compr, o, c, w))


KEYLIST_VISIT = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, u64p, C.c_uint64)


def seal_kswitch_keys_lists(b: bytes, max_bytes=0, visit_status=0):
    """hec_seal_kswitch_keys_foreach[_ex]: every non-empty key list in one pass -> ({index: u64 words}, list count,
    bytes consumed).  max_bytes bounds the decompressed object (0: the library's default); a non-zero visit_status
    is what the visitor returns for the first list (the walk stops with that status)."""
    got = {}

    def visit(_user, index, words, nwords):
        got[int(index)] = np.ctypeslib.as_array(words, shape=(int(nwords),)).copy()
        return visit_status
    cb = KEYLIST_VISIT(visit)
    lists, used = C.c_uint64(), C.c_uint64()
    src, n = _bytes_in(b)
    rc = lib().hec_seal_kswitch_keys_foreach_ex(src, n, max_bytes, cb, None, C.byref(lists), C.byref(used))
    if rc != 0 and rc == visit_status:
        raise HecError(rc, lib().hec_seal_last_error().decode())
    _seal_check(rc)
    return got, lists.value, used.value


def seal_kswitch_keys_load(b: bytes, index, max_bytes=0):
    """key list `index` as u64 words (u64[L][2][K][N] flattened), and the object's list count"""
    lists, words, used = C.c_uint64(), C.c_uint64(), C.c_uint64()
    src, n = _bytes_in(b)
    _seal_check(lib().hec_seal_kswitch_keys_load_ex(src, n, index, max_bytes, C.byref(lists), None, 0, C.byref(words),
                                                    C.byref(used)))
    out = np.zeros(words.value, dtype=np.uint64)
    _seal_check(lib().hec_seal_kswitch_keys_load_ex(src, n, index, max_bytes, None, _p(out), out.size, None, None))
    return out, lists.value, used.value


def create_coeff_modulus(N, bits):
    out = np.zeros(len(bits), dtype=np.uint64)
    _check(lib().hec_create_coeff_modulus(N, (C.c_int * len(bits))(*bits), len(bits), _p(out)))
    return [int(x) for x in out]


class Context:
    """seal::SEALContext + seal::Evaluator on one GPU (one per process/device)."""

    def __init__(self, N, coeff_modulus, device=0):
        self.N = int(N)
        self.moduli = [int(x) for x in coeff_modulus]
        self.K = len(self.moduli)
        self.L = self.K - 1
        self.device = int(device)
        m = np.array(self.moduli, dtype=np.uint64)
        h = C.c_void_p()
        _check(lib().hec_context_create(self.N, _p(m), self.K, int(device), C.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            lib().hec_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr):
        _check(lib().hec_context_set_stream(self.h, C.c_void_p(stream_ptr) if stream_ptr else None))

    def synchronize(self):
        _check(lib().hec_context_synchronize(self.h))

    def set_option(self, name: str, value: int):
        """hec_context_set_option: an engine knob (lanes, poison, lane_serial, hoist, ...) on the context and its
        batch lanes; every setting computes the same bits."""
        _check(lib().hec_context_set_option(self.h, name.encode(), int(value)))

    def elt_from_step(self, step):
        e = lib().hec_galois_elt_from_step(self.h, int(step))
        if e == 0:
            _check(1)
        return int(e)

    def default_galois_elts(self):
        n = lib().hec_default_galois_elts(self.h, None)
        out = (C.c_uint32 * n)()
        lib().hec_default_galois_elts(self.h, out)
        return list(out)

    # -------------------------------------------------------------- objects
    def ciphertext(self, data=None, scale=1.0):
        ct = Ciphertext(self)
        if data is not None:
            ct.upload(data, scale)
        return ct

    def plaintext(self, data, scale):
        return Plaintext(self, data, scale)

    def encode(self, values, scale, level=None):
        """seal::CKKSEncoder::encode on the GPU (hec_encode): `values` is one slot vector or a 2-D array of
        `count` vectors (real or complex, at most N/2 slots each) -> list of NTT-form Plaintexts (a single
        Plaintext for a 1-D input)."""
        v = np.asarray(values)
        single = v.ndim == 1
        v = v.reshape(1, -1) if single else v
        level = level or (self.K - 1)
        re = np.ascontiguousarray(v.real, dtype=np.float64)
        im = np.ascontiguousarray(v.imag, dtype=np.float64) if np.iscomplexobj(v) else None
        pts = [Plaintext(self, None, scale) for _ in range(v.shape[0])]
        arr = (C.c_void_p * len(pts))(*[p.h.value for p in pts])
        dp = C.POINTER(C.c_double)
        _check(lib().hec_encode(self.h, re.ctypes.data_as(dp), im.ctypes.data_as(dp) if im is not None else None,
                                v.shape[1], v.shape[0], float(scale), level, arr))
        return pts[0] if single else pts

    def encode_scalar(self, value, scale, level=None):
        """seal::CKKSEncoder::encode(double value, parms_id, scale, pt) (hec_encode_scalar): the constant plaintext
        he::util::drop_chain_levels and he::math multiply by (he_util.h:33)"""
        level = level or (self.K - 1)
        pt = Plaintext(self, None, scale)
        _check(lib().hec_encode_scalar(self.h, float(value), float(scale), level, pt.h))
        return pt

    def relin_key(self, data=None, seed=None):
        return KSwitchKey(self, data, seed)

    def galois_keys(self, keys: dict | None = None, uniform_elts=None, seed=0):
        g = GaloisKeys(self)
        for e, d in (keys or {}).items():
            g.add(e, d)
        for i, e in enumerate(uniform_elts or []):
            g.add_uniform(e, seed + 7919 * i)
        return g

    # -------------------------------------------------------------- evaluator (in place)
    def negate(self, a):
        _check(lib().hec_negate_inplace(self.h, a.h)); return a

    def add(self, a, b):
        _check(lib().hec_add_inplace(self.h, a.h, b.h)); return a

    def sub(self, a, b):
        _check(lib().hec_sub_inplace(self.h, a.h, b.h)); return a

    def add_plain(self, a, p):
        _check(lib().hec_add_plain_inplace(self.h, a.h, p.h)); return a

    def sub_plain(self, a, p):
        _check(lib().hec_sub_plain_inplace(self.h, a.h, p.h)); return a

    def multiply(self, a, b):
        _check(lib().hec_multiply_inplace(self.h, a.h, b.h)); return a

    def multiply_plain(self, a, p):
        _check(lib().hec_multiply_plain_inplace(self.h, a.h, p.h)); return a

    def square(self, a):
        _check(lib().hec_square_inplace(self.h, a.h)); return a

    def relinearize(self, a, rk):
        _check(lib().hec_relinearize_inplace(self.h, a.h, rk.h)); return a

    def rescale_to_next(self, a):
        _check(lib().hec_rescale_to_next_inplace(self.h, a.h)); return a

    def mod_switch_to_next(self, a):
        _check(lib().hec_mod_switch_to_next_inplace(self.h, a.h)); return a

    def rotate_vector(self, a, steps, gk):
        _check(lib().hec_rotate_vector_inplace(self.h, a.h, int(steps), gk.h)); return a

    def apply_galois(self, a, elt, gk):
        _check(lib().hec_apply_galois_inplace(self.h, a.h, int(elt), gk.h)); return a

    # -------------------------------------------------------------- linalg
    @staticmethod
    def _arr(cts):
        # None entries pass a null handle (diagonals a sharded rank does not hold; never dereferenced)
        return (C.c_void_p * len(cts))(*[(c.h if c is not None else None) for c in cts])

    def matmul_diag_col(self, diags, cols, rk, gk, out=None):
        out = out or [Ciphertext(self) for _ in cols]
        _check(lib().hec_matmul_diag_col(self.h, self._arr(diags), len(diags), self._arr(cols), len(cols), rk.h,
                                         gk.h, self._arr(out)))
        return out

    def comm_init(self, rank, world, unique_id: bytes | None = None):
        buf = C.create_string_buffer(unique_id, 128) if unique_id is not None else None
        _check(lib().hec_comm_init(self.h, rank, world, buf))

    def comm_init_ops(self, rank, world, comm: HostComm):
        """hec_comm_init_ops: the sharded matvec over the caller's host collectives (e.g. gloo)."""
        self._host_comm = comm  # the engine keeps the callbacks
        _check(lib().hec_comm_init_ops(self.h, rank, world, C.byref(comm.ops)))

    def matmul_diag_col_sharded(self, diags, cols, rk, gk, out=None):
        """hec_matmul_diag_col_sharded: every rank calls it; returns all p outputs on every rank."""
        out = out or [Ciphertext(self) for _ in cols]
        _check(lib().hec_matmul_diag_col_sharded(self.h, self._arr(diags), len(diags), self._arr(cols), len(cols),
                                                 rk.h, gk.h, self._arr(out)))
        return out

    def matmul_diagpt_col(self, pdiags, cols, gk, out=None):
        """ct x pt matvec: plaintext diagonals (multiply_plain), one rescale per output, no relin."""
        out = out or [Ciphertext(self) for _ in cols]
        _check(lib().hec_matmul_diagpt_col(self.h, self._arr(pdiags), len(pdiags), self._arr(cols), len(cols), gk.h,
                                           self._arr(out)))
        return out

    def matmul_diag_col_partial(self, diags, j_begin, j_end, cols, gk, out=None):
        out = out or [Ciphertext(self) for _ in cols]
        _check(lib().hec_matmul_diag_col_partial(self.h, self._arr(diags), len(diags), j_begin, j_end,
                                                 self._arr(cols), len(cols), gk.h, self._arr(out)))
        return out

    def matmul_diag_col_partial_set(self, diags, js, cols, gk, out=None):
        out = out or [Ciphertext(self) for _ in cols]
        idx = np.ascontiguousarray(js, dtype=np.uint64)
        _check(lib().hec_matmul_diag_col_partial_set(self.h, self._arr(diags), len(diags), _p(idx), len(idx),
                                                     self._arr(cols), len(cols), gk.h, self._arr(out)))
        return out

    def matmul_finish(self, accs, rk, out=None):
        out = out or [Ciphertext(self) for _ in accs]
        _check(lib().hec_matmul_finish(self.h, self._arr(accs), len(accs), rk.h, self._arr(out)))
        return out

    def reduce(self, ct):
        """Reduce every word of ct mod its prime (after a partial-sum exchange)."""
        _check(lib().hec_ciphertext_reduce(self.h, ct.h)); return ct

    def matmul_col_colT(self, A, B, p, rk, gk):
        out = [Ciphertext(self) for _ in range(p)]
        _check(lib().hec_matmul_col_colT(self.h, self._arr(A), len(A), self._arr(B), p, rk.h, gk.h,
                                         self._arr(out)))
        return out

    def matrix_matmul(self, A, ar, ac, atr, B, br, bc, btr, rk):
        r1 = ac if atr else ar
        c2 = br if btr else bc
        out = [Ciphertext(self) for _ in range(r1 * c2)]
        _check(lib().hec_matrix_matmul(self.h, self._arr(A), ar, ac, int(atr), self._arr(B), br, bc, int(btr),
                                       rk.h, self._arr(out)))
        return out

    # -------------------------------------------------------------- primitives
    def ntt(self, host: np.ndarray, limb0=0, inverse=False):
        """host u64[npolys][nlimbs][N] -> transformed copy (device round trip)."""
        a = np.ascontiguousarray(host, dtype=np.uint64)
        npolys, nl = (a.shape[0], a.shape[1]) if a.ndim == 3 else (1, a.shape[0])
        buf = DeviceBuffer(self, a.nbytes)
        buf.upload(a)
        fn = lib().hec_ntt_inverse if inverse else lib().hec_ntt_forward
        _check(fn(self.h, buf.p, limb0, nl, npolys))
        return buf.download(a.shape)

    def ntt_device(self, buf, nl, npolys, limb0=0, inverse=False):
        """in place on device words u64[npolys][nl][N] (hec_ntt_forward / hec_ntt_inverse, stream ordered)"""
        fn = lib().hec_ntt_inverse if inverse else lib().hec_ntt_forward
        _check(fn(self.h, buf.p, limb0, nl, npolys))

    def dyadic_device(self, a, b, out, nl, npolys, limb0=0):
        """out = a (*) b on device words u64[npolys][nl][N] (hec_dyadic_multiply, stream ordered)"""
        _check(lib().hec_dyadic_multiply(self.h, a.p, b.p, out.p, limb0, nl, npolys))

    def dyadic_multiply(self, a: np.ndarray, b: np.ndarray, limb0=0):
        """a, b host u64[npolys][nlimbs][N] -> (a * b) mod q_(limb0 + limb) (device round trip)."""
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        if a.shape != b.shape or a.ndim != 3:
            raise InvalidArgument(1, "operands must have the same shape u64[npolys][nlimbs][N]")
        bufs = [DeviceBuffer(self, a.nbytes) for _ in range(3)]
        bufs[0].upload(a)
        bufs[1].upload(b)
        _check(lib().hec_dyadic_multiply(self.h, bufs[0].p, bufs[1].p, bufs[2].p, limb0, a.shape[1], a.shape[0]))
        return bufs[2].download(a.shape)

    def profile(self, mode=1):
        """0 off, 1 synchronous per phase, 2 asynchronous event pairs (resolved by profile_read)."""
        _check(lib().hec_profile_enable(self.h, int(mode)))

    def profile_read(self, cls):
        ms = C.c_double()
        n = C.c_uint64()
        _check(lib().hec_profile_read(self.h, cls.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def profile_read_ex(self, cls):
        """(ms, scopes, algorithmic bytes, kernel launches) of one profile class."""
        ms, n, b, kl = C.c_double(), C.c_uint64(), C.c_double(), C.c_uint64()
        _check(lib().hec_profile_read_ex(self.h, cls.encode(), C.byref(ms), C.byref(n), C.byref(b), C.byref(kl)))
        return ms.value, n.value, b.value, kl.value

    def profile_classes(self):
        need = lib().hec_profile_classes(self.h, None, 0)
        buf = C.create_string_buffer(int(need))
        lib().hec_profile_classes(self.h, buf, need)
        return [x for x in buf.value.decode().split("\n") if x]


class DeviceBuffer:
    def __init__(self, ctx: Context, nbytes):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _check(lib().hec_device_alloc(ctx.h, self.nbytes, C.byref(p)))
        self.p = p

    def upload(self, a):
        a = np.ascontiguousarray(a)
        _check(lib().hec_memcpy_h2d(self.ctx.h, self.p, a.ctypes.data_as(C.c_void_p), a.nbytes))

    def download(self, shape, dtype=np.uint64):
        out = np.empty(shape, dtype=dtype)
        _check(lib().hec_memcpy_d2h(self.ctx.h, out.ctypes.data_as(C.c_void_p), self.p, out.nbytes))
        return out

    def __del__(self):
        try:
            if self.p:
                lib().hec_device_free(self.ctx.h, self.p)
                self.p = None
        except Exception:
            pass


class Ciphertext:
    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        _check(lib().hec_ciphertext_create(ctx.h, C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().hec_ciphertext_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def upload(self, data: np.ndarray, scale: float):
        a = np.ascontiguousarray(data, dtype=np.uint64)
        _check(lib().hec_ciphertext_upload(self.h, _p(a), a.shape[0], a.shape[1], float(scale)))
        return self

    def fill_uniform(self, size, level, scale, seed):
        _check(lib().hec_ciphertext_fill_uniform(self.h, size, level, float(scale), seed))
        return self

    def info(self):
        s, l, sc = C.c_uint64(), C.c_uint64(), C.c_double()
        _check(lib().hec_ciphertext_info(self.h, C.byref(s), C.byref(l), C.byref(sc)))
        return s.value, l.value, sc.value

    @property
    def scale(self):
        return self.info()[2]

    def download(self):
        s, l, _ = self.info()
        out = np.empty((s, l, self.ctx.N), dtype=np.uint64)
        _check(lib().hec_ciphertext_download(self.h, _p(out)))
        return out

    def export_device(self, dev_ptr):
        """Copy the u64[size][level][N] words into device memory at dev_ptr (stream ordered)."""
        _check(lib().hec_ciphertext_export_device(self.h, C.c_void_p(dev_ptr)))

    def import_device(self, dev_ptr, size, level, scale):
        _check(lib().hec_ciphertext_import_device(self.h, C.c_void_p(dev_ptr), size, level, float(scale)))
        return self

    def copy(self):
        c = Ciphertext(self.ctx)
        _check(lib().hec_ciphertext_copy(c.h, self.h))
        return c

    def load_seal(self, b: bytes):
        """Ciphertext::load(context, in, size) from SEAL's wire format; returns the bytes read."""
        used = C.c_uint64()
        _check(lib().hec_ciphertext_load_seal(self.h, C.c_char_p(b), len(b), C.byref(used)))
        return used.value

    def save_seal(self, compr=COMPR_ZSTD) -> bytes:
        """Ciphertext::save(stream, compr_mode) in SEAL's wire format."""
        n = C.c_uint64()
        _check(lib().hec_ciphertext_save_seal(self.h, compr, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().hec_ciphertext_save_seal(self.h, compr, buf, n.value, C.byref(n)))
        return buf.raw[: n.value]


class Plaintext:
    def __init__(self, ctx: Context, data, scale):
        self.ctx = ctx
        h = C.c_void_p()
        _check(lib().hec_plaintext_create(ctx.h, C.byref(h)))
        self.h = h
        if data is not None:
            a = np.ascontiguousarray(data, dtype=np.uint64)
            _check(lib().hec_plaintext_upload(self.h, _p(a), a.shape[0], float(scale)))

    def fill_uniform(self, level, scale, seed):
        _check(lib().hec_plaintext_fill_uniform(self.h, level, float(scale), seed))
        return self

    def info(self):
        lv, sc = C.c_uint64(), C.c_double()
        _check(lib().hec_plaintext_info(self.h, C.byref(lv), C.byref(sc)))
        return lv.value, sc.value

    def download(self):
        lv, _ = self.info()
        out = np.empty((lv, self.ctx.N), dtype=np.uint64)
        _check(lib().hec_plaintext_download(self.h, _p(out)))
        return out

    def __del__(self):
        try:
            if self.h:
                lib().hec_plaintext_destroy(self.h)
                self.h = None
        except Exception:
            pass


class KSwitchKey:
    def __init__(self, ctx: Context, data=None, seed=None, seal_bytes: bytes | None = None):
        self.ctx = ctx
        h = C.c_void_p()
        if seal_bytes is not None:  # RelinKeys::load(context, in, size)
            used = C.c_uint64()
            _check(lib().hec_kswitch_key_load_seal(ctx.h, C.c_char_p(seal_bytes), len(seal_bytes), C.byref(h),
                                                   C.byref(used)))
        elif data is not None:
            a = np.ascontiguousarray(data, dtype=np.uint64)
            _check(lib().hec_kswitch_key_upload(ctx.h, _p(a), C.byref(h)))
        else:
            _check(lib().hec_kswitch_key_fill_uniform(ctx.h, int(seed or 0), C.byref(h)))
        self.h = h

    def download(self):
        """u64[L][2][K][N] (hec_kswitch_key_download)"""
        c = self.ctx
        a = np.empty((c.L, 2, c.K, c.N), dtype=np.uint64)
        _check(lib().hec_kswitch_key_download(self.h, _p(a)))
        return a

    def __del__(self):
        try:
            if self.h:
                lib().hec_kswitch_key_destroy(self.h)
                self.h = None
        except Exception:
            pass


class GaloisKeys:
    def __init__(self, ctx: Context):
        self.ctx = ctx
        h = C.c_void_p()
        _check(lib().hec_galois_keys_create(ctx.h, C.byref(h)))
        self.h = h

    def add(self, elt, data):
        a = np.ascontiguousarray(data, dtype=np.uint64)
        _check(lib().hec_galois_keys_add(self.h, int(elt), _p(a)))

    def add_uniform(self, elt, seed):
        _check(lib().hec_galois_keys_add_uniform(self.h, int(elt), int(seed)))

    def has(self, elt):
        return bool(lib().hec_galois_keys_has(self.h, int(elt)))

    def download(self, elt):
        """the key of one Galois element, u64[L][2][K][N] (hec_galois_keys_download)"""
        c = self.ctx
        a = np.empty((c.L, 2, c.K, c.N), dtype=np.uint64)
        _check(lib().hec_galois_keys_download(self.h, int(elt), _p(a)))
        return a

    def load_seal(self, b: bytes, max_lists=None):
        """GaloisKeys::load(context, in, size): every key list of a SEAL-serialized GaloisKeys (at most max_lists
        non-empty lists; None: the library's fixed default, hec_galois_keys_load_seal_default_lists)."""
        used = C.c_uint64()
        if max_lists is None:
            _check(lib().hec_galois_keys_load_seal(self.h, C.c_char_p(b), len(b), C.byref(used)))
        else:
            _check(lib().hec_galois_keys_load_seal_ex(self.h, C.c_char_p(b), len(b), int(max_lists), C.byref(used)))
        return used.value

    def __del__(self):
        try:
            if self.h:
                lib().hec_galois_keys_destroy(self.h)
                self.h = None
        except Exception:
            pass
