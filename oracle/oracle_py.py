"""ORACLE Python binding — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/_build/liboracle.so (the CPU restatement of SEAL 4.1 semantics for the
reference's he_linalg / he_operators hot path; see oracle/oracle.hpp for what each call restates and
for the parity status: parity vs SEAL is UNPINNED).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# HEC_ORACLE_LIB: another build of the same sources (bench.py's cpu_baseline uses a -march=native build)
_LIB_PATH = os.environ.get("HEC_ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

u64p = C.POINTER(C.c_uint64)


class OrcCt(C.Structure):
    _fields_ = [("data", u64p), ("size", C.c_uint64), ("level", C.c_uint64), ("scale", C.c_double)]


class OracleError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code  # 1 invalid_argument, 2 logic_error, 3 other


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_last_error.restype = C.c_char_p
        L.orc_ctx_new.restype = C.c_void_p
        L.orc_ctx_new.argtypes = [C.c_uint64, C.c_uint64, u64p]
        L.orc_ctx_free.argtypes = [C.c_void_p]
        L.orc_ntt_root.restype = C.c_uint64
        L.orc_ntt_root.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_barrett128.restype = C.c_uint64
        L.orc_barrett128.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.orc_is_prime.argtypes = [C.c_uint64]
        L.orc_elt_from_step.restype = C.c_uint32
        L.orc_elt_from_step.argtypes = [C.c_void_p, C.c_int]
        L.orc_default_galois_elts.restype = C.c_uint64
        L.orc_naf.restype = C.c_uint64
        for name in ("orc_ntt_fwd", "orc_ntt_inv"):
            getattr(L, name).argtypes = [C.c_void_p, C.c_uint64, u64p]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u64p)


def _check(rc):
    if rc != 0:
        raise OracleError(rc, lib().orc_last_error().decode())


@dataclass
class Ct:
    """Ciphertext in SEAL layout: data u64[size][level][N] (NTT form) + scale."""
    data: np.ndarray
    scale: float

    @property
    def size(self):
        return self.data.shape[0]

    @property
    def level(self):
        return self.data.shape[1]

    def copy(self):
        return Ct(self.data.copy(), self.scale)


class Oracle:
    def __init__(self, N: int, moduli):
        self.N = int(N)
        self.moduli = np.ascontiguousarray(np.array(moduli, dtype=np.uint64))
        self.K = len(self.moduli)
        self.L = self.K - 1
        self._h = lib().orc_ctx_new(self.N, self.K, _p(self.moduli))
        if not self._h:
            raise OracleError(1, lib().orc_last_error().decode())
        self._keep = []

    def __del__(self):
        try:
            if self._h:
                lib().orc_ctx_free(C.c_void_p(self._h))
        except Exception:
            pass

    @property
    def h(self):
        return C.c_void_p(self._h)

    # ------------------------------------------------------------------ params / NTT ----------
    @staticmethod
    def create_coeff_modulus(N, bits):
        out = np.zeros(len(bits), dtype=np.uint64)
        arr = (C.c_int * len(bits))(*bits)
        _check(lib().orc_create_coeff_modulus(C.c_uint64(N), C.c_uint64(len(bits)), arr, _p(out)))
        return [int(x) for x in out]

    @staticmethod
    def barrett128(lo, hi, q):
        return int(lib().orc_barrett128(lo, hi, q))

    def root(self, i):
        return int(lib().orc_ntt_root(self.h, i))

    def ntt_fwd(self, i, a):
        a = np.ascontiguousarray(a, dtype=np.uint64).copy()
        lib().orc_ntt_fwd(self.h, i, _p(a))
        return a

    def ntt_inv(self, i, a):
        a = np.ascontiguousarray(a, dtype=np.uint64).copy()
        lib().orc_ntt_inv(self.h, i, _p(a))
        return a

    def elt_from_step(self, step):
        e = lib().orc_elt_from_step(self.h, int(step))
        if e == 0:
            raise OracleError(1, lib().orc_last_error().decode())
        return int(e)

    def default_galois_elts(self):
        n = lib().orc_default_galois_elts(self.h, None)
        out = (C.c_uint32 * n)()
        lib().orc_default_galois_elts(self.h, out)
        return list(out)

    @staticmethod
    def naf(v):
        out = (C.c_int * 40)()
        n = lib().orc_naf(int(v), out)
        return list(out[:n])

    def apply_galois_ntt(self, a, elt):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        out = np.empty_like(a)
        nl = a.size // self.N
        lib().orc_apply_galois_ntt(self.h, _p(a), C.c_uint64(nl), C.c_uint32(elt), _p(out))
        return out

    # ------------------------------------------------------------------ keys / encode ---------
    def secret_key(self, seed):
        out = np.zeros((self.K, self.N), dtype=np.uint64)
        _check(lib().orc_secret_key(self.h, C.c_uint64(seed), _p(out)))
        return out

    def key_shape(self):
        return (self.L, 2, self.K, self.N)

    def relin_key(self, sk, seed):
        out = np.zeros(self.key_shape(), dtype=np.uint64)
        _check(lib().orc_relin_key(self.h, _p(sk), C.c_uint64(seed), _p(out)))
        return out

    def galois_key(self, sk, elt, seed):
        out = np.zeros(self.key_shape(), dtype=np.uint64)
        _check(lib().orc_galois_key(self.h, _p(sk), C.c_uint32(elt), C.c_uint64(seed), _p(out)))
        return out

    def galois_keys(self, sk, elts, seed):
        return {int(e): self.galois_key(sk, e, seed + 7919 * i) for i, e in enumerate(elts)}

    def encode(self, values, scale, level):
        v = np.asarray(values)
        re = np.ascontiguousarray(v.real, dtype=np.float64)
        im = np.ascontiguousarray(v.imag if np.iscomplexobj(v) else np.zeros_like(re), dtype=np.float64)
        out = np.zeros((level, self.N), dtype=np.uint64)
        dp = C.POINTER(C.c_double)
        _check(lib().orc_encode(self.h, re.ctypes.data_as(dp), im.ctypes.data_as(dp), C.c_uint64(len(re)),
                                C.c_double(scale), C.c_uint64(level), _p(out)))
        return out

    def encode_scalar(self, value, scale, level):
        """CKKSEncoder::encode(double, parms_id, scale, pt): u64[level][N], every word of limb j the residue"""
        out = np.zeros((level, self.N), dtype=np.uint64)
        _check(lib().orc_encode_scalar(self.h, C.c_double(value), C.c_double(scale), C.c_uint64(level), _p(out)))
        return out

    def decode(self, pt, scale):
        pt = np.ascontiguousarray(pt, dtype=np.uint64)
        re = np.zeros(self.N // 2)
        im = np.zeros(self.N // 2)
        dp = C.POINTER(C.c_double)
        _check(lib().orc_decode(self.h, _p(pt), C.c_uint64(pt.shape[0]), C.c_double(scale),
                                re.ctypes.data_as(dp), im.ctypes.data_as(dp)))
        return re + 1j * im

    def encrypt(self, sk, pt, scale, seed):
        level = pt.shape[0]
        out = np.zeros((2, level, self.N), dtype=np.uint64)
        _check(lib().orc_encrypt(self.h, _p(sk), _p(np.ascontiguousarray(pt)), C.c_uint64(level),
                                 C.c_double(scale), C.c_uint64(seed), _p(out)))
        return Ct(out, float(scale))

    def encrypt_many(self, sk, values, scale, level, seed0, nthreads=8):
        """encode + encrypt each row of `values` (real slot vectors); row v uses seed0 + v (threaded)."""
        v = np.ascontiguousarray(values, dtype=np.float64)
        out = np.zeros((v.shape[0], 2, level, self.N), dtype=np.uint64)
        _check(lib().orc_encrypt_many(self.h, _p(sk), v.ctypes.data_as(C.POINTER(C.c_double)), C.c_uint64(v.shape[1]),
                                      C.c_uint64(v.shape[0]), C.c_double(scale), C.c_uint64(level), C.c_uint64(seed0),
                                      C.c_int(nthreads), _p(out)))
        return out

    def decrypt(self, sk, ct: Ct):
        out = np.zeros((ct.level, self.N), dtype=np.uint64)
        s = self._in(ct)
        _check(lib().orc_decrypt(self.h, _p(sk), C.byref(s), _p(out)))
        return out

    # ------------------------------------------------------------------ evaluator -------------
    def _in(self, ct: Ct, cap_size=None):
        buf = np.zeros(((cap_size or max(ct.size, 3)) * ct.level * self.N,), dtype=np.uint64)
        buf[: ct.data.size] = ct.data.ravel()
        self._keep.append(buf)
        return OrcCt(_p(buf), ct.size, ct.level, ct.scale)

    def _out(self, s: OrcCt):
        n = s.size * s.level * self.N
        arr = np.ctypeslib.as_array(s.data, shape=(n,)).copy().reshape(s.size, s.level, self.N)
        self._keep.clear()
        return Ct(arr, s.scale)

    def _unary(self, fn, a):
        s = self._in(a)
        _check(getattr(lib(), fn)(self.h, C.byref(s)))
        return self._out(s)

    def _binary(self, fn, a, b):
        s, t = self._in(a, a.size + b.size), self._in(b)
        _check(getattr(lib(), fn)(self.h, C.byref(s), C.byref(t)))
        return self._out(s)

    def negate(self, a):
        return self._unary("orc_negate", a)

    def square(self, a):
        return self._unary("orc_square", a)

    def rescale(self, a):
        return self._unary("orc_rescale", a)

    def mod_switch(self, a):
        return self._unary("orc_mod_switch", a)

    def add(self, a, b):
        return self._binary("orc_add", a, b)

    def sub(self, a, b):
        return self._binary("orc_sub", a, b)

    def multiply(self, a, b):
        return self._binary("orc_multiply", a, b)

    def _plain(self, fn, a, pt, scale):
        s = self._in(a)
        pt = np.ascontiguousarray(pt, dtype=np.uint64)
        _check(getattr(lib(), fn)(self.h, C.byref(s), _p(pt), C.c_uint64(pt.shape[0]), C.c_double(scale)))
        return self._out(s)

    def add_plain(self, a, pt, scale):
        return self._plain("orc_add_plain", a, pt, scale)

    def sub_plain(self, a, pt, scale):
        return self._plain("orc_sub_plain", a, pt, scale)

    def multiply_plain(self, a, pt, scale):
        return self._plain("orc_multiply_plain", a, pt, scale)

    def relinearize(self, a, rk):
        s = self._in(a)
        _check(lib().orc_relinearize(self.h, C.byref(s), _p(rk)))
        return self._out(s)

    def switch_key(self, a, target, key):
        s = self._in(a)
        _check(lib().orc_switch_key(self.h, C.byref(s), _p(np.ascontiguousarray(target)), _p(key)))
        return self._out(s)

    def _gk(self, gk: dict):
        elts = (C.c_uint32 * len(gk))(*gk.keys())
        ptrs = (u64p * len(gk))(*[_p(v) for v in gk.values()])
        return elts, ptrs, C.c_uint64(len(gk))

    def apply_galois(self, a, elt, gk):
        s = self._in(a)
        _check(lib().orc_apply_galois(self.h, C.byref(s), C.c_uint32(elt), *self._gk(gk)))
        return self._out(s)

    def rotate(self, a, steps, gk):
        s = self._in(a)
        _check(lib().orc_rotate(self.h, C.byref(s), C.c_int(steps), *self._gk(gk)))
        return self._out(s)

    def sum_elems(self, a, dim, gk):
        """BatchedVector::sum_elems_inplace (he_linalg.cpp:667-713)."""
        s = self._in(a)
        _check(lib().orc_sum_elems(self.h, C.byref(s), C.c_uint64(dim), *self._gk(gk)))
        return self._out(s)

    # ------------------------------------------------------------------ linalg ----------------
    def _many(self, cts, cap=3):
        arr = (OrcCt * len(cts))()
        bufs = []
        for i, c in enumerate(cts):
            buf = np.zeros((max(cap, c.size) * c.level * self.N,), dtype=np.uint64)
            buf[: c.data.size] = c.data.ravel()
            bufs.append(buf)
            arr[i] = OrcCt(_p(buf), c.size, c.level, c.scale)
        return arr, bufs

    def _outs(self, arr, n):
        res = []
        for i in range(n):
            s = arr[i]
            m = s.size * s.level * self.N
            res.append(Ct(np.ctypeslib.as_array(s.data, shape=(m,)).copy().reshape(s.size, s.level, self.N),
                          s.scale))
        return res

    def matmul_diag_col(self, A, X, rk, gk, nthreads=1, j_begin=0, j_end=None, finish=True):
        a, ab = self._many(A)
        x, xb = self._many(X)
        lvl = X[0].level
        outs, ob = self._many([Ct(np.zeros((3, lvl, self.N), np.uint64), 1.0) for _ in X])
        _check(lib().orc_matmul_diag_col(self.h, a, C.c_uint64(len(A)), x, C.c_uint64(len(X)), _p(rk),
                                         *self._gk(gk), outs, C.c_int(nthreads), C.c_uint64(j_begin),
                                         C.c_uint64(len(A) if j_end is None else j_end), C.c_int(int(finish))))
        return self._outs(outs, len(X))

    def matmul_diag_col_set(self, A, js, X, rk, gk, nthreads=1, finish=False):
        """he_linalg.cpp:977-997 restricted to the diagonals js (A[k] is diagonal js[k])."""
        a, ab = self._many(A)
        x, xb = self._many(X)
        jj = np.ascontiguousarray(np.array(js, dtype=np.uint64))
        lvl = X[0].level
        outs, ob = self._many([Ct(np.zeros((3, lvl, self.N), np.uint64), 1.0) for _ in X])
        _check(lib().orc_matmul_diag_col_set(self.h, a, _p(jj), C.c_uint64(len(js)), x, C.c_uint64(len(X)), _p(rk),
                                             *self._gk(gk), outs, C.c_int(nthreads), C.c_int(int(finish))))
        return self._outs(outs, len(X))

    def matmul_diagpt_col_set(self, P, pscale, js, X, gk, nthreads=1, finish=True):
        """ct x pt form over the diagonals js: P[k] (u64[level][N] NTT-form plaintext at scale pscale) is diagonal
        js[k]; out[i] = rescale(sum_k multiply_plain(rot(X[i], js[k]), P[k])) (rescale only when finish)."""
        pts = np.ascontiguousarray(np.stack([np.asarray(q, dtype=np.uint64) for q in P]))
        x, xb = self._many(X)
        jj = np.ascontiguousarray(np.array(js, dtype=np.uint64))
        lvl = X[0].level
        outs, ob = self._many([Ct(np.zeros((2, lvl, self.N), np.uint64), 1.0) for _ in X])
        _check(lib().orc_matmul_diagpt_col_set(self.h, _p(pts), C.c_uint64(pts.shape[1]), C.c_double(pscale), _p(jj),
                                               C.c_uint64(len(js)), x, C.c_uint64(len(X)), *self._gk(gk), outs,
                                               C.c_int(nthreads), C.c_int(int(finish))))
        return self._outs(outs, len(X))

    def _views(self, cts):
        """OrcCt records pointing at the callers' own C-contiguous u64 arrays (inputs the C side copies in): no
        padded host copy, which matters for the 21.5 GB of cfg3 diagonals"""
        arr = (OrcCt * len(cts))()
        keep = []
        for i, c in enumerate(cts):
            d = np.ascontiguousarray(c.data, dtype=np.uint64)
            keep.append(d)
            arr[i] = OrcCt(_p(d), c.size, c.level, c.scale)
        return arr, keep

    def bench_matvec(self, A, n, X, rk, gk, nthreads=1, j_begin=0, j_end=None, finish=True, outputs=False):
        """Seconds for one diag x col matvec of n diagonals (cycling over the distinct A) over X (C++ timer);
        outputs=True: (seconds, the results)."""
        a, ab = self._views(A)
        x, xb = self._views(X)
        secs = C.c_double()
        lvl = X[0].level
        outs, ob = self._many([Ct(np.zeros((3, lvl, self.N), np.uint64), 1.0) for _ in X]) if outputs else (None, None)
        _check(lib().orc_bench_matvec(self.h, a, C.c_uint64(len(A)), C.c_uint64(n), x, C.c_uint64(len(X)), _p(rk),
                                      *self._gk(gk), C.c_int(nthreads), C.c_uint64(j_begin),
                                      C.c_uint64(n if j_end is None else j_end), C.c_int(int(finish)),
                                      C.byref(secs), outs))
        if outputs:
            return secs.value, self._outs(outs, len(X))
        return secs.value

    def matmul_col_colT(self, A, B, p, rk, gk, nthreads=1):
        a, ab = self._many(A)
        b, bb = self._many(B)
        lvl = A[0].level
        outs, ob = self._many([Ct(np.zeros((3, lvl, self.N), np.uint64), 1.0) for _ in range(p)])
        _check(lib().orc_matmul_col_colT(self.h, a, C.c_uint64(len(A)), b, C.c_uint64(p), _p(rk),
                                         *self._gk(gk), outs, C.c_int(nthreads)))
        return self._outs(outs, p)

    def matrix_matmul(self, A, ar, ac, atr, B, br, bc, btr, rk):
        a, ab = self._many(A)
        b, bb = self._many(B)
        r = (ac if atr else ar)
        c = (br if btr else bc)
        lvl = A[0].level
        outs, ob = self._many([Ct(np.zeros((3, lvl, self.N), np.uint64), 1.0) for _ in range(r * c)])
        _check(lib().orc_matrix_matmul(self.h, a, C.c_uint64(ar), C.c_uint64(ac), C.c_int(int(atr)), b,
                                       C.c_uint64(br), C.c_uint64(bc), C.c_int(int(btr)), _p(rk), outs))
        return self._outs(outs, r * c)
