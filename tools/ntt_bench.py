"""Micro-benchmark: batched forward NTT time per limb for FP64-path (40-bit) vs integer-path (60-bit)
primes at N = 2^15 (development tool; not part of the product)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402  (one HIP runtime)
torch.cuda.is_available()
from _helpers import load_hecdna  # noqa: E402

hec = load_hecdna()
L = hec.lib()
L.hec_time_ntt_forward.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
for logN in (15, 16):
    N = 1 << logN
    for bits in (40, 60):
        m = hec.create_coeff_modulus(N, [bits] * 11)
        ctx = hec.Context(N, m)
        npolys = 64
        buf = hec.DeviceBuffer(ctx, npolys * 11 * N * 8)
        host = np.stack([np.stack([np.random.randint(0, 2**31, N).astype(np.uint64) for _ in range(11)])
                         for _ in range(npolys)])
        buf.upload(host)
        ms = C.c_double()
        L.hec_time_ntt_forward(ctx.h, buf.p, 11, npolys, 3, C.byref(ms))
        L.hec_time_ntt_forward(ctx.h, buf.p, 11, npolys, 10, C.byref(ms))
        per = ms.value * 1e3 / (11 * npolys)
        bfly = N // 2 * logN
        print(f"logN={logN} bits={bits}: {ms.value:.3f} ms for {11*npolys} limb-NTTs -> {per:.3f} us/limb, "
              f"{bfly / per / 1e6:.2f} T butterflies/s, {2 * N * 8 / per / 1e3:.0f} GB/s in+out")
