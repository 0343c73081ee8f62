"""Generate the committed golden fixtures in tests/golden/ from the CPU oracle.

Inputs are regenerated deterministically from the seeds recorded in each fixture, so a fixture is
(params, seeds, SHA-256 of the inputs, SHA-256 of every output ciphertext).  The GPU parity tests
recompute the outputs through the C-ABI and must reproduce every hash byte for byte.

cfg1 mirrors the reference demo `demo matrix_operations batched_matmul_ckks` with COL_OR_DIAG = 1
(src/demos/matrix_operations.cpp:1042-1175): N = 2^13, CoeffModulus::Create(N, {60,40,40,60}),
scale 2^40, 64x64 data  mat1[c][r] = 2 + 64c + (r mod 64)  (:1079-1087), the same 64 column
ciphertexts used as A's diagonals and as B's columns (:1129-1131), out = A.matmul(eval, rk, gk, B).

cfg1_colcolT is the reference's compiled default, COL_OR_DIAG = 0 (:1123-1128): the same 64 column
ciphertexts as a col-batched A, B = A^T (a transposed copy), out = A.matmul(eval, rk, gk, B), i.e. the
col x col^T branch of he_linalg.cpp:977-1002: out[i] = rescale(relin(sum_j rot(A[j], i) (*) A[j])), the i-th
diagonal of A.A^T.

Usage: python tests/golden/make_golden.py [--threads 8] [--only cfg1_colcolT]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from _helpers import load_oracle  # noqa: E402


def sha(ct_data, scale=None):
    h = hashlib.sha256(np.ascontiguousarray(ct_data, dtype=np.uint64).tobytes())
    if scale is not None:
        h.update(np.float64(scale).tobytes())
    return h.hexdigest()


CFG1 = dict(N=1 << 13, bits=[60, 40, 40, 60], scale=2.0**40, n=64, sk_seed=1001, rk_seed=1002, gk_seed=1003,
            enc_seed0=2000)


def cfg1_inputs(orc, cfg=CFG1):
    O = orc.Oracle
    N, n = cfg["N"], cfg["n"]
    m = O.create_coeff_modulus(N, cfg["bits"])
    o = O(N, m)
    sk = o.secret_key(cfg["sk_seed"])
    rk = o.relin_key(sk, cfg["rk_seed"])
    gk = o.galois_keys(sk, o.default_galois_elts(), cfg["gk_seed"])
    slots = N // 2
    level = len(m) - 1
    cts = []
    for c in range(n):  # matrix_operations.cpp:1081-1087
        vals = np.array([2 + n * c + (r % n) for r in range(slots)], dtype=np.float64)
        pt = o.encode(vals, cfg["scale"], level)
        cts.append(o.encrypt(sk, pt, cfg["scale"], cfg["enc_seed0"] + c))
    return o, m, sk, rk, gk, cts


def cfg1_expected_plain(n, slots):
    """Plaintext value of out[i] slot r: sum_j col_i[(r+j) mod n] * col_j[r mod n]."""
    col = lambda c, r: 2 + n * c + (r % n)  # noqa: E731
    return [np.array([sum(col(i, r + j) * col(j, r) for j in range(n)) for r in range(n)], dtype=np.float64)
            for i in range(n)]


def cfg1_colcolT_expected_plain(n):
    """Plaintext value of out[i] slot r (r < n): sum_j col_j[(r+i) mod n] * col_j[r] = (A A^T)[r][(r+i) mod n]."""
    col = lambda c, r: 2 + n * c + (r % n)  # noqa: E731
    return [np.array([sum(col(j, r + i) * col(j, r) for j in range(n)) for r in range(n)], dtype=np.float64)
            for i in range(n)]


def make_colcolT(orc, threads):
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    outs = o.matmul_col_colT(cts, cts, CFG1["n"], rk, gk, nthreads=threads)
    exp = cfg1_colcolT_expected_plain(CFG1["n"])
    for i in (0, 1, 33, 63):
        d = o.decode(o.decrypt(sk, outs[i]), outs[i].scale).real[: CFG1["n"]]
        err = np.max(np.abs(d - exp[i]) / np.abs(exp[i]))
        assert err < 1e-6, (i, err)
    fx = dict(CFG1)
    fx.update(moduli=[int(x) for x in m], form="COL_OR_DIAG=0: col(A) x col(A)^T -> diag output",
              input_sha256=[sha(c.data, c.scale) for c in cts],
              output_sha256=[sha(c.data, c.scale) for c in outs],
              output_level=outs[0].level, output_scale=outs[0].scale)
    with open(os.path.join(HERE, "cfg1_colcolT.json"), "w") as f:
        json.dump(fx, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    orc = load_oracle()
    if args.only == "cfg1_colcolT":
        make_colcolT(orc, args.threads)
        return
    make_colcolT(orc, args.threads)
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    outs = o.matmul_diag_col(cts, cts, rk, gk, nthreads=args.threads)
    fx = dict(CFG1)
    fx.update(moduli=[int(x) for x in m],
              input_sha256=[sha(c.data, c.scale) for c in cts],
              rk_sha256=sha(rk), gk_sha256={str(e): sha(k) for e, k in gk.items()},
              output_sha256=[sha(c.data, c.scale) for c in outs],
              output_level=outs[0].level, output_scale=outs[0].scale)
    # functional sanity (CKKS error): decrypt a few outputs
    exp = cfg1_expected_plain(CFG1["n"], CFG1["N"] // 2)
    for i in (0, 17, 63):
        d = o.decode(o.decrypt(sk, outs[i]), outs[i].scale).real[: CFG1["n"]]
        err = np.max(np.abs(d - exp[i]) / np.abs(exp[i]))
        assert err < 1e-6, (i, err)
    with open(os.path.join(HERE, "cfg1_matvec.json"), "w") as f:
        json.dump(fx, f, indent=1)
    # cfg2 primitive fixture: batched NTT of seeded random residues, N = 2^15, 10+1 primes
    N = 1 << 15
    m2 = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 9 + [60])
    o2 = orc.Oracle(N, m2)
    rng = np.random.default_rng(2024)
    data = np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m2])
    fwd = np.stack([o2.ntt_fwd(i, data[i]) for i in range(len(m2))])
    fx2 = dict(N=N, bits=[60] + [40] * 9 + [60], moduli=[int(x) for x in m2], rng_seed=2024,
               input_sha256=sha(data), forward_sha256=[sha(fwd[i]) for i in range(len(m2))])
    with open(os.path.join(HERE, "cfg2_ntt.json"), "w") as f:
        json.dump(fx2, f, indent=1)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
