"""Development tool: the full n = 4096 cfg3 matvec (48 vectors, 3 lanes) and the same 4 vectors alone, under
several engine settings (env applied at context creation), compared bit for bit across settings.
usage: python tools/bisect_full.py [--reps R] "ENV=a ENV2=b" ...   (the first setting is the reference)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime)
torch.cuda.is_available()
from _helpers import load_hecdna, load_oracle  # noqa: E402

hec = load_hecdna()
orc = load_oracle()
N, n, p = 1 << 15, 4096, 48
m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 9 + [60])
o = orc.Oracle(N, m)
L = len(m) - 1
sk = o.secret_key(3131)
rk_h = o.relin_key(sk, 3132)
gk_h = o.galois_keys(sk, o.default_galois_elts(), 3133)
rng = np.random.default_rng(4096)
slots = N // 2
M = rng.uniform(-1, 1, (n, n))
xs = rng.uniform(-1, 1, (p, n))
r = np.arange(slots) % n
t0 = time.time()
raw = o.encrypt_many(sk, np.stack([M[r, (r + j) % n] for j in range(n)]), 2.0**40, L, 70000, nthreads=16)
rawx = o.encrypt_many(sk, xs[:, r], 2.0**40, L, 90000, nthreads=16)
print("encrypted in %.1f s" % (time.time() - t0), flush=True)
alone_idx = [0, 16, 32, 47]
ref = None
args = sys.argv[1:]
reps = 1
if args and args[0] == "--reps":
    reps, args = int(args[1]), args[2:]
for setting in args:
    env = dict(kv.split("=") for kv in setting.split()) if setting.strip() else {}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    ctx = hec.Context(N, m)
    for k, v in old.items():
        if v is None:
            del os.environ[k]
        else:
            os.environ[k] = v
    gA = [ctx.ciphertext(raw[j], 2.0**40) for j in range(n)]
    gX = [ctx.ciphertext(rawx[i], 2.0**40) for i in range(p)]
    rk, gk = ctx.relin_key(rk_h), ctx.galois_keys(gk_h)
    for rep in range(reps):
        full = [c.download() for c in ctx.matmul_diag_col(gA, gX, rk, gk)]
        alone = [c.download() for c in ctx.matmul_diag_col(gA, [gX[i] for i in alone_idx], rk, gk)]
        a_eq = [bool(np.array_equal(a, full[i])) for a, i in zip(alone, alone_idx)]
        if ref is None:
            ref = (full, alone)
        bad = [i for i, (x, y) in enumerate(zip(full, ref[0])) if not np.array_equal(x, y)]
        al_eq = [bool(np.array_equal(x, y)) for x, y in zip(alone, ref[1])]
        print(repr(setting), rep, "alone==full:", a_eq, "full!=ref at:", bad, "alone==ref_alone:", al_eq, flush=True)
    del gA, gX, ctx
