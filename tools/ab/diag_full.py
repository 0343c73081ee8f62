"""Development tool: the sequence of tests/test_gpu_fullsize.py (subset partials, then the full n = 4096 matvec)
on one context, then the same 4 vectors alone several ways, to locate a lane / batch-size dependence."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
torch.cuda.is_available()
from _helpers import load_hecdna, load_oracle, trie_subset  # noqa: E402
from test_gpu_parity import Env  # noqa: E402

hec, orc = load_hecdna(), load_oracle()
settings = [a for a in sys.argv[1:] if "=" in a]
os.environ.update(dict(kv.split("=") for a in settings for kv in a.split()))
e = Env(orc, hec, 1 << 15, [60] + [40] * 9 + [60], seed=3131)
if "--garbage" in sys.argv:  # freed device memory full of random words, so later allocations start dirty
    junk_host = np.random.default_rng(1).integers(0, 2**63, (2, 10, e.N), dtype=np.uint64) % np.uint64(1 << 36)
    junk = [e.ctx.ciphertext(junk_host, 2.0**40) for _ in range(2000)]  # 2000 x 5.8 MB
    del junk
    import gc
    gc.collect()
    print("garbage freed", flush=True)
n, p, L = 4096, 48, len(e.m) - 1
if "--subset" in sys.argv:
    js = trie_subset(e.N, n, target=64)
    vals = e.rng.uniform(-1, 1, (len(js), e.N // 2))
    A = [e.orc.Ct(r, 2.0**40) for r in e.o.encrypt_many(e.sk, vals, 2.0**40, L, 5000, nthreads=16)]
    vals = e.rng.uniform(-1, 1, (p, e.N // 2))
    X = [e.orc.Ct(r, 2.0**40) for r in e.o.encrypt_many(e.sk, vals, 2.0**40, L, 6000, nthreads=16)]
    g = [e.up(c) for c in A]
    diags = [g[0]] * n
    for k, j in enumerate(js):
        diags[j] = g[k]
    got = e.ctx.matmul_diag_col_partial_set(diags, js, [e.up(x) for x in X], e.gk)
    fin = e.ctx.matmul_finish([got[i] for i in [0, 16, 47]], e.rk)
    print("subset done", flush=True)
slots = e.N // 2
rng = np.random.default_rng(4096)
M = rng.uniform(-1, 1, (n, n))
xs = rng.uniform(-1, 1, (p, n))
r = np.arange(slots) % n
raw = e.o.encrypt_many(e.sk, np.stack([M[r, (r + j) % n] for j in range(n)]), 2.0**40, L, 70000, nthreads=16)
gA = [e.ctx.ciphertext(raw[j], 2.0**40) for j in range(n)]
rawx = e.o.encrypt_many(e.sk, xs[:, r], 2.0**40, L, 90000, nthreads=16)
gX = [e.ctx.ciphertext(rawx[i], 2.0**40) for i in range(p)]
ref = xs @ M.T


def err(outs, idx):
    w = []
    for g, i in zip(outs, idx):
        ct = e.orc.Ct(g.download(), g.scale)
        d = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
        w.append(float(np.max(np.abs(d - ref[i][r]))))
    return w


full = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)
fd = [f.download() for f in full]
print("full err max", max(err(full, range(p))), flush=True)
idx = [0, 16, 32, 47]
for name, ctx_ in [("alone", e.ctx), ("alone again", e.ctx)]:
    a = ctx_.matmul_diag_col(gA, [gX[i] for i in idx], e.rk, e.gk)
    print(name, [bool(np.array_equal(x.download(), fd[i])) for x, i in zip(a, idx)], "err", err(a, idx), flush=True)
a16 = e.ctx.matmul_diag_col(gA, gX[:16], e.rk, e.gk)
print("first 16 (one lane)", sum(bool(np.array_equal(x.download(), fd[i])) for i, x in enumerate(a16)), "/16", flush=True)
full2 = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)
print("full again", sum(bool(np.array_equal(x.download(), fd[i])) for i, x in enumerate(full2)), "/48", flush=True)
