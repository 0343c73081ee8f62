"""Development tool: repeat the sequence of tests/test_gpu_fullsize.py's first two tests in one
process — the 64-diagonal subset over 48 vectors (3 lanes) checked against the oracle, then the full n = 4096 cfg3
matvec over 48 vectors and the same 4 vectors alone — and classify every bit mismatch:
  * which side decrypts to M x (the decrypt error of both sides),
  * the shape of the difference: INTT of (alone - lanes) per limb, centred; a small sparse integer vector that is
    the same in every limb is a rounding / off-by-q difference (a valid ciphertext either way), anything else is
    garbage from a wrong read.
usage: python tools/determinism_full.py [--reps R] [--poison-reps P] [--serial-reps S] [--onelane-reps O]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401  (one HIP runtime)
torch.cuda.is_available()
from _helpers import load_hecdna, load_oracle, trie_subset  # noqa: E402
from test_gpu_parity import Env  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=6)
ap.add_argument("--poison-reps", type=int, default=1)
ap.add_argument("--serial-reps", type=int, default=1)
ap.add_argument("--onelane-reps", type=int, default=1)
a = ap.parse_args()

hec, orc = load_hecdna(), load_oracle()
T = 16
t0 = time.time()
e = Env(orc, hec, 1 << 15, [60] + [40] * 9 + [60], seed=3131)
n, p, L = 4096, 48, len(e.m) - 1
slots = e.N // 2
js = trie_subset(e.N, n, target=64)
vals = e.rng.uniform(-1, 1, (len(js), slots))
A = [e.orc.Ct(r, 2.0**40) for r in e.o.encrypt_many(e.sk, vals, 2.0**40, L, 5000, nthreads=T)]
vals = e.rng.uniform(-1, 1, (p, slots))
X = [e.orc.Ct(r, 2.0**40) for r in e.o.encrypt_many(e.sk, vals, 2.0**40, L, 6000, nthreads=T)]
exp = e.o.matmul_diag_col_set(A, js, X, e.rk_h, e.gk_h, nthreads=T)
gsub = [e.up(c) for c in A]
sdiags = [gsub[0]] * n
for k, j in enumerate(js):
    sdiags[j] = gsub[k]
gXs = [e.up(x) for x in X]
rng = np.random.default_rng(4096)
M = rng.uniform(-1, 1, (n, n))
xs = rng.uniform(-1, 1, (p, n))
r = np.arange(slots) % n
raw = e.o.encrypt_many(e.sk, np.stack([M[r, (r + j) % n] for j in range(n)]), 2.0**40, L, 70000, nthreads=T)
gA = [e.ctx.ciphertext(raw[j], 2.0**40) for j in range(n)]
del raw
rawx = e.o.encrypt_many(e.sk, xs[:, r], 2.0**40, L, 90000, nthreads=T)
gX = [e.ctx.ciphertext(rawx[i], 2.0**40) for i in range(p)]
ref = xs @ M.T
e.ctx.set_option("lanes", 3)  # the opt-in lanes (one lane is the default since round 5)
print("setup %.1f s" % (time.time() - t0), flush=True)
idx = [0, 16, 32, 47]


def dec_err(d, i):
    ct = e.orc.Ct(d, 2.0**40 * 2.0**40 / e.m[L - 1])
    v = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
    return float(np.max(np.abs(v - ref[i][r])))


def diff_shape(x, y):
    """x, y: (2, l, N) NTT-form words; INTT per limb of (x - y) mod q, centred."""
    out = []
    for k in range(2):
        per = []
        for i in range(x.shape[1]):
            q = np.uint64(e.m[i])
            dv = (x[k, i] + (q - y[k, i])) % q
            c = np.array(e.o.ntt_inv(i, dv), dtype=np.uint64).astype(object)
            cc = np.array([int(v) if int(v) <= int(q) // 2 else int(v) - int(q) for v in c], dtype=object)
            nz = np.nonzero(cc)[0]
            per.append((len(nz), int(max(abs(v) for v in cc)) if len(nz) else 0, list(nz[:4]), [int(cc[t]) for t in nz[:4]]))
        out.append(per)
    return out


base_full = base_alone = None


def one(tag):
    global base_full, base_alone
    t = time.time()
    got = e.ctx.matmul_diag_col_partial_set(sdiags, js, gXs, e.gk)
    sub_bad = [i for i, (g, c) in enumerate(zip(got, exp)) if not np.array_equal(g.download(), c.data)]
    fin = e.ctx.matmul_finish([got[i] for i in [0, 16, 47]], e.rk)
    del fin, got
    full = [c.download() for c in e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)]
    alone = [c.download() for c in e.ctx.matmul_diag_col(gA, [gX[i] for i in idx], e.rk, e.gk)]
    eq = [bool(np.array_equal(x, full[i])) for x, i in zip(alone, idx)]
    if base_full is None:
        base_full, base_alone = full, alone
    fb = [i for i in range(p) if not np.array_equal(full[i], base_full[i])]
    ab = [k for k in range(len(idx)) if not np.array_equal(alone[k], base_alone[k])]
    print("%-10s subset_bad=%s alone==lanes=%s lanes!=first at %s alone!=first at %s (%.1f s)" %
          (tag, sub_bad, eq, fb, ab, time.time() - t), flush=True)
    for k, i in enumerate(idx):
        if not eq[k]:
            print("   vec %d: decrypt err lanes %.3g alone %.3g" % (i, dec_err(full[i], i), dec_err(alone[k], i)),
                  flush=True)
            print("   diff (count, max|c|, first idx, first vals) per limb, c0:", diff_shape(alone[k], full[i])[0][:3],
                  flush=True)
    for i in fb[:2]:
        print("   lanes vec %d vs first: decrypt err now %.3g first %.3g" % (i, dec_err(full[i], i),
                                                                          dec_err(base_full[i], i)), flush=True)


for rep in range(a.reps):
    one("lanes3/%d" % rep)
e.ctx.set_option("lane_serial", 1)
for rep in range(a.serial_reps):
    one("serial/%d" % rep)
e.ctx.set_option("lane_serial", 0)
e.ctx.set_option("lanes", 1)
for rep in range(a.onelane_reps):
    one("onelane/%d" % rep)
e.ctx.set_option("lanes", 3)
e.ctx.set_option("poison", 1)
for rep in range(a.poison_reps):
    one("poison/%d" % rep)
print("done %.1f s" % (time.time() - t0), flush=True)
