"""GPU parity at the shapes bench.py times (VERDICT r01 "next round" #1).

- cfg3 (N = 2^15, {60, 40 x 9, 60}, the 29 default Galois keys): a diagonal subset of the n = 4096 matvec
  whose rotation prefix trie has every shape of the full one — the root with all 23 children (hoisted,
  split into groups of HOIST_GROUP = 6), the busiest depth-1 node, the deepest 7-key-switch NAF chains with
  a terminal at every depth — run for 48 input vectors, i.e. the 3 concurrent batch lanes of 16 the bench
  runs, bit-exact against the oracle's partials of the same diagonals (he_linalg.cpp:977-997);
- the full n = 4096 matvec over 48 encrypted vectors, decrypted and compared with M @ x, and each lane's
  outputs equal to the same vectors run alone (size-independent properties: the oracle would need
  18,204 key switches per vector);
- cfg5 (N = 2^16, {60, 40 x 15, 60}): the same subset construction on the n = 1024 matmul with 32 columns
  (2 lanes of 16) and only the keys the subset touches, bit-exact, then relinearize + rescale.
"""
import os

import numpy as np
import pytest

from _helpers import rotation_seq, subset_trie_shape, trie_subset

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)))


@pytest.fixture(scope="module")
def env15(orc, hecdna):
    """BASELINE cfg3 parameters, N = 2^15, {60, 40 x 9, 60}, the 29 default Galois keys."""
    from test_gpu_parity import Env
    e = Env(orc, hecdna, 1 << 15, [60] + [40] * 9 + [60], seed=3131)
    assert len(e.elts) == 29
    return e


def _place(e, js, cts, n):
    """n diagonal handles with the subset's ciphertexts at their indices (the rest are never read)."""
    g = [e.up(c) for c in cts]
    diags = [g[0]] * n
    for k, j in enumerate(js):
        diags[j] = g[k]
    return diags


def _enc_many(e, count, seed0, level):
    vals = e.rng.uniform(-1, 1, (count, e.N // 2))
    raw = e.o.encrypt_many(e.sk, vals, 2.0**40, level, seed0, nthreads=THREADS)
    return [e.orc.Ct(raw[v], 2.0**40) for v in range(count)]


@pytest.mark.timeout(900)
def test_cfg3_bench_schedule_subset_bitexact(env15):
    e = env15
    n, p, L = 4096, 48, len(e.m) - 1
    js = trie_subset(e.N, n, target=64)
    root_kids, max_kids, depth, ks = subset_trie_shape(e.N, js)
    assert (root_kids, depth) == (23, 7) and max_kids > 6 and len(js) == 64
    A = _enc_many(e, len(js), 5000, L)
    X = _enc_many(e, p, 6000, L)
    exp = e.o.matmul_diag_col_set(A, js, X, e.rk_h, e.gk_h, nthreads=THREADS)
    got = e.ctx.matmul_diag_col_partial_set(_place(e, js, A, n), js, [e.up(x) for x in X], e.gk)
    assert len(got) == p
    for g, c in zip(got, exp):
        e.same(g, c)
    # the lazy relinearize + rescale of the bench's finish, on one output per lane
    pick = [0, 16, 47]
    fin = e.ctx.matmul_finish([got[i] for i in pick], e.rk)
    for f, i in zip(fin, pick):
        e.same(f, e.o.rescale(e.o.relinearize(exp[i], e.rk_h)))


@pytest.mark.timeout(900)
def test_cfg3_full_n_lanes_decrypt_and_lane_independence(env15):
    """The whole bench workload shape: n = 4096 encrypted diagonals of a random M, 48 encrypted x (3 lanes);
    decrypt(out[i]) ~ M @ x_i within CKKS error, and lane outputs equal the same vectors run alone."""
    e = env15
    n, p, L = 4096, 48, len(e.m) - 1
    slots = e.N // 2
    rng = np.random.default_rng(4096)
    M = rng.uniform(-1, 1, (n, n))
    xs = rng.uniform(-1, 1, (p, n))
    r = np.arange(slots) % n
    diag_vals = np.stack([M[r, (r + j) % n] for j in range(n)])          # diagonal j, slot r (cyclic)
    raw = e.o.encrypt_many(e.sk, diag_vals, 2.0**40, L, 70000, nthreads=THREADS)
    del diag_vals
    gA = [e.ctx.ciphertext(raw[j], 2.0**40) for j in range(n)]
    del raw
    rawx = e.o.encrypt_many(e.sk, xs[:, r], 2.0**40, L, 90000, nthreads=THREADS)
    gX = [e.ctx.ciphertext(rawx[i], 2.0**40) for i in range(p)]
    out = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)
    ref = xs @ M.T                                                          # (M x_i)[row]
    worst = 0.0
    for i, g in enumerate(out):
        ct = e.orc.Ct(g.download(), g.scale)
        assert ct.level == L - 1 and ct.size == 2
        d = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
        worst = max(worst, float(np.max(np.abs(d - ref[i][r]))))
    assert worst < 1e-3, worst
    alone_idx = [0, 16, 32, 47]                                             # one batch of 4: a single lane
    alone = e.ctx.matmul_diag_col(gA, [gX[i] for i in alone_idx], e.rk, e.gk)
    for a, i in zip(alone, alone_idx):
        assert np.array_equal(a.download(), out[i].download()) and a.scale == out[i].scale


@pytest.mark.timeout(900)
def test_cfg5_subset_bitexact(orc, hecdna):
    from test_gpu_parity import Env
    N, n, p = 1 << 16, 1024, 32
    bits = [60] + [40] * 15 + [60]
    js = trie_subset(N, n, target=0)
    root_kids, max_kids, depth, ks = subset_trie_shape(N, js)
    assert root_kids == max_kids == 19 and depth == 6
    o = orc.Oracle(N, orc.Oracle.create_coeff_modulus(N, bits))
    steps = sorted({s for j in js if j for s in rotation_seq(N, j)})
    e = Env(orc, hecdna, N, bits, seed=505, elts=[o.elt_from_step(s) for s in steps])
    L = len(e.m) - 1
    A = _enc_many(e, len(js), 8000, L)
    X = _enc_many(e, p, 9000, L)
    exp = e.o.matmul_diag_col_set(A, js, X, e.rk_h, e.gk_h, nthreads=THREADS)
    got = e.ctx.matmul_diag_col_partial_set(_place(e, js, A, n), js, [e.up(x) for x in X], e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)
    fin = e.ctx.matmul_finish([got[0], got[p - 1]], e.rk)
    e.same(fin[0], e.o.rescale(e.o.relinearize(exp[0], e.rk_h)))
    e.same(fin[1], e.o.rescale(e.o.relinearize(exp[p - 1], e.rk_h)))
