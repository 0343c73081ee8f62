"""GPU parity at the shapes bench.py times (VERDICT r01 "next round" #1, r04 item 1).

- cfg3 (N = 2^15, {60, 40 x 9, 60}, the 29 default Galois keys): a diagonal subset of the n = 4096 matvec
  whose rotation prefix trie has every shape of the full one — the root with all 23 children (hoisted,
  split into groups of HOIST_GROUP = 6), the busiest depth-1 node, the deepest 7-key-switch NAF chains with
  a terminal at every depth — run for 48 input vectors in one batch and for 4 of them alone, both bit-exact
  against the oracle's partials of the same diagonals (he_linalg.cpp:977-997);
- the full n = 4096 matvec over 48 encrypted vectors, decrypted and compared with M @ x, and the same vectors run
  as a batch of 4 equal to them bit for bit; both sides are decrypted, so a mismatch names the side that is wrong
  (size-independent properties: the oracle would need 18,204 key switches per vector);
- cfg5 (N = 2^16, {60, 40 x 15, 60}): the same subset construction on the n = 1024 matmul with 32 columns
  and only the keys the subset touches, bit-exact, then relinearize + rescale;
- cfg3 in BASELINE's literal ct x pt form (configs[2], "ct x pt matvec 4096 x 4096"): the full n = 4096 matvec with
  GPU-encoded plaintext diagonals over 48 vectors, bit-exact against the oracle on the 64-diagonal trie
  subset (the other diagonals are zero plaintexts, whose products are exactly zero), and on a random M decrypted
  against M @ x with batch independence;
- cfg5 at full size: the whole 1024 x 1024 x 1024 product over 32 columns with the 31 default keys, decrypted
  against M @ X, and batch independence.
Every matvec here runs the default schedule (one lane: the whole batch on the context's stream; the opt-in
concurrent lanes are covered at N = 2^11 in test_gpu_parity.py).
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
    # the lazy relinearize + rescale of the bench's finish
    pick = [0, 16, 47]
    fin = e.ctx.matmul_finish([got[i] for i in pick], e.rk)
    for f, i in zip(fin, pick):
        e.same(f, e.o.rescale(e.o.relinearize(exp[i], e.rk_h)))
    # the same trie for 4 of the vectors alone (another batch size, so other kernel tilings and grids): oracle bits
    alone_idx = [0, 16, 32, 47]
    alone = e.ctx.matmul_diag_col_partial_set(_place(e, js, A, n), js, [e.up(X[i]) for i in alone_idx], e.gk)
    for g, i in zip(alone, alone_idx):
        e.same(g, exp[i])


def _dec_err(e, g, ref_row, r):
    ct = e.orc.Ct(g.download(), g.scale)
    d = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
    return float(np.max(np.abs(d - ref_row[r])))


def _batch_independence(e, out, alone, alone_idx, ref, r):
    """alone[k] (the vectors alone_idx run as one small batch) equals out[alone_idx[k]] bit for bit; when not, the
    assertion names the side whose decryption is off"""
    for a, i in zip(alone, alone_idx):
        if not (np.array_equal(a.download(), out[i].download()) and a.scale == out[i].scale):
            raise AssertionError("vector %d: batch of %d vs alone differ; decrypt error batch %.3g, alone %.3g" %
                                 (i, len(out), _dec_err(e, out[i], ref[i], r), _dec_err(e, a, ref[i], r)))


@pytest.mark.timeout(900)
def test_cfg3_full_n_decrypt_and_batch_independence(env15):
    """The whole bench workload shape: n = 4096 encrypted diagonals of a random M, 48 encrypted x in one batch;
    decrypt(out[i]) ~ M @ x_i within CKKS error, and the outputs equal the same vectors run as a batch of 4."""
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
    alone_idx = [0, 16, 32, 47]                                             # a batch of 4
    alone = e.ctx.matmul_diag_col(gA, [gX[i] for i in alone_idx], e.rk, e.gk)
    _batch_independence(e, out, alone, alone_idx, ref, r)


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


def _ctpt_full(e, vals_of, n, X):
    """hec_matmul_diagpt_col over n GPU-encoded plaintext diagonals (row j of vals_of(j0, j1)), in chunks."""
    L = len(e.m) - 1
    P = []
    for j0 in range(0, n, 512):
        P += e.ctx.encode(vals_of(j0, min(n, j0 + 512)), 2.0**40, L)
    return P, e.ctx.matmul_diagpt_col(P, X, e.gk)


@pytest.mark.timeout(900)
def test_cfg3_ctpt_full_matvec_subset_bitexact(env15):
    """The n = 4096 ct x pt matvec at cfg3 (hec_matmul_diagpt_col, he_operators.cpp:128-142 multiply_plain) with 48
    vectors: diagonals outside the 64-diagonal trie subset are zero, so the outputs equal the oracle's
    subset sum (rotate, multiply_plain, add, rescale) bit for bit while the GPU runs the whole trie."""
    e = env15
    n, p, L = 4096, 48, len(e.m) - 1
    js = trie_subset(e.N, n, target=64)
    where = {j: k for k, j in enumerate(js)}
    sub = e.rng.uniform(-1, 1, (len(js), e.N // 2))

    def vals_of(j0, j1):
        v = np.zeros((j1 - j0, e.N // 2))
        for j in range(j0, j1):
            if j in where:
                v[j - j0] = sub[where[j]]
        return v
    X = _enc_many(e, p, 6100, L)
    P, got = _ctpt_full(e, vals_of, n, [e.up(x) for x in X])
    exp = e.o.matmul_diagpt_col_set([P[j].download() for j in js], 2.0**40, js, X, e.gk_h, nthreads=THREADS)
    assert len(got) == p
    for g, c in zip(got, exp):
        e.same(g, c)


@pytest.mark.timeout(900)
def test_cfg3_ctpt_full_n_decrypt_and_batch_independence(env15):
    """cfg3 ct x pt over a random 4096 x 4096 M (GPU-encoded diagonals) and 48 encrypted x: decrypt(out_i) = M x_i
    within CKKS error, and the outputs equal the same vectors run as a batch of 4."""
    e = env15
    n, p, L = 4096, 48, len(e.m) - 1
    slots = e.N // 2
    rng = np.random.default_rng(40960)
    M = rng.uniform(-1, 1, (n, n))
    xs = rng.uniform(-1, 1, (p, n))
    r = np.arange(slots) % n

    def vals_of(j0, j1):
        return np.stack([M[r, (r + j) % n] for j in range(j0, j1)])
    rawx = e.o.encrypt_many(e.sk, xs[:, r], 2.0**40, L, 91000, nthreads=THREADS)
    gX = [e.ctx.ciphertext(rawx[i], 2.0**40) for i in range(p)]
    P, out = _ctpt_full(e, vals_of, n, gX)
    ref = xs @ M.T
    worst = 0.0
    for i, g in enumerate(out):
        ct = e.orc.Ct(g.download(), g.scale)
        assert ct.level == L - 1 and ct.size == 2
        d = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
        worst = max(worst, float(np.max(np.abs(d - ref[i][r]))))
    assert worst < 1e-3, worst
    alone_idx = [0, 16, 32, 47]
    alone = e.ctx.matmul_diagpt_col(P, [gX[i] for i in alone_idx], e.gk)
    _batch_independence(e, out, alone, alone_idx, ref, r)


@pytest.mark.timeout(900)
def test_cfg5_full_product_decrypt_and_batch_independence(orc, hecdna):
    """BASELINE cfg5 at full size on one GPU: the 1024 x 1024 x 1024 ct x ct matmul as BatchedMatrix::matmul diag x
    col (matrix_operations.cpp:844-850 parameters: N = 2^16, {60, 40 x 15, 60}, the 31 default keys) over 32 output
    columns in one batch: decrypt(out_c) = (M B)[:, c] within CKKS error; they equal the columns run as a batch of 4."""
    from test_gpu_parity import Env
    N, n, p = 1 << 16, 1024, 32
    bits = [60] + [40] * 15 + [60]
    e = Env(orc, hecdna, N, bits, seed=5151)
    assert len(e.elts) == 31
    L = len(e.m) - 1
    slots = N // 2
    rng = np.random.default_rng(1024)
    M = rng.uniform(-1, 1, (n, n))
    Bm = rng.uniform(-1, 1, (n, p))
    r = np.arange(slots) % n
    gA = []
    for j0 in range(0, n, 256):
        raw = e.o.encrypt_many(e.sk, np.stack([M[r, (r + j) % n] for j in range(j0, j0 + 256)]), 2.0**40, L,
                               50000 + j0, nthreads=THREADS)
        gA += [e.ctx.ciphertext(raw[k], 2.0**40) for k in range(256)]
        del raw
    rawx = e.o.encrypt_many(e.sk, Bm.T[:, r], 2.0**40, L, 60000, nthreads=THREADS)
    gX = [e.ctx.ciphertext(rawx[c], 2.0**40) for c in range(p)]
    out = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)
    ref = (M @ Bm).T
    worst = 0.0
    for c, g in enumerate(out):
        ct = e.orc.Ct(g.download(), g.scale)
        assert ct.level == L - 1 and ct.size == 2
        d = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
        worst = max(worst, float(np.max(np.abs(d - ref[c][r]))))
    assert worst < 1e-3, worst
    alone_idx = [0, 15, 16, 31]
    alone = e.ctx.matmul_diag_col(gA, [gX[c] for c in alone_idx], e.rk, e.gk)
    _batch_independence(e, out, alone, alone_idx, ref, r)
