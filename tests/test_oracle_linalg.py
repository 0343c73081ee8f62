"""Oracle: the he_linalg hot path restated (he_linalg.cpp:943-1006, 202-236) decrypts to the plaintext
products (functional), and the all-cores variant is bit-identical to the single-threaded one."""
import numpy as np
import pytest

from _helpers import col_vector, diag_vectors

N = 1 << 11
SLOTS = N // 2


@pytest.fixture(scope="module")
def env(orc):
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
    o = orc.Oracle(N, m)
    sk = o.secret_key(3)
    rk = o.relin_key(sk, 4)
    gk = o.galois_keys(sk, o.default_galois_elts(), 5)
    return o, m, sk, rk, gk


def enc(o, sk, v, seed, level=3):
    return o.encrypt(sk, o.encode(v, 2.0**40, level), 2.0**40, seed)


def dec(o, sk, ct):
    return o.decode(o.decrypt(sk, ct), ct.scale).real


def test_matvec_diag_col_functional_and_threads(env):
    o, m, sk, rk, gk = env
    n = 16
    rng = np.random.default_rng(0)
    M = rng.uniform(-1, 1, (n, n))
    xs = [rng.uniform(-1, 1, n) for _ in range(2)]
    A = [enc(o, sk, d, 10 + j) for j, d in enumerate(diag_vectors(M, SLOTS))]
    X = [enc(o, sk, col_vector(x, SLOTS), 50 + i) for i, x in enumerate(xs)]
    out1 = o.matmul_diag_col(A, X, rk, gk, nthreads=1)
    out4 = o.matmul_diag_col(A, X, rk, gk, nthreads=4)
    for a, b, x in zip(out1, out4, xs):
        assert np.array_equal(a.data, b.data) and a.scale == b.scale
        assert a.level == 2
        got = dec(o, sk, a)[:n]
        assert np.max(np.abs(got - M @ x)) < 1e-4


def test_partial_sums_recombine(env, orc):
    o, m, sk, rk, gk = env
    n = 8
    rng = np.random.default_rng(1)
    A = [enc(o, sk, rng.uniform(-1, 1, SLOTS), 100 + j) for j in range(n)]
    X = [enc(o, sk, rng.uniform(-1, 1, SLOTS), 200)]
    full = o.matmul_diag_col(A, X, rk, gk)[0]
    p1 = o.matmul_diag_col(A, X, rk, gk, j_begin=0, j_end=3, finish=False)[0]
    p2 = o.matmul_diag_col(A, X, rk, gk, j_begin=3, j_end=n, finish=False)[0]
    # integer sum of partials (what an RCCL/gloo all-reduce computes), then canonicalise mod q
    s = p1.data.astype(np.uint64) + p2.data.astype(np.uint64)
    for i in range(p1.level):
        s[:, i] %= np.uint64(m[i])
    acc = orc.Ct(s, p1.scale)
    fin = o.rescale(o.relinearize(acc, rk))
    assert np.array_equal(fin.data, full.data)


def test_col_colT_and_matrix_matmul_functional(env):
    o, m, sk, rk, gk = env
    n = 4
    rng = np.random.default_rng(2)
    a = [rng.uniform(-1, 1, SLOTS) for _ in range(n)]
    b = [rng.uniform(-1, 1, SLOTS) for _ in range(n)]
    A = [enc(o, sk, v, 300 + j) for j, v in enumerate(a)]
    B = [enc(o, sk, v, 400 + j) for j, v in enumerate(b)]
    p = 3
    out = o.matmul_col_colT(A, B, p, rk, gk)
    for i in range(p):
        exp = sum(np.roll(b[j], -i) * a[j] for j in range(n))
        assert np.max(np.abs(dec(o, sk, out[i]) - exp)) < 1e-4
    # Matrix::matmul on slot-wise scalars: 2x2 (column-major elems)
    Mx = [rng.uniform(-1, 1, SLOTS) for _ in range(4)]
    My = [rng.uniform(-1, 1, SLOTS) for _ in range(4)]
    CX = [enc(o, sk, v, 500 + k) for k, v in enumerate(Mx)]
    CY = [enc(o, sk, v, 600 + k) for k, v in enumerate(My)]
    R = o.matrix_matmul(CX, 2, 2, False, CY, 2, 2, False, rk)
    for i in range(2):
        for j in range(2):
            exp = sum(Mx[i + 2 * k] * My[k + 2 * j] for k in range(2))
            assert np.max(np.abs(dec(o, sk, R[i + 2 * j]) - exp)) < 1e-4


def test_sum_elems_functional(orc):
    """BatchedVector::sum_elems_inplace restated (he_linalg.cpp:667-713): slot r of the result holds
    sum_{k<dim} x[r + k], for odd and even dims; the reference demo's vector sums to 92 in slot 0
    (matrix_operations.cpp:780-799)."""
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
    o = orc.Oracle(N, m)
    sk = o.secret_key(1)
    gk = o.galois_keys(sk, o.default_galois_elts(), 3)
    op = np.array([-11, 8, 8, 7, -10, 80, 4, 2, 3, 1], dtype=float)
    r = o.sum_elems(o.encrypt(sk, o.encode(op, 2.0**40, 3), 2.0**40, 5), 10, gk)
    assert abs(o.decode(o.decrypt(sk, r), r.scale).real[0] - 92.0) < 1e-5
    slots = N // 2
    for dim in (1, 2, 3, 6, 7, 13):
        x = np.random.default_rng(dim).uniform(-1, 1, slots)
        r = o.sum_elems(o.encrypt(sk, o.encode(x, 2.0**40, 3), 2.0**40, 7), dim, gk)
        d = o.decode(o.decrypt(sk, r), r.scale).real
        exp = np.array([x[(np.arange(dim) + j) % slots].sum() for j in range(slots)])
        assert np.max(np.abs(d - exp)) < 1e-5
