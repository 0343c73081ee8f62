"""Oracle pinning: the NTT convention and the Galois table (a3) by known answers:
naive O(N^2) evaluation at psi^(2*bitrev(j)+1), inverse round trip, the negacyclic convolution
theorem, and NTT-domain Galois permutation == coefficient-domain automorphism X -> X^elt."""
import numpy as np
import pytest

N = 1 << 10


def brv(x, b):
    return int(format(x, "0%db" % b)[::-1], 2)


@pytest.fixture(scope="module")
def small(orc):
    m = orc.Oracle.create_coeff_modulus(N, [50, 40, 40, 50])
    return orc.Oracle(N, m), m


def poly_eval(a, x, q):
    v = 0
    for c in reversed(a):
        v = (v * x + int(c)) % q
    return v


def test_ntt_matches_naive_evaluation(small):
    o, m = small
    rng = np.random.default_rng(0)
    for i, q in enumerate(m):
        a = rng.integers(0, q, N, dtype=np.uint64)
        A = o.ntt_fwd(i, a)
        psi = o.root(i)
        for j in list(range(8)) + [N // 2, N - 1] + list(rng.integers(0, N, 8)):
            assert int(A[j]) == poly_eval(a, pow(psi, 2 * brv(int(j), 10) + 1, q), q)
        assert np.array_equal(o.ntt_inv(i, A), a)
        assert (A < q).all()


def test_negacyclic_convolution(small):
    o, m = small
    q = m[1]
    rng = np.random.default_rng(1)
    a = rng.integers(0, q, N, dtype=np.uint64)
    b = rng.integers(0, q, N, dtype=np.uint64)
    A, B = o.ntt_fwd(1, a), o.ntt_fwd(1, b)
    C = np.array([(int(x) * int(y)) % q for x, y in zip(A, B)], dtype=np.uint64)
    c = o.ntt_inv(1, C)
    ai, bi = [int(x) for x in a], [int(x) for x in b]
    ref = [0] * N
    for i in range(N):
        if ai[i] == 0:
            continue
        for j in range(N):
            k = i + j
            if k < N:
                ref[k] += ai[i] * bi[j]
            else:
                ref[k - N] -= ai[i] * bi[j]
    assert [x % q for x in ref] == [int(x) for x in c]


def test_galois_ntt_equals_coefficient_automorphism(small):
    o, m = small
    q = m[0]
    rng = np.random.default_rng(2)
    a = rng.integers(0, q, N, dtype=np.uint64)
    for elt in [3, 9, pow(3, N // 2 - 1, 2 * N), 2 * N - 1, 5 ** 3 % (2 * N)]:
        coeff = [0] * N
        for i, c in enumerate(a):  # a(X^elt) mod X^N + 1
            e = i * elt % (2 * N)
            if e < N:
                coeff[e] = (coeff[e] + int(c)) % q
            else:
                coeff[e - N] = (coeff[e - N] - int(c)) % q
        expect = o.ntt_fwd(0, np.array(coeff, dtype=np.uint64))
        got = o.apply_galois_ntt(o.ntt_fwd(0, a), elt)
        assert np.array_equal(got, expect), elt
