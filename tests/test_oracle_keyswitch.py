"""Oracle pinning: key switching and rescale (a8) against an independent pure-Python
restatement whose rounding is computed with big integers:
  mod-down:  out_i = floor((Y + floor(P/2)) / P)      mod q_i   (Y = CRT lift over {q_0..q_{l-1}, P})
  rescale:   out_i = floor((X + floor(q_l/2)) / q_l)  mod q_i   (X = CRT lift over {q_0..q_{l-1}})
(any CRT lift gives the same residues), plus the digit decomposition / key MAC restated per prime.
Only the NTT (pinned in test_oracle_ntt.py) is shared with the C++ oracle."""
import numpy as np
import pytest

N = 1 << 10


@pytest.fixture(scope="module")
def setup(orc):
    m = orc.Oracle.create_coeff_modulus(N, [50, 40, 40, 50])
    o = orc.Oracle(N, m)
    sk = o.secret_key(11)
    return o, m, sk


def crt(residues, moduli):
    Q = 1
    for q in moduli:
        Q *= q
    x = 0
    for r, q in zip(residues, moduli):
        Qi = Q // q
        x += int(r) * Qi * pow(Qi, -1, q)
    return x % Q


def py_switch_key(o, m, ct, target, key):
    """SEAL Evaluator::switch_key_inplace restated; returns new ct data [2][l][N]."""
    l, K, P = target.shape[0], len(m), m[-1]
    coeff = [o.ntt_inv(J, target[J]) for J in range(l)]
    prod = [[None] * (l + 1) for _ in range(2)]
    for I in range(l + 1):
        kI = K - 1 if I == l else I
        qI = m[kI]
        acc = [[0] * N, [0] * N]
        for J in range(l):
            op = target[J] if I == J else o.ntt_fwd(kI, coeff[J] % np.uint64(qI))
            for k in range(2):
                kk = key[J, k, kI]
                acc[k] = [a + int(x) * int(y) for a, x, y in zip(acc[k], op, kk)]
        for k in range(2):
            prod[k][I] = np.array([a % qI for a in acc[k]], dtype=np.uint64)
    out = ct.data.copy()
    for k in range(2):
        cd = [o.ntt_inv(i, prod[k][i]) for i in range(l)] + [o.ntt_inv(K - 1, prod[k][l])]
        mods = m[:l] + [P]
        vals = [(crt([cd[i][t] for i in range(l + 1)], mods) + P // 2) // P for t in range(N)]
        for i in range(l):
            r = o.ntt_fwd(i, np.array([v % m[i] for v in vals], dtype=np.uint64))
            out[k, i] = (out[k, i] + r) % np.uint64(m[i])
    return out


def py_rescale(o, m, ct):
    l = ct.level
    ql = m[l - 1]
    out = np.zeros((ct.size, l - 1, N), dtype=np.uint64)
    for k in range(ct.size):
        cd = [o.ntt_inv(i, ct.data[k, i]) for i in range(l)]
        vals = [(crt([cd[i][t] for i in range(l)], m[:l]) + ql // 2) // ql for t in range(N)]
        for i in range(l - 1):
            out[k, i] = o.ntt_fwd(i, np.array([v % m[i] for v in vals], dtype=np.uint64))
    return out


def random_ct(m, size, level, seed):
    rng = np.random.default_rng(seed)
    d = np.stack([np.stack([rng.integers(0, m[i], N, dtype=np.uint64) for i in range(level)]) for _ in range(size)])
    return d


def test_switch_key_matches_bigint_restatement(setup, orc):
    o, m, sk = setup
    rk = o.relin_key(sk, 5)
    for level in (3, 2):
        ct = orc.Ct(random_ct(m, 2, level, level), 2.0**40)
        target = random_ct(m, 1, level, 10 + level)[0]
        got = o.switch_key(ct, target, rk)
        assert np.array_equal(got.data, py_switch_key(o, m, ct, target, rk)), level


def test_relinearize_is_switch_key_of_c2(setup, orc):
    o, m, sk = setup
    rk = o.relin_key(sk, 6)
    d = random_ct(m, 3, 3, 21)
    ct3 = orc.Ct(d, 2.0**40)
    got = o.relinearize(ct3, rk)
    exp = py_switch_key(o, m, orc.Ct(d[:2].copy(), 2.0**40), d[2], rk)
    assert got.size == 2 and np.array_equal(got.data, exp)


def test_rescale_matches_bigint_rounding(setup, orc):
    o, m, sk = setup
    for level, size in ((3, 2), (3, 3), (2, 2)):
        ct = orc.Ct(random_ct(m, size, level, 30 + level + size), 2.0**80)
        got = o.rescale(ct)
        assert got.level == level - 1 and got.scale == 2.0**80 / m[level - 1]
        assert np.array_equal(got.data, py_rescale(o, m, ct))


def test_rescale_end_of_chain(setup, orc):
    o, m, sk = setup
    ct = orc.Ct(random_ct(m, 2, 1, 40), 2.0**40)
    with pytest.raises(orc.OracleError, match="end of modulus switching chain reached"):
        o.rescale(ct)
    with pytest.raises(orc.OracleError, match="end of modulus switching chain reached"):
        o.mod_switch(ct)


def test_galois_is_permutation_then_switch_key(setup, orc):
    o, m, sk = setup
    elt = 3
    gk = {elt: o.galois_key(sk, elt, 77)}
    d = random_ct(m, 2, 3, 50)
    got = o.apply_galois(orc.Ct(d, 2.0**40), elt, gk)
    c0 = o.apply_galois_ntt(d[0], elt)
    c1 = o.apply_galois_ntt(d[1], elt)
    base = orc.Ct(np.stack([c0, np.zeros_like(c1)]), 2.0**40)
    assert np.array_equal(got.data, py_switch_key(o, m, base, c1, gk[elt]))


def test_errors_follow_seal(setup, orc):
    o, m, sk = setup
    a = orc.Ct(random_ct(m, 2, 3, 60), 2.0**40)
    b = orc.Ct(random_ct(m, 2, 3, 61), 2.0**41)
    with pytest.raises(orc.OracleError, match="scale mismatch"):
        o.add(a, b)
    with pytest.raises(orc.OracleError, match="parameter mismatch"):
        o.add(a, orc.Ct(random_ct(m, 2, 2, 62), 2.0**40))
    with pytest.raises(orc.OracleError, match="Galois key not present"):
        o.apply_galois(a, 3, {})
    with pytest.raises(orc.OracleError, match="scale out of bounds"):
        o.multiply(orc.Ct(a.data, 2.0**70), orc.Ct(a.data, 2.0**70))
