"""CPU: the oracle's restatement of the reference's he::math / he::util schedules (oracle/he_math_ref.py) computes
what the reference's comments say they compute (include/he_math.h:8-33): decrypted, 1/x, 1/sqrt(2x), sqrt(x), |x|
within the CKKS noise and the iteration's own error, the least-squares line of the reference's data
(matrix_operations.cpp:890-891), and drop / reach_chain_level land on the right level with the scale SEAL keeps.
These fix the math of the restatement; the GPU drop-in is then checked bit for bit against it
(tests/test_gpu_he_math.py)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import he_math_ref as hm  # noqa: E402


@pytest.fixture(scope="module")
def env(orc):
    N = 1 << 10
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 10 + [60])
    o = orc.Oracle(N, m)
    sk = o.secret_key(5)
    rk = o.relin_key(sk, 6)
    rng = np.random.default_rng(7)
    x = rng.uniform(0.5, 1.5, N // 2)
    s = rng.uniform(0.3, 1.0, N // 2) * rng.choice([-1.0, 1.0], N // 2)
    scale = 2.0**40
    enc = lambda v, seed: o.encrypt(sk, o.encode(v, scale, 10), scale, seed)  # noqa: E731
    return o, sk, rk, x, s, enc(x, 8), enc(s, 9)


def dec(o, sk, ct):
    return o.decode(o.decrypt(sk, ct), ct.scale).real


def test_signed_inv(env):
    o, sk, rk, x, s, cx, cs = env
    y = hm.signed_inv(o, rk, cx, 1.0, 4)   # |1 - x| < 0.5: error 0.5^(2^4)
    assert y.level == 10 - 1 - 1 - 3 and y.size == 2
    assert np.max(np.abs(dec(o, sk, y) - 1 / x)) < 1e-4
    y1 = hm.signed_inv(o, rk, cx, 1.0, 1)  # 2a - a^2 x
    assert np.max(np.abs(dec(o, sk, y1) - (2 - x))) < 1e-6


def test_inv_sqrt_sqrt_abs(env):
    o, sk, rk, x, s, cx, cs = env
    y = hm.inv_sqrt_twice(o, rk, cx, 0.7, 3)
    assert y.level == 10 - 5
    # three Newton steps from 0.7: a few 1e-3 at the ends of (0.5, 1.5)
    assert np.max(np.abs(dec(o, sk, y) - 1 / np.sqrt(2 * x))) < 2e-2
    r = hm.sqrt(o, rk, cx, 1.0, 3)
    assert np.max(np.abs(dec(o, sk, r) - np.sqrt(x))) < 2e-2
    a = hm.abs_(o, rk, cs, 1.0, 4)
    assert a.level == 10 - 1 - 7 - 1
    assert np.max(np.abs(dec(o, sk, a) - np.abs(s))) < 5e-2


def test_drop_and_reach_chain_level(env):
    o, sk, rk, x, s, cx, cs = env
    (d,) = hm.drop_chain_levels(o, [cx], 3)
    assert d.level == 7 and np.max(np.abs(dec(o, sk, d) - x)) < 1e-6
    # the scale follows SEAL: each level multiplies by the plaintext scale (= the ciphertext's) and divides by q_last
    sc = cx.scale
    for lvl in (10, 9, 8):
        sc = sc * sc / float(o.moduli[lvl - 1])
    assert d.scale == sc
    e, f = hm.reach_chain_level(o, [cx, cs], d)
    assert e.level == f.level == 7 and np.max(np.abs(dec(o, sk, f) - s)) < 1e-6


def test_least_squares_reference_data(orc):
    """the reference demo's data (matrix_operations.cpp:890-891) through the restated flow: a, b of the fitted line"""
    N = 1 << 10
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 15 + [60])
    o = orc.Oracle(N, m)
    sk = o.secret_key(11)
    rk = o.relin_key(sk, 12)
    gk = o.galois_keys(sk, [o.elt_from_step(k) for k in (1, 2, 4)], 13)
    xs = np.array([6, 5.8, 6.5, 5.4, 6.8])
    ys = np.array([2, 1.4, 2.4, 1.5, 2.4])
    scale = 2.0**40
    cx = o.encrypt(sk, o.encode(xs, scale, 16), scale, 14)
    cy = o.encrypt(sk, o.encode(ys, scale, 16), scale, 15)
    out = hm.least_squares_2d(o, rk, gk, cx, cy, 5)
    n = 5
    denom = n * np.sum(xs * xs) - np.sum(xs) ** 2
    a = (n * np.sum(xs * ys) - np.sum(xs) * np.sum(ys)) / denom
    b = (np.sum(ys) * np.sum(xs * xs) - np.sum(xs) * np.sum(xs * ys)) / denom
    got = [dec(o, sk, c)[0] for c in out]
    assert abs(got[0] - denom) < 1e-3 and abs(got[1] - 1 / denom) < 1e-5
    assert abs(got[4] - a) < 1e-3 and abs(got[5] - b) < 1e-2
    assert out[1].level == 6 and out[4].level == out[5].level == 5  # 16 - 2 - 1 (denominator) - 7 (inverse) - 1
