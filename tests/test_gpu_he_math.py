"""The he_math.h / he_util.h half of the drop-in boundary (north_star; reference include/he_math.h:15-33,
include/he_util.h:13-77, src/core/he_math.cpp:22-269) on the GPU, bit for bit against the oracle's restatement of the
same schedules (oracle/he_math_ref.py): the scalar CKKSEncoder::encode(double, parms_id, scale) (hec_encode_scalar),
the drop_chain_levels pattern (scalar encode -> multiply_plain -> rescale, repeated) through the C ABI, and signed_inv /
inv_sqrt_twice / sqrt / abs / drop_chain_levels / reach_chain_level / the least-squares flow through the C++ drop-in
(bin/he_demo, cpp/src/he_math.cpp).  The decrypted values are checked against numpy as well."""
import os
import sys

import numpy as np
import pytest

from test_gpu_cpp_facade import demo, run, same  # noqa: F401  (module fixture)

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import he_math_ref as hm  # noqa: E402


@pytest.mark.parametrize("value,scale,level", [(1.0, 2.0**40, 10), (-0.25, 2.0**40, 7), (3.0 / 2 * 0.7, 2.0**40, 4),
                                               (0.0, 2.0**40, 10), (-2.0, 2.0**40, 1), (5.0, 2.0**40, 3),
                                               (1e25, 2.0**60, 10), (-3.3e27, 2.0**62, 10), (1.4142135623730951, 2.0**30, 2)])
def test_encode_scalar_bitexact(orc, hecdna, value, scale, level):
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 9 + [60])
    o = orc.Oracle(N, m)
    ctx = hecdna.Context(N, m)
    pt = ctx.encode_scalar(value, scale, level)
    assert pt.info() == (level, scale)
    assert np.array_equal(pt.download(), o.encode_scalar(value, scale, level))


def test_encode_scalar_errors(orc, hecdna):
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
    ctx = hecdna.Context(N, m)
    o = orc.Oracle(N, m)
    for args, msg in [((2.0**100, 2.0**30, 3), "encoded value is too large"),
                      ((float("inf"), 2.0**30, 3), "encoded value is too large"),
                      ((float("nan"), 2.0**30, 3), "encoded value is too large"),
                      ((1.0, 2.0**125, 3), "scale out of bounds"), ((1.0, 2.0**30, 4), "parms_id is not valid")]:
        with pytest.raises(hecdna.InvalidArgument, match=msg):
            ctx.encode_scalar(*args)
        with pytest.raises(orc.OracleError, match=msg):
            o.encode_scalar(*args)


def test_drop_chain_levels_pattern_cabi(orc, hecdna):
    """he_util.h:27-48 through the C ABI: per level, encode(1, ct.parms_id, ct.scale) -> multiply_plain -> rescale, on
    two ciphertexts sharing the plaintext, down to the last level, bit-exact at every step"""
    N = 1 << 12
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 9 + [60])
    o = orc.Oracle(N, m)
    ctx = hecdna.Context(N, m)
    sk = o.secret_key(3)
    rng = np.random.default_rng(4)
    scale = 2.0**40
    cts = [o.encrypt(sk, o.encode(rng.uniform(-1, 1, N // 2), scale, 10), scale, 5 + i) for i in range(2)]
    gpu = [ctx.ciphertext(c.data, c.scale) for c in cts]
    for _ in range(9):
        _, level, sc = gpu[0].info()
        one = ctx.encode_scalar(1.0, sc, level)
        for g in gpu:
            ctx.multiply_plain(g, one)
            ctx.rescale_to_next(g)
        cts = hm.drop_chain_levels(o, cts, 1)
        for g, c in zip(gpu, cts):
            assert np.array_equal(g.download(), c.data) and g.scale == c.scale
    assert cts[0].level == 1
    with pytest.raises(hecdna.InvalidArgument, match="end of modulus switching chain reached"):
        ctx.rescale_to_next(gpu[0])


@pytest.fixture(scope="module")
def math_env(orc):
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 10 + [60])
    o = orc.Oracle(N, m)
    sk = o.secret_key(31)
    rk = o.relin_key(sk, 32)
    rng = np.random.default_rng(33)
    x = rng.uniform(0.5, 1.5, N // 2)
    s = rng.uniform(0.3, 1.0, N // 2) * rng.choice([-1.0, 1.0], N // 2)
    scale = 2.0**40
    cts = [o.encrypt(sk, o.encode(v, scale, 10), scale, 34 + i) for i, v in enumerate((x, s, x[::-1].copy()))]
    return N, m, o, sk, rk, x, s, cts


@pytest.mark.parametrize("iters", [1, 3])
def test_demo_he_math(demo, math_env, tmp_path, iters):
    N, m, o, sk, rk, x, s, cts = math_env
    out = run(demo, f"math:{iters}", tmp_path, N, m, cts[:2], rk, {})
    exp = [hm.signed_inv(o, rk, cts[0], 1.0, iters), hm.inv_sqrt_twice(o, rk, cts[0], 0.7, iters),
           hm.sqrt(o, rk, cts[0], 1.0, iters), hm.abs_(o, rk, cts[1], 1.0, iters)]
    assert len(out) == 4
    for g, e in zip(out, exp):
        same(g, e)
    if iters == 3:
        dec = [o.decode(o.decrypt(sk, e), e.scale).real for e in exp]
        assert np.max(np.abs(dec[0] - 1 / x)) < 1e-2
        assert np.max(np.abs(dec[1] - 1 / np.sqrt(2 * x))) < 2e-2
        assert np.max(np.abs(dec[2] - np.sqrt(x))) < 2e-2
        assert np.max(np.abs(dec[3] - np.abs(s))) < 0.15


def test_demo_he_util(demo, math_env, tmp_path):
    import subprocess
    from test_gpu_cpp_facade import read_output, write_input
    N, m, o, sk, rk, x, s, cts = math_env
    inp, outp = str(tmp_path / "util.in"), str(tmp_path / "util.out")
    write_input(inp, N, m, cts, rk, {})
    txt = subprocess.check_output([demo, "util", inp, outp]).decode()
    out = read_output(outp, N)
    (d0,) = hm.drop_chain_levels(o, [cts[0]], 2)
    d1, d2 = hm.reach_chain_level(o, [cts[1], cts[2]], d0)
    for g, e in zip(out, [d0, d1, d2]):
        same(g, e)
    # SEAL's chain walk from the key level: key K-1, first K-2, ..., last 0, and
    # key_context_data()->next_context_data() is first_context_data()
    K = len(m)
    chain = next(line for line in txt.splitlines() if line.startswith("chain "))
    assert chain == "chain " + " ".join(str(i) for i in range(K - 1, -1, -1)) + " first %d key_next 1" % (K - 2)


def test_demo_least_squares(demo, orc, tmp_path):
    """the reference's bench_he_least_squares_2d after encryption (matrix_operations.cpp:915-1003; its data
    :890-891), at N = 2^11 with its 17-prime chain {60, 40 x 15, 60}: sum_elems, square, ct x ct with relin, scalar
    encodes at ciphertext parms_ids, signed_inv(0.05, 6), reach_chain_level over a vector of pointers"""
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 15 + [60])
    o = orc.Oracle(N, m)
    sk = o.secret_key(41)
    rk = o.relin_key(sk, 42)
    gk = o.galois_keys(sk, [o.elt_from_step(k) for k in (1, 2, 4)], 43)
    xs = np.array([6, 5.8, 6.5, 5.4, 6.8])
    ys = np.array([2, 1.4, 2.4, 1.5, 2.4])
    scale = 2.0**40
    cx = o.encrypt(sk, o.encode(xs, scale, 16), scale, 44)
    cy = o.encrypt(sk, o.encode(ys, scale, 16), scale, 45)
    out = run(demo, "least_squares", tmp_path, N, m, [cx, cy], rk, gk)
    exp = hm.least_squares_2d(o, rk, gk, cx, cy, 5)
    assert len(out) == 6
    for g, e in zip(out, exp):
        same(g, e)
    n = 5
    denom = n * np.sum(xs * xs) - np.sum(xs) ** 2
    a = (n * np.sum(xs * ys) - np.sum(xs) * np.sum(ys)) / denom
    b = (np.sum(ys) * np.sum(xs * xs) - np.sum(xs) * np.sum(xs * ys)) / denom
    got = [o.decode(o.decrypt(sk, e), e.scale).real[0] for e in exp]
    assert abs(got[4] - a) < 1e-3 and abs(got[5] - b) < 1e-2
