"""The oracle's CKKS encoder is SEAL 4.1's CKKSEncoder::encode_internal operation for operation (oracle/oracle.cpp,
each step checked against the reference's build/demo read as data).  Pinned here (CPU):

- against an independent pure-Python restatement of the same SEAL source sequence (matrix_reps_index_map_,
  ComplexRoots + get_root symmetry, inv_root_powers_, DWTHandler::transform_from_rev with fix = scale / N folded
  into the last layer, __muldc3 products, std::round, negate_uint_mod), bit for bit at small N: Python floats are
  IEEE doubles and math.cos / math.sin are the same glibc calls;
- the root tables against exp(2 pi i k / 2N) (the symmetry logic), and the slot map against the Galois generator 3;
- decode(encode(v)) = v within 2^-30 relative (the decoder is the oracle's independent CRT + FFT restatement).
"""
import math

import numpy as np
import pytest


def _bitrev(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def seal_tables(N):
    """CKKSEncoder::CKKSEncoder: matrix_reps_index_map_ and inv_root_powers_ (ComplexRoots(2N), get_root)."""
    logn, m, slots = N.bit_length() - 1, 2 * N, N // 2
    idx = [0] * N
    pos = 1
    for i in range(slots):
        idx[i] = _bitrev((pos - 1) >> 1, logn)
        idx[slots | i] = _bitrev((m - pos - 1) >> 1, logn)
        pos = (pos * 3) & (m - 1)
    roots = [(math.cos(t), math.sin(t)) for t in ((i * 6.283185307179586) / m for i in range(m // 8 + 1))]

    def get_root(k):
        k &= m - 1
        if k <= m // 8:
            return roots[k]
        if k <= m // 4:
            a = roots[m // 4 - k]
            return (a[1], a[0])
        if k <= m // 2:
            a = get_root(m // 2 - k)
            return (-a[0], a[1])
        if k <= 3 * m // 4:
            a = get_root(k - m // 2)
            return (-a[0], -a[1])
        a = get_root(m - k)
        return (a[0], -a[1])
    inv = [(0.0, 0.0)] + [None] * (N - 1)
    for i in range(1, N):
        r = get_root(_bitrev(i - 1, logn) + 1)
        inv[i] = (r[0], -r[1])
    return idx, inv


def _mul(x, w):  # __muldc3, finite operands
    return (x[0] * w[0] - x[1] * w[1], x[0] * w[1] + x[1] * w[0])


def seal_encode_coeffs(N, values, scale):
    """encode_internal up to the rounded coefficients (pure Python)."""
    idx, inv = seal_tables(N)
    slots = N // 2
    v = [(0.0, 0.0)] * N
    for i, z in enumerate(values):
        z = complex(z)
        v[idx[i]] = (z.real, z.imag)
        v[idx[i + slots]] = (z.real, -z.imag)
    fix = scale / N
    gap, m, r = 1, N >> 1, 0
    while m > 1:
        off = 0
        for _ in range(m):
            r += 1
            w = inv[r]
            for j in range(off, off + gap):
                u, t = v[j], v[j + gap]
                v[j] = (u[0] + t[0], u[1] + t[1])
                v[j + gap] = _mul((u[0] - t[0], u[1] - t[1]), w)
            off += gap << 1
        gap <<= 1
        m >>= 1
    w = inv[r + 1]
    sw = (w[0] * fix, w[1] * fix)
    for j in range(gap):
        u, t = v[j], v[j + gap]
        v[j] = ((u[0] + t[0]) * fix, (u[1] + t[1]) * fix)
        v[j + gap] = _mul((u[0] - t[0], u[1] - t[1]), sw)
    return [float(np.round(x[0])) for x in v], max(abs(x[0]) for x in v)


def _residues(coeffs, q):
    out = []
    for c in coeffs:
        a = abs(int(c))
        rr = a % q
        out.append(q - rr if (math.copysign(1.0, c) < 0 and rr) else rr)
    return np.array(out, dtype=np.uint64)


@pytest.mark.parametrize("N,bits,scale,kind", [(1 << 10, [50, 36, 36, 50], 2.0**40, "real"),
                                               (1 << 11, [60, 40, 40, 60], 2.0**40, "complex"),
                                               (1 << 11, [50, 36, 36, 50], 2.0**25, "few"),
                                               (1 << 10, [60, 50, 50, 60], 2.0**70, "wide")])
def test_oracle_encode_equals_python_restatement(orc, N, bits, scale, kind):
    m = orc.Oracle.create_coeff_modulus(N, bits)
    o = orc.Oracle(N, m)
    rng = np.random.default_rng(N + len(kind))
    vals = {"real": lambda: rng.uniform(-1, 1, N // 2),
            "complex": lambda: rng.uniform(-1, 1, N // 2) + 1j * rng.uniform(-1, 1, N // 2),
            "few": lambda: rng.uniform(-100, 100, 37),
            "wide": lambda: rng.uniform(-1e3, 1e3, N // 2)}[kind]()   # coefficients beyond 2^64: SEAL's wide paths
    L = len(m) - 1
    coeffs, mx = seal_encode_coeffs(N, list(vals), scale)
    if kind == "wide":
        assert mx > 2.0**64
    exp = np.stack([o.ntt_fwd(i, _residues(coeffs, m[i])) for i in range(L)])
    assert np.array_equal(o.encode(vals, scale, L), exp)


def test_root_tables_and_slot_map(orc):
    N = 1 << 12
    idx, inv = seal_tables(N)
    m, logn = 2 * N, 11 + 1
    for i in range(1, N):
        k = _bitrev(i - 1, logn) + 1
        ref = np.conj(np.exp(2j * np.pi * k / m))
        assert abs(complex(*inv[i]) - ref) < 1e-15
    assert sorted(idx) == list(range(N))                        # a permutation of the N positions
    pos = 1
    for i in range(N // 2):                                     # slot i <-> 3^i mod 2N (generator 3), bit-reversed
        assert idx[i] == _bitrev((pos - 1) >> 1, logn)
        pos = pos * 3 % m


@pytest.mark.parametrize("N", [1 << 11, 1 << 13])
def test_encode_decode_round_trip(orc, N):
    m = orc.Oracle.create_coeff_modulus(N, [60, 40, 40, 60])
    o = orc.Oracle(N, m)
    rng = np.random.default_rng(7)
    v = rng.uniform(-1, 1, N // 2) + 1j * rng.uniform(-1, 1, N // 2)
    d = o.decode(o.encode(v, 2.0**40, 3), 2.0**40)
    assert np.max(np.abs(d - v)) < 2.0**-30


def test_encode_too_large_uses_unrounded_maximum(orc):
    """SEAL's bound: ceil(log2(max(max |Re|, 1))) + 1 >= total coeff-modulus bits -> "encoded values are too large"."""
    N = 1 << 10
    m = orc.Oracle.create_coeff_modulus(N, [30, 20, 30])
    o = orc.Oracle(N, m)
    with pytest.raises(orc.OracleError, match="encoded values are too large"):
        o.encode(np.full(8, 2.0**40), 2.0**20, 2)
    o.encode(np.full(8, 2.0**10), 2.0**20, 2)


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf, complex(0.5, np.nan)])
def test_encode_rejects_non_finite(orc, bad):
    """A NaN or infinite slot value is "encoded values are too large", as the GPU encoder reports it (no cast of a
    non-finite double to an integer)."""
    N = 1 << 10
    o = orc.Oracle(N, orc.Oracle.create_coeff_modulus(N, [30, 20, 30]))
    v = np.zeros(8, dtype=complex)
    v[3] = bad
    with pytest.raises(orc.OracleError, match="encoded values are too large"):
        o.encode(v, 2.0**20, 2)


def _scalar_reference(value, scale, moduli, level, N):
    """SEAL 4.1 CKKSEncoder::encode_internal(double, ...) in Python integers: round(value * scale) as the exact integer
    the double holds, its residue per prime (negated when negative), every coefficient of the NTT-form limb."""
    import math
    v = value * scale
    c = round(v) if abs(v - math.trunc(v)) != 0.5 else (math.trunc(v) + (1 if v > 0 else -1))  # std::round: half away
    out = np.zeros((level, N), dtype=np.uint64)
    for j in range(level):
        out[j] = c % moduli[j]
    return out


@pytest.mark.parametrize("value,scale", [(1.0, 2.0**40), (-0.05**2, 2.0**40), (2 * 0.05, 2.0**30), (3.0 / 2, 2.0**40),
                                         (0.0, 2.0**40), (-1.0, 2.0**40), (5.0, 2.0**40), (1.4142135623730951, 2.0**40),
                                         (-3.7e9, 2.0**40), (1e20, 2.0**62), (-7.5e22, 2.0**62), (0.5, 1.0),
                                         (-2.5, 1.0)])
def test_encode_scalar_matches_integer_restatement(orc, value, scale):
    """encode_scalar: the 64-bit, 128-bit and multi-word cases (|value scale| up to 2^138 at 17 primes) against Python's
    exact integers; std::round rounds halves away from zero"""
    N = 1 << 10
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 15 + [60])
    o = orc.Oracle(N, m)
    L = len(m) - 1
    for level in (L, 3, 1):
        if abs(value * scale) >= 2.0 ** (sum(q.bit_length() for q in m[:level]) - 2):
            continue
        assert np.array_equal(o.encode_scalar(value, scale, level), _scalar_reference(value, scale, m, level, N))


def test_encode_scalar_decodes_to_constant_and_errors(orc):
    N = 1 << 10
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
    o = orc.Oracle(N, m)
    pt = o.encode_scalar(-0.3125, 2.0**30, 3)
    d = o.decode(pt, 2.0**30)
    assert np.max(np.abs(d - (-0.3125))) < 2.0**-25
    with pytest.raises(orc.OracleError, match="encoded value is too large"):
        o.encode_scalar(2.0**100, 2.0**30, 3)
    with pytest.raises(orc.OracleError, match="encoded value is too large"):
        o.encode_scalar(float("nan"), 2.0**30, 3)
    with pytest.raises(orc.OracleError, match="scale out of bounds"):
        o.encode_scalar(1.0, 2.0**125, 3)
    with pytest.raises(orc.OracleError, match="parms_id is not valid"):
        o.encode_scalar(1.0, 2.0**30, 4)
