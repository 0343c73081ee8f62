"""GPU CKKS encoder (hec_encode) vs the oracle's encode() on the same values, bit-exact.
Both restate SEAL 4.1's CKKSEncoder::encode_internal operation for operation (matrix_reps_index_map_ scatter,
DWTHandler::transform_from_rev over inv_root_powers_ with fix = scale / N in the last layer, std::round, residues,
NTT); the oracle's restatement is pinned to an independent pure-Python one and to the reference binary's code read
as data (tests/test_oracle_encode.py), so these plaintexts are SEAL's to the extent that reading pins them (no SEAL
vectors exist here)."""
import numpy as np
import pytest

from test_gpu_parity import Env, _ctpt_oracle, env11, env15  # noqa: F401  (module fixtures)

pytestmark = pytest.mark.gpu


def _check(e, vals, scale, level):
    vals = np.asarray(vals)
    rows = vals if vals.ndim == 2 else vals.reshape(1, -1)
    got = e.ctx.encode(rows, scale, level)
    for r, g in zip(rows, got):
        assert g.info() == (level, scale)
        assert np.array_equal(g.download(), e.o.encode(r, scale, level))


@pytest.mark.parametrize("N,bits", [(1 << 10, [50, 36, 36, 50]), (1 << 11, [50, 36, 36, 50]),
                                    (1 << 13, [60, 40, 40, 60])])
def test_encode_bitexact_small(orc, hecdna, N, bits):
    e = Env(orc, hecdna, N, bits, seed=3, elts=[])
    rng = np.random.default_rng(N)
    L = len(bits) - 1
    _check(e, rng.uniform(-1, 1, (3, N // 2)), 2.0**40, L)                      # real, all slots
    z = rng.uniform(-1, 1, (2, N // 2)) + 1j * rng.uniform(-1, 1, (2, N // 2))
    _check(e, z, 2.0**30, L)                                                   # complex
    _check(e, rng.uniform(-100, 100, (2, 37)), 2.0**25, L - 1)                 # few slots, lower level
    _check(e, np.zeros((1, 4)), 2.0**40, L)                                    # all zero
    _check(e, rng.uniform(-1e3, 1e3, (2, N // 2)), 2.0**62, L)                 # coefficients beyond 2^64


def test_encode_reference_data_cfg1(orc, hecdna):
    """The reference demo's matrix (matrix_operations.cpp:1079-1087, values up to 4097) at cfg1."""
    from _helpers import reference_matrix, col_vector
    N = 1 << 13
    e = Env(orc, hecdna, N, [60, 40, 40, 60], seed=5, elts=[])
    M = reference_matrix(64)
    cols = np.stack([col_vector(M[:, c], N // 2) for c in range(0, 64, 9)])
    _check(e, cols, 2.0**40, 3)


@pytest.mark.parametrize("logN,L", [(15, 10), (16, 16)])
def test_encode_bitexact_full_size(orc, hecdna, logN, L):
    """BASELINE cfg2/3 (N = 2^15, l = 10) and cfg5 (N = 2^16, l = 16): the register-held FFT tail runs
    4 and 5 stages."""
    N = 1 << logN
    bits = [60] + [40] * (L - 1) + [60]
    e = Env(orc, hecdna, N, bits, seed=11, elts=[])
    rng = np.random.default_rng(logN)
    _check(e, rng.uniform(-1, 1, (2, N // 2)) + 1j * rng.uniform(-1, 1, (2, N // 2)), 2.0**40, L)


def test_encode_errors_follow_oracle(orc, hecdna):
    e = Env(orc, hecdna, 1 << 11, [50, 36, 36, 50], seed=3, elts=[])
    with pytest.raises(hecdna.HecError, match="values has invalid size"):
        e.ctx.encode(np.zeros((1, (1 << 10) + 1)), 2.0**30, 3)
    with pytest.raises(hecdna.HecError, match="scale out of bounds"):
        e.ctx.encode(np.zeros((1, 8)), 2.0**130, 3)
    with pytest.raises(hecdna.HecError, match="parms_id is not valid"):
        e.ctx.encode(np.zeros((1, 8)), 2.0**30, 4)
    with pytest.raises(hecdna.HecError, match="encoded values are too large"):
        e.ctx.encode(np.full((1, 8), 1e30), 2.0**40, 3)
    for vals, scale, level in [(np.zeros((1 << 10) + 1), 2.0**30, 3), (np.full(8, 1e30), 2.0**40, 3)]:
        with pytest.raises(orc.OracleError):
            e.o.encode(vals, scale, level)
    for bad in (np.nan, np.inf, -np.inf):          # non-finite input: both sides raise the same error
        v = np.zeros((1, 8))
        v[0, 5] = bad
        with pytest.raises(hecdna.HecError, match="encoded values are too large"):
            e.ctx.encode(v, 2.0**40, 3)
        with pytest.raises(orc.OracleError, match="encoded values are too large"):
            e.o.encode(v[0], 2.0**40, 3)


@pytest.mark.parametrize("which,n", [("env11", 9), ("env15", 4)])
def test_matvec_ct_x_pt_gpu_encoded_diagonals(request, which, n):
    """The ct x pt matvec with its plaintext diagonals encoded on the GPU equals the oracle's SEAL flow
    (oracle encode, rotate, multiply_plain, add, rescale)."""
    e = request.getfixturevalue(which)
    L = len(e.m) - 1
    pscale = 2.0**40
    vals = e.rng.uniform(-1, 1, (n, e.N // 2))
    P = [e.o.encode(v, pscale, L) for v in vals]
    X = [e.enc(seed=760 + i) for i in range(2)]
    exp = _ctpt_oracle(e, P, pscale, X)
    got = e.ctx.matmul_diagpt_col(e.ctx.encode(vals, pscale, L), [e.up(x) for x in X], e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)
