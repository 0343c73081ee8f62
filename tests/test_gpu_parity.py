"""GPU parity: every HIP path through the C-ABI vs the CPU oracle on the same seeded inputs, bit-exact
(integer work: SURVEY §8(c)).  Run on the MI355X box with `pytest -m gpu`."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a, scale=None):
    h = hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes())
    if scale is not None:
        h.update(np.float64(scale).tobytes())
    return h.hexdigest()


class Env:
    """Oracle + GPU context over the same parameters and the same keys."""

    def __init__(self, orc, hecdna, N, bits, seed=7, elts=None):
        self.orc, self.hec = orc, hecdna
        self.m = orc.Oracle.create_coeff_modulus(N, bits)
        self.o = orc.Oracle(N, self.m)
        self.N = N
        self.ctx = hecdna.Context(N, self.m)
        self.sk = self.o.secret_key(seed)
        self.rk_h = self.o.relin_key(self.sk, seed + 1)
        self.elts = elts if elts is not None else self.o.default_galois_elts()
        self.gk_h = self.o.galois_keys(self.sk, self.elts, seed + 2)
        self.rk = self.ctx.relin_key(self.rk_h)
        self.gk = self.ctx.galois_keys(self.gk_h)
        self.rng = np.random.default_rng(seed)

    def enc(self, vals=None, level=None, scale=2.0**40, seed=0):
        level = level or len(self.m) - 1
        if vals is None:
            vals = self.rng.uniform(-1, 1, self.N // 2)
        pt = self.o.encode(vals, scale, level)
        return self.o.encrypt(self.sk, pt, scale, 1000 + seed)

    def rand_ct(self, size, level, scale=2.0**40):
        d = np.stack([np.stack([self.rng.integers(0, self.m[i], self.N, dtype=np.uint64) for i in range(level)])
                      for _ in range(size)])
        return self.orc.Ct(d, scale)

    def up(self, ct):
        return self.ctx.ciphertext(ct.data, ct.scale)

    def same(self, g, ct):
        s, l, sc = g.info()
        assert (s, l) == (ct.size, ct.level)
        assert sc == ct.scale
        assert np.array_equal(g.download(), ct.data)


@pytest.fixture(scope="module")
def env11(orc, hecdna):
    return Env(orc, hecdna, 1 << 11, [50, 36, 36, 50])


@pytest.fixture(scope="module")
def env15(orc, hecdna):
    # BASELINE cfg2/cfg3 parameters: N = 2^15, {60, 40 x 9, 60}; keys only for what the tests rotate by
    return Env(orc, hecdna, 1 << 15, [60] + [40] * 9 + [60], seed=99, elts=None)


# ------------------------------------------------------------------------------- NTT ----
@pytest.mark.parametrize("logN", [10, 11, 12, 13, 14, 15, 16])
def test_ntt_bitexact(orc, hecdna, logN):
    N = 1 << logN
    bits = [60, 40, 50, 60] if logN < 16 else [60, 40, 60]
    m = orc.Oracle.create_coeff_modulus(N, bits)
    o = orc.Oracle(N, m)
    ctx = hecdna.Context(N, m)
    rng = np.random.default_rng(logN)
    K = len(m)
    a = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m]) for _ in range(3)])
    fwd = ctx.ntt(a)
    exp = np.stack([np.stack([o.ntt_fwd(i, a[p, i]) for i in range(K)]) for p in range(3)])
    assert np.array_equal(fwd, exp)
    assert np.array_equal(ctx.ntt(fwd, inverse=True), a)
    # limb offset: limbs 1..K-1 only
    sub = np.ascontiguousarray(a[:, 1:])
    assert np.array_equal(ctx.ntt(sub, limb0=1), exp[:, 1:])


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("logN", [13, 14, 15, 16])
def test_ntt_pass_b_shuffle_bitexact(orc, hecdna, logN, mode):
    """The opt-in wave-shuffle forward pass B (hec_context_set_option "nttb_shfl"; k_nttb_shfl, 128-point columns
    exchanged through DPP lane moves instead of LDS; mode 2 swaps back to coalesced stores) gives the oracle's bits
    wherever it applies (128-point pass B), and the LDS pass elsewhere."""
    N = 1 << logN
    bits = [60, 40, 50, 60] if logN < 16 else [60, 40, 60]
    m = orc.Oracle.create_coeff_modulus(N, bits)
    o = orc.Oracle(N, m)
    ctx = hecdna.Context(N, m)
    ctx.set_option("nttb_shfl", mode)
    rng = np.random.default_rng(700 + logN)
    a = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m]) for _ in range(2)])
    exp = np.stack([np.stack([o.ntt_fwd(i, a[p, i]) for i in range(len(m))]) for p in range(2)])
    fwd = ctx.ntt(a)
    assert np.array_equal(fwd, exp)
    assert np.array_equal(ctx.ntt(fwd, inverse=True), a)
    assert np.array_equal(ctx.ntt(np.ascontiguousarray(a[:, 1:]), limb0=1), exp[:, 1:])


@pytest.mark.parametrize("mode,dr", [(1, 0), (2, 0), (2, 1)])
def test_cfg3_shuffle_pass_b_keyswitch_bitexact(env15, mode, dr):
    """cfg3 parameters with the wave-shuffle pass B on (the mod-up digits' forward transforms; dr: the mod-down's
    divide-and-round pass B too): rotations and a small hoisted matvec equal the oracle's bits."""
    e = env15
    e.ctx.set_option("nttb_shfl", mode)
    e.ctx.set_option("nttb_shfl_dr", dr)
    try:
        a = e.enc(seed=5)
        for steps in (1, 4095):
            e.same(e.ctx.rotate_vector(e.up(a), steps, e.gk), e.o.rotate(a, steps, e.gk_h))
        A = [e.enc(seed=60 + j) for j in range(5)]
        X = [e.enc(seed=90 + i) for i in range(2)]
        exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h, nthreads=8)
        got = e.ctx.matmul_diag_col([e.up(x) for x in A], [e.up(x) for x in X], e.rk, e.gk)
        for g, c in zip(got, exp):
            e.same(g, c)
        low = e.enc(seed=9, level=4)  # a lower level: fewer digits and targets
        e.same(e.ctx.rotate_vector(e.up(low), 3, e.gk), e.o.rotate(low, 3, e.gk_h))
    finally:
        e.ctx.set_option("nttb_shfl", 0)
        e.ctx.set_option("nttb_shfl_dr", 0)


def test_cfg3_single_pass_moddown_bitexact(env15):
    """cfg3 parameters with the single-pass mod-down (hec_context_set_option "moddown1"; k_moddown1: the rounding limb,
    its whole forward NTT and the divide-and-round in one kernel per data limb, FP64 and 60-bit classes): rotations
    (the per-rotation path, IN read through the permutation) and a hoisted matvec (sibling-group mod-downs) equal the
    oracle's bits."""
    e = env15
    e.ctx.set_option("moddown1", 1)
    try:
        a = e.enc(seed=7)
        for steps in (1, 3, 4095):
            e.same(e.ctx.rotate_vector(e.up(a), steps, e.gk), e.o.rotate(a, steps, e.gk_h))
        A = [e.enc(seed=70 + j) for j in range(6)]
        X = [e.enc(seed=95 + i) for i in range(3)]
        exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h, nthreads=8)
        got = e.ctx.matmul_diag_col([e.up(x) for x in A], [e.up(x) for x in X], e.rk, e.gk)
        for g, c in zip(got, exp):
            e.same(g, c)
        # a lower level (l = 4: fewer data limbs, the same special prime)
        low = e.enc(seed=8, level=4)
        for steps in (1, 5):
            e.same(e.ctx.rotate_vector(e.up(low), steps, e.gk), e.o.rotate(low, steps, e.gk_h))
    finally:
        e.ctx.set_option("moddown1", 0)


def test_objects_outlive_their_context(orc, hecdna):
    """Objects destroyed after their context (SEAL's objects hold the context by shared_ptr, and a garbage collector
    finalising a reference cycle picks its own order; r06 suite: a Galois key set finalised after its context read
    the freed context): each destroy frees its own device memory and touches the context only while it is alive.
    Then a new context (possibly at the same address) works, and its objects still sync on it."""
    import gc
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
    for round_ in range(3):
        ctx = hecdna.Context(N, m)
        rng = np.random.default_rng(round_)
        data = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m[:3]]) for _ in range(2)])
        ct = ctx.ciphertext(data, 2.0 ** 30)
        pt = ctx.plaintext(data[0], 2.0 ** 30)
        rk = ctx.relin_key(seed=11)
        o = orc.Oracle(N, m)
        gk = ctx.galois_keys(uniform_elts=[o.elt_from_step(1)], seed=5)
        ctx.close()
        del ct, pt, rk, gk
        gc.collect()
    ctx = hecdna.Context(N, m)
    a = np.stack([np.stack([np.random.default_rng(9).integers(0, q, N, dtype=np.uint64) for q in m])])
    o = orc.Oracle(N, m)
    assert np.array_equal(ctx.ntt(a)[0], np.stack([o.ntt_fwd(i, a[0, i]) for i in range(len(m))]))
    ct = ctx.ciphertext(np.zeros((2, 3, N), np.uint64), 1.0)
    del ct
    gc.collect()


def test_ntt_cfg2_golden(orc, hecdna):
    fx = json.load(open(os.path.join(GOLD, "cfg2_ntt.json")))
    N, m = fx["N"], fx["moduli"]
    rng = np.random.default_rng(fx["rng_seed"])
    data = np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m])
    assert sha(data) == fx["input_sha256"]
    ctx = hecdna.Context(N, m)
    out = ctx.ntt(data[None])[0]
    assert [sha(out[i]) for i in range(len(m))] == fx["forward_sha256"]


def test_cfg2_device_pipeline_bitexact(orc, hecdna):
    """bench.py --config cfg2's step on device-resident buffers (Context.ntt_device / dyadic_device: the forward NTT
    in place, the dyadic product into a third buffer, its inverse NTT in place) equals the oracle's
    ntt_fwd -> (a * b) mod q -> ntt_inv, limb by limb, at N = 2^15 over the 10 data primes."""
    N, nl, npolys = 1 << 15, 10, 3
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 9 + [60])
    o = orc.Oracle(N, m)
    ctx = hecdna.Context(N, m)
    rng = np.random.default_rng(22)
    a = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m[:nl]]) for _ in range(npolys)])
    b = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m[:nl]]) for _ in range(npolys)])
    bufs = [hecdna.DeviceBuffer(ctx, a.nbytes) for _ in range(3)]
    bufs[0].upload(a)
    bufs[1].upload(b)
    ctx.ntt_device(bufs[0], nl, npolys)
    ctx.dyadic_device(bufs[0], bufs[1], bufs[2], nl, npolys)
    ctx.ntt_device(bufs[2], nl, npolys, inverse=True)
    ctx.synchronize()
    fa = bufs[0].download(a.shape)
    out = bufs[2].download(a.shape)
    exp_f = np.stack([np.stack([o.ntt_fwd(i, a[p, i]) for i in range(nl)]) for p in range(npolys)])
    assert np.array_equal(fa, exp_f)
    q = np.array(m[:nl], dtype=object).reshape(1, nl, 1)
    prod = (exp_f.astype(object) * b.astype(object) % q).astype(np.uint64)
    exp = np.stack([np.stack([o.ntt_inv(i, prod[p, i]) for i in range(nl)]) for p in range(npolys)])
    assert np.array_equal(out, exp)


def test_dyadic_multiply_cfg2(orc, hecdna):
    """BASELINE cfg2 primitive: dyadic_product_coeffmod over u64[npolys][10][2^15] (the 10 data primes of
    {60, 40 x 9, 60}) through hec_dyadic_multiply, and at a limb offset; equal to (a * b) mod q_i."""
    N = 1 << 15
    m = orc.Oracle.create_coeff_modulus(N, [60] + [40] * 9 + [60])
    ctx = hecdna.Context(N, m)
    rng = np.random.default_rng(15)
    a = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m[:10]]) for _ in range(3)])
    b = np.stack([np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m[:10]]) for _ in range(3)])
    q = np.array(m[:10], dtype=object).reshape(1, 10, 1)
    exp = (a.astype(object) * b.astype(object) % q).astype(np.uint64)
    assert np.array_equal(ctx.dyadic_multiply(a, b), exp)
    sub_a, sub_b = np.ascontiguousarray(a[:, 4:]), np.ascontiguousarray(b[:, 4:])
    assert np.array_equal(ctx.dyadic_multiply(sub_a, sub_b, limb0=4), exp[:, 4:])


# ------------------------------------------------------------------------------- ops -----
def test_add_sub_negate(env11):
    e = env11
    a, b = e.rand_ct(2, 3), e.rand_ct(2, 3)
    e.same(e.ctx.add(e.up(a), e.up(b)), e.o.add(a, b))
    e.same(e.ctx.sub(e.up(a), e.up(b)), e.o.sub(a, b))
    e.same(e.ctx.negate(e.up(a)), e.o.negate(a))
    c3 = e.rand_ct(3, 3)
    e.same(e.ctx.add(e.up(a), e.up(c3)), e.o.add(a, c3))   # size grows 2 -> 3 (copy extra poly)
    e.same(e.ctx.sub(e.up(a), e.up(c3)), e.o.sub(a, c3))   # extra poly negated
    e.same(e.ctx.add(e.up(c3), e.up(a)), e.o.add(c3, a))


def test_multiply_square_plain(env11):
    e = env11
    a, b = e.rand_ct(2, 3), e.rand_ct(2, 3)
    e.same(e.ctx.multiply(e.up(a), e.up(b)), e.o.multiply(a, b))
    e.same(e.ctx.square(e.up(a)), e.o.square(a))
    c3 = e.rand_ct(3, 3)
    e.same(e.ctx.multiply(e.up(c3), e.up(a)), e.o.multiply(c3, a))
    pt = e.rand_ct(1, 3).data[0]
    p = e.ctx.plaintext(pt, 2.0**40)
    e.same(e.ctx.multiply_plain(e.up(a), p), e.o.multiply_plain(a, pt, 2.0**40))
    e.same(e.ctx.add_plain(e.up(a), p), e.o.add_plain(a, pt, 2.0**40))
    e.same(e.ctx.sub_plain(e.up(a), p), e.o.sub_plain(a, pt, 2.0**40))


def test_relinearize_rescale_modswitch(env11):
    e = env11
    for level in (3, 2):
        c3 = e.rand_ct(3, level, 2.0**60)
        e.same(e.ctx.relinearize(e.up(c3), e.rk), e.o.relinearize(c3, e.rk_h))
        e.same(e.ctx.rescale_to_next(e.up(c3)), e.o.rescale(c3))
        c2 = e.rand_ct(2, level, 2.0**40)
        e.same(e.ctx.rescale_to_next(e.up(c2)), e.o.rescale(c2))
        e.same(e.ctx.mod_switch_to_next(e.up(c2)), e.o.mod_switch(c2))


@pytest.mark.parametrize("steps", [1, 2, 3, 5, 7, -1, -6, 100, 255, 511, -511, 333])
def test_rotate(env11, steps):
    e = env11
    a = e.rand_ct(2, 3)
    e.same(e.ctx.rotate_vector(e.up(a), steps, e.gk), e.o.rotate(a, steps, e.gk_h))


def test_apply_galois_conjugate(env11):
    e = env11
    a = e.rand_ct(2, 2)
    elt = 2 * e.N - 1
    e.same(e.ctx.apply_galois(e.up(a), elt, e.gk), e.o.apply_galois(a, elt, e.gk_h))


def test_rotation_decrypts(env11):
    e = env11
    v = e.rng.uniform(-1, 1, e.N // 2)
    g = e.up(e.enc(v))
    e.ctx.rotate_vector(g, 37, e.gk)
    ct = e.orc.Ct(g.download(), g.scale)
    d = e.o.decode(e.o.decrypt(e.sk, ct), ct.scale).real
    assert np.max(np.abs(d - np.roll(v, -37))) < 1e-5


def test_errors_follow_seal(env11, hecdna):
    e = env11
    a = e.up(e.rand_ct(2, 3, 2.0**40))
    b = e.up(e.rand_ct(2, 3, 2.0**41))
    with pytest.raises(hecdna.InvalidArgument, match="scale mismatch"):
        e.ctx.add(a, b)
    with pytest.raises(hecdna.InvalidArgument, match="parameter mismatch"):
        e.ctx.add(a, e.up(e.rand_ct(2, 2)))
    with pytest.raises(hecdna.InvalidArgument, match="end of modulus switching chain reached"):
        e.ctx.rescale_to_next(e.up(e.rand_ct(2, 1)))
    empty = e.ctx.galois_keys({})
    with pytest.raises(hecdna.InvalidArgument, match="Galois key not present"):
        e.ctx.rotate_vector(a, 1, empty)
    with pytest.raises(hecdna.InvalidArgument, match="step count too large"):
        e.ctx.rotate_vector(a, e.N // 2, e.gk)
    with pytest.raises(hecdna.InvalidArgument, match="scale out of bounds"):
        e.ctx.multiply(e.up(e.rand_ct(2, 3, 2.0**70)), e.up(e.rand_ct(2, 3, 2.0**70)))
    with pytest.raises(hecdna.InvalidArgument, match="encrypted size must be 2"):
        e.ctx.rotate_vector(e.up(e.rand_ct(3, 3)), 1, e.gk)


# ------------------------------------------------------------------------------- linalg --
def test_matvec_cfg1_golden(orc, hecdna):
    """The reference demo (matrix_operations.cpp:1042-1175, COL_OR_DIAG=1): all 64 output
    ciphertexts of the 64x64 diag x col product byte-identical to the oracle's golden hashes."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import cfg1_inputs, sha as gsha
    fx = json.load(open(os.path.join(GOLD, "cfg1_matvec.json")))
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    assert [gsha(c.data, c.scale) for c in cts] == fx["input_sha256"]
    ctx = hecdna.Context(fx["N"], m)
    g = [ctx.ciphertext(c.data, c.scale) for c in cts]
    out = ctx.matmul_diag_col(g, g, ctx.relin_key(rk), ctx.galois_keys(gk))
    hashes = [gsha(x.download(), x.scale) for x in out]
    assert hashes == fx["output_sha256"]


def test_matmul_col_colT_cfg1_golden(orc, hecdna):
    """The reference demo's compiled default, COL_OR_DIAG = 0 (matrix_operations.cpp:1123-1128): col-batched A
    times B = A^T, i.e. out[i] = sum_j rot(A[j], i) (*) A[j] on the 64x64 cfg1 data; all 64 diagonal outputs
    byte-identical to the golden hashes."""
    import sys
    sys.path.insert(0, GOLD)
    from make_golden import cfg1_inputs, sha as gsha
    fx = json.load(open(os.path.join(GOLD, "cfg1_colcolT.json")))
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    ctx = hecdna.Context(fx["N"], m)
    g = [ctx.ciphertext(c.data, c.scale) for c in cts]
    out = ctx.matmul_col_colT(g, g, fx["n"], ctx.relin_key(rk), ctx.galois_keys(gk))
    assert [gsha(x.download(), x.scale) for x in out] == fx["output_sha256"]


def test_matvec_batched_equals_single_and_oracle(env11):
    e = env11
    n = 12
    A = [e.enc(seed=j) for j in range(n)]
    X = [e.enc(seed=100 + i) for i in range(3)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
    gA = [e.up(a) for a in A]
    gX = [e.up(x) for x in X]
    got = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)
    one = e.ctx.matmul_diag_col(gA, gX[1:2], e.rk, e.gk)[0]
    e.same(one, exp[1])


@pytest.fixture
def lanes3(env11):
    """The opt-in concurrent batch lanes (hec_context_set_option "lanes"; the default is one lane since round 5)."""
    env11.ctx.set_option("lanes", 3)
    yield env11
    env11.ctx.set_option("lanes", 1)


def test_matvec_batch_lanes_bitexact(lanes3):
    """With lanes on, a batch of >= 32 vectors runs as concurrent lanes (one host thread, HIP stream and workspace
    per lane, hec_engine.hip matvec_lanes): 48 columns -> 3 lanes of 16; every output equals the oracle's."""
    e = lanes3
    n = 10
    A = [e.enc(seed=3000 + j) for j in range(n)]
    X = [e.enc(seed=3100 + i) for i in range(48)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h, nthreads=8)
    got = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)
    # a second call reuses the lanes (their streams, workspaces and the per-key tables)
    got2 = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X[:33]], e.rk, e.gk)
    for g, c in zip(got2, exp[:33]):
        e.same(g, c)
    # profiling runs the whole batch as one lane on the context's own workspace, after returning the idle lanes'
    # workspaces (bench.py's profile step); the lanes then grow theirs again
    e.ctx.profile(2)
    got3 = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    e.ctx.synchronize()
    e.ctx.profile(0)
    got4 = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    for g3, g4, c in zip(got3, got4, exp):
        e.same(g3, c)
        e.same(g4, c)


def test_lane_workspace_growth_while_lanes_run(orc, hecdna):
    """A fresh context: a 3-lane matvec at a small shape, then at a larger one, so each lane grows its workspace
    from its own host thread while the other lanes are launching (the round-2 lane hazard); then the small shape
    again (the outgrown bases were reclaimed after the lanes joined).  Every output equals the oracle's."""
    e = Env(orc, hecdna, 1 << 11, [50, 36, 36, 50], seed=5151)
    e.ctx.set_option("lanes", 3)
    X = [e.enc(seed=5000 + i) for i in range(48)]
    gX = [e.up(x) for x in X]
    for n in (3, 24, 3):
        A = [e.enc(seed=5100 + j) for j in range(n)]
        exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h, nthreads=8)
        got = e.ctx.matmul_diag_col([e.up(a) for a in A], gX, e.rk, e.gk)
        for g, c in zip(got, exp):
            e.same(g, c)


def test_matvec_partial_finish_equals_full(env11):
    e = env11
    n = 10
    A = [e.up(e.enc(seed=j)) for j in range(n)]
    X = [e.up(e.enc(seed=50 + i)) for i in range(2)]
    full = e.ctx.matmul_diag_col(A, X, e.rk, e.gk)
    p1 = e.ctx.matmul_diag_col_partial(A, 0, 4, X, e.gk)
    p2 = e.ctx.matmul_diag_col_partial(A, 4, n, X, e.gk)
    for a, b in zip(p1, p2):
        e.ctx.add(a, b)
    fin = e.ctx.matmul_finish(p1, e.rk)
    for f, g in zip(fin, full):
        assert np.array_equal(f.download(), g.download()) and f.scale == g.scale


def test_matmul_col_colT(env11):
    e = env11
    n, p = 6, 5
    A = [e.enc(seed=j) for j in range(n)]
    B = [e.enc(seed=30 + j) for j in range(n)]
    exp = e.o.matmul_col_colT(A, B, p, e.rk_h, e.gk_h)
    got = e.ctx.matmul_col_colT([e.up(a) for a in A], [e.up(b) for b in B], p, e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


def test_matrix_matmul(env11):
    e = env11
    A = [e.enc(seed=j) for j in range(6)]   # 2x3 column-major
    B = [e.enc(seed=20 + j) for j in range(6)]  # 3x2
    for atr, btr, dims in [(0, 0, (2, 3, 3, 2)), (1, 1, (3, 2, 2, 3))]:
        ar, ac, br, bc = dims
        exp = e.o.matrix_matmul(A, ar, ac, atr, B, br, bc, btr, e.rk_h)
        got = e.ctx.matrix_matmul([e.up(a) for a in A], ar, ac, atr, [e.up(b) for b in B], br, bc, btr, e.rk)
        assert len(got) == len(exp)
        for g, c in zip(got, exp):
            e.same(g, c)


# ------------------------------------------------------------------------------- full size
def test_cfg3_rotations_bitexact(env15):
    """N = 2^15, L = 10 (BASELINE cfg3 parameters): rotations with 1..7 NAF key switches."""
    e = env15
    a = e.enc(seed=1)
    for steps in (1, 3, 4095, -77):
        e.same(e.ctx.rotate_vector(e.up(a), steps, e.gk), e.o.rotate(a, steps, e.gk_h))


def test_cfg3_matvec_small_n_bitexact(env15):
    e = env15
    n = 6
    A = [e.enc(seed=10 + j) for j in range(n)]
    X = [e.enc(seed=40 + i) for i in range(2)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h, nthreads=8)
    got = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


def test_cfg5_params_matvec_bitexact(orc, hecdna):
    """BASELINE cfg5 parameters, N = 2^16 with the 17-prime chain {60, 40 x 15, 60} (l = 16, K = 17;
    SURVEY §8 table): rotations and a small diag x col matvec (hoisted root, NAF rotations, lazy
    relinearize + rescale) bit-exact against the oracle.  Keys only for steps +-1, 2, 4 (a full default
    key set is 8.8 GB on the host)."""
    N = 1 << 16
    bits = [60] + [40] * 15 + [60]
    o = orc.Oracle(N, orc.Oracle.create_coeff_modulus(N, bits))
    elts = [o.elt_from_step(s) for s in (1, -1, 2, 4)]
    e = Env(orc, hecdna, N, bits, seed=161, elts=elts)
    assert len(e.m) == 17
    a = e.enc(seed=1)
    for steps in (1, 3, 5):
        e.same(e.ctx.rotate_vector(e.up(a), steps, e.gk), e.o.rotate(a, steps, e.gk_h))
    A = [e.enc(seed=170 + j) for j in range(5)]
    X = [e.enc(seed=180 + i) for i in range(2)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h, nthreads=8)
    got = e.ctx.matmul_diag_col([e.up(x) for x in A], [e.up(x) for x in X], e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


@pytest.mark.parametrize("env", [{"HEC_FUSED_MODUP_MAC": "0"},
                                 {"HEC_FUSE_GALOIS": "0"}, {"HEC_FUSE_GALOIS": "0", "HEC_FUSED_MODUP_MAC": "0"},
                                 {"HEC_TENSOR_DEFER": "1"}, {"HEC_TENSOR_BUFS": "1"}, {"HEC_TENSOR_DEFER": "3"},
                                 {"HEC_TENSOR_XCD": "1"}, {"HEC_TENSOR_XCD": "3"},
                                 {"HEC_FAN": "0"}, {"HEC_FAN": "1", "HEC_FUSE_GALOIS": "0"},
                                 {"HEC_HOIST": "0"}, {"HEC_HOIST_MIN": "1"}, {"HEC_HOIST_MIN": "1", "HEC_FAN": "0"},
                                 {"HEC_HMAC": "0"}, {"HEC_HMAC": "0", "HEC_HOIST_MIN": "1"},
                                 {"HEC_HMAC": "1"}, {"HEC_HMAC": "1", "HEC_HMAC_ODD3": "0"},
                                 {"HEC_HOIST_SCAN": "0"}, {"HEC_KERNEL_MEMOPS": "0"}, {"HEC_SPLIT_BFLY": "0"},
                                 {"HEC_SPLIT_BFLY": "1"}, {"HEC_SPLIT_BFLY": "3"}, {"HEC_BMAC_SPLIT": "0"},
                                 {"HEC_HMAC_INT": "0"}])
def test_keyswitch_variants_bitexact(orc, hecdna, env):
    """The engine's alternative key-switch schedules (separate mod-up pass B + MAC kernels; the fused
    kernel's key-load placements) give the same bits as the oracle."""
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e = Env(orc, hecdna, 1 << 12, [60, 40, 40, 60], seed=77)  # contexts read the switches at creation
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    A = [e.enc(seed=j) for j in range(6)]
    X = [e.enc(seed=40 + i) for i in range(2)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
    got = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


def _ctpt_oracle(e, P, pscale, X):
    """ct x pt matvec composed from pinned oracle ops: out[i] = rescale(sum_j multiply_plain(rot(X[i], j), P[j]))."""
    outs = []
    for x in X:
        acc = None
        for j, pj in enumerate(P):
            r = x if j == 0 else e.o.rotate(x, j, e.gk_h)
            t = e.o.multiply_plain(r, pj, pscale)
            acc = t if acc is None else e.o.add(acc, t)
        outs.append(e.o.rescale(acc))
    return outs


@pytest.mark.parametrize("which,n", [("env11", 12), ("env15", 5)])
def test_matvec_ct_x_pt_bitexact(request, which, n):
    e = request.getfixturevalue(which)
    L = len(e.m) - 1
    pscale = 2.0**40
    P = [e.o.encode(e.rng.uniform(-1, 1, e.N // 2), pscale, L) for _ in range(n)]
    X = [e.enc(seed=700 + i) for i in range(2)]
    exp = _ctpt_oracle(e, P, pscale, X)
    got = e.ctx.matmul_diagpt_col([e.ctx.plaintext(p, pscale) for p in P], [e.up(x) for x in X], e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


def test_matvec_ct_x_pt_batch_lanes(lanes3):
    """The ct x pt form over 40 vectors (with lanes on: 2 concurrent lanes of 20) equals the oracle's SEAL flow."""
    e = lanes3
    L = len(e.m) - 1
    pscale = 2.0**40
    P = [e.o.encode(e.rng.uniform(-1, 1, e.N // 2), pscale, L) for _ in range(7)]
    X = [e.enc(seed=3300 + i) for i in range(40)]
    exp = _ctpt_oracle(e, P, pscale, X)
    got = e.ctx.matmul_diagpt_col([e.ctx.plaintext(p, pscale) for p in P], [e.up(x) for x in X], e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


def test_matvec_ct_x_pt_errors(env11, hecdna):
    e = env11
    L = len(e.m) - 1
    pts = [e.ctx.plaintext(e.o.encode(e.rng.uniform(-1, 1, e.N // 2), 2.0**40, L - 1), 2.0**40) for _ in range(3)]
    X = [e.up(e.enc(seed=800))]
    with pytest.raises(hecdna.InvalidArgument, match="parameter mismatch"):
        e.ctx.matmul_diagpt_col(pts, X, e.gk)


# ----------------------------------------------------------------- matvec edge cases --
def test_matvec_single_diagonal_no_rotation(env11):
    """n = 1: only the j = 0 term (he_linalg.cpp:979, no rotation), then relin + rescale."""
    e = env11
    A, X = [e.enc(seed=900)], [e.enc(seed=901), e.enc(seed=902)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
    got = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)


def test_matvec_key_subset_uses_naf(orc, hecdna):
    """With only the keys for steps +-1, 2, 4, 8 (no conjugation, no larger powers), rotations by
    3, 5, 6, 7 decompose by NAF into those keys exactly as SEAL's rotate_internal does."""
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
    o = orc.Oracle(N, m)
    elts = [o.elt_from_step(s) for s in (1, -1, 2, -2, 4, -4, 8, -8)]
    e = Env(orc, hecdna, N, [50, 36, 36, 50], seed=55, elts=elts)
    A = [e.enc(seed=910 + j) for j in range(8)]
    X = [e.enc(seed=920)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
    got = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    e.same(got[0], exp[0])


def test_matvec_errors_follow_seal(env11, hecdna):
    e = env11
    X = [e.up(e.enc(seed=930))]
    A = [e.up(e.enc(seed=931 + j)) for j in range(4)]
    partial_keys = e.ctx.galois_keys({k: v for k, v in e.gk_h.items() if k == e.o.elt_from_step(1)})
    with pytest.raises(hecdna.InvalidArgument, match="Galois key not present"):
        e.ctx.matmul_diag_col(A, X, e.rk, partial_keys)        # rot by 2 needs the step-2 key
    with pytest.raises(hecdna.InvalidArgument, match="scale mismatch"):
        e.ctx.matmul_diag_col(A[:3] + [e.up(e.enc(seed=935, scale=2.0**39))], X, e.rk, e.gk)
    with pytest.raises(hecdna.InvalidArgument, match="parameter mismatch"):
        e.ctx.matmul_diag_col(A[:3] + [e.up(e.enc(seed=936, level=2))], X, e.rk, e.gk)
    low = [e.up(e.enc(seed=940 + j, level=1, scale=2.0**20)) for j in range(2)]
    with pytest.raises(hecdna.InvalidArgument, match="end of modulus switching chain reached"):
        e.ctx.matmul_diag_col(low, [e.up(e.enc(seed=945, level=1, scale=2.0**20))], e.rk, e.gk)
    with pytest.raises(hecdna.InvalidArgument, match="scale out of bounds"):   # SEAL's multiply check first
        e.ctx.matmul_diag_col([e.up(e.enc(seed=946, level=1))], [e.up(e.enc(seed=947, level=1))], e.rk, e.gk)
    big = [A[0]] * (e.N // 2 + 1)                                 # j = N/2 is outside the slot range
    with pytest.raises(hecdna.InvalidArgument, match="step count too large"):
        e.ctx.matmul_diag_col(big, X, e.rk, e.gk)
    with pytest.raises(hecdna.InvalidArgument):
        e.ctx.matmul_diag_col([], X, e.rk, e.gk)


def test_matvec_partial_sum_of_all_singletons(env11):
    """Sum of the n single-diagonal partials mod q = the full accumulator (any j order)."""
    e = env11
    n = 6
    gA = [e.up(e.enc(seed=950 + j)) for j in range(n)]
    gX = [e.up(e.enc(seed=960))]
    full = e.ctx.matmul_diag_col_partial(gA, 0, n, gX, e.gk)[0].download()
    q = np.array(e.m[:3], dtype=np.uint64).reshape(1, 3, 1)
    acc = np.zeros_like(full)
    for j in reversed(range(n)):
        acc = (acc + e.ctx.matmul_diag_col_partial_set(gA, [j], gX, e.gk)[0].download()) % q
    assert np.array_equal(acc, full)


def _with_coeff_zeros(e, ct, limbs_zeros):
    """Copy of ct whose c1 has zero coefficients (coefficient form) at the given positions per limb."""
    d = ct.data.copy()
    for J, pos in limbs_zeros.items():
        coef = e.o.ntt_inv(J, d[1][J])
        coef[np.asarray(pos)] = 0
        d[1][J] = e.o.ntt_fwd(J, coef)
    return e.orc.Ct(d, ct.scale)


def _env_with(orc, hecdna, env, *args, **kw):
    """An Env whose context was created under the given HEC_* switches (read at context creation)."""
    import os
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Env(orc, hecdna, *args, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("nzeros", [3, 40])  # 40 > HEC_ZCAP: the hoisted walk recomputes without hoisting
@pytest.mark.parametrize("variant", [{}, {"HEC_HMAC": "0"}, {"HEC_HMAC": "1"}, {"HEC_HMAC": "1", "HEC_HMAC_ODD3": "0"},
                                     {"HEC_HMAC_INT": "0"}])
def test_hoisted_modup_zero_coefficients(orc, hecdna, nzeros, variant):
    """The hoisted mod-up corrects for zero digit coefficients that the Galois automorphism negates
    (SEAL maps -0 to 0, not to q_J); a limb with more zeros than the kernels list falls back.  Every hoisted MAC
    schedule (k_hmacm over a whole sibling group, pairs and triples, one k_hmac per child)."""
    e = _env_with(orc, hecdna, variant, 1 << 11, [50, 36, 36, 50])
    rng = np.random.default_rng(nzeros)
    X = [_with_coeff_zeros(e, e.enc(seed=1100 + i), {0: rng.choice(e.N, nzeros, replace=False),
                                                     2: rng.choice(e.N, 2, replace=False)}) for i in range(2)]
    A = [e.enc(seed=1200 + j) for j in range(12)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
    got = e.ctx.matmul_diag_col([e.up(a) for a in A], [e.up(x) for x in X], e.rk, e.gk)
    for g, c in zip(got, exp):
        e.same(g, c)
