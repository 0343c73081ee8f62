"""GPU side of the row-sharded matvec in one process: every simulated rank computes its
trie-subtree partial through hec_matmul_diag_col_partial_set, the partials travel through device
int64 tensors (hec_ciphertext_export_device / import_device, the buffers RCCL reduces), are summed,
reduced mod q on the GPU (hec_ciphertext_reduce) and finished; the bits equal the 1-GPU matvec and
the oracle."""
import numpy as np
import pytest

from test_gpu_parity import Env

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env(orc, hecdna):
    return Env(orc, hecdna, 1 << 11, [50, 36, 36, 50], seed=31)


@pytest.mark.parametrize("G", [2, 3, 5])
def test_sharded_partials_sum_to_full_matvec(env, hecdna, G):
    import torch
    import hecdna.shard as shard
    e = env
    n, p = 24, 3
    A = [e.enc(seed=j) for j in range(n)]
    X = [e.enc(seed=300 + i) for i in range(p)]
    exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
    gA, gX = [e.up(a) for a in A], [e.up(x) for x in X]
    plan = shard.plan_diagonal_shards(e.N, n, G)
    dev = torch.device("cuda", 0)
    total = None
    for r in range(G):
        accs = e.ctx.matmul_diag_col_partial_set(gA, plan[r], gX, e.gk)
        size, level, scale = accs[0].info()
        assert (size, level) == (3, 3)
        buf = torch.empty((p, size * level * e.N), dtype=torch.int64, device=dev)
        for i, a in enumerate(accs):
            a.export_device(buf[i].data_ptr())
        e.ctx.synchronize()
        total = buf.clone() if total is None else total + buf
    torch.cuda.synchronize()
    red = []
    for i in range(p):
        c = hecdna.Ciphertext(e.ctx).import_device(total[i].data_ptr(), 3, 3, scale)
        e.ctx.reduce(c)
        red.append(c)
    fin = e.ctx.matmul_finish(red, e.rk)
    for g, c in zip(fin, exp):
        e.same(g, c)


def test_partial_set_any_order_equals_range(env):
    e = env
    n = 9
    gA = [e.up(e.enc(seed=400 + j)) for j in range(n)]
    gX = [e.up(e.enc(seed=500))]
    a = e.ctx.matmul_diag_col_partial(gA, 2, 7, gX, e.gk)[0]
    b = e.ctx.matmul_diag_col_partial_set(gA, [6, 2, 4, 3, 5], gX, e.gk)[0]
    assert np.array_equal(a.download(), b.download()) and a.scale == b.scale


def test_partial_set_rejects_bad_indices(env, hecdna):
    e = env
    gA = [e.up(e.enc(seed=600 + j)) for j in range(4)]
    gX = [e.up(e.enc(seed=610))]
    with pytest.raises(hecdna.InvalidArgument):
        e.ctx.matmul_diag_col_partial_set(gA, [1, 1], gX, e.gk)
    with pytest.raises(hecdna.InvalidArgument):
        e.ctx.matmul_diag_col_partial_set(gA, [0, 4], gX, e.gk)
    with pytest.raises(hecdna.InvalidArgument):
        e.ctx.matmul_diag_col_partial_set(gA, [], gX, e.gk)


def test_cabi_sharded_matvec_one_rank_rccl(env, hecdna):
    """hec_comm_init with a real one-rank RCCL communicator + hec_matmul_diag_col_sharded (planner, partials,
    ncclAllReduce of the u64 words, reduction mod q, finish on every rank) equals hec_matmul_diag_col bit for
    bit; without a communicator the call runs the world-1 path."""
    e = env
    n, p = 20, 3
    gA = [e.up(e.enc(seed=700 + j)) for j in range(n)]
    gX = [e.up(e.enc(seed=800 + i)) for i in range(p)]
    ref = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)
    ctx = hecdna.Context(e.N, e.m)
    rk, gk = ctx.relin_key(e.rk_h), ctx.galois_keys(e.gk_h)
    A = [ctx.ciphertext(a.download(), a.scale) for a in gA]
    X = [ctx.ciphertext(x.download(), x.scale) for x in gX]
    plain = ctx.matmul_diag_col_sharded(A, X, rk, gk)            # no communicator: world 1
    ctx.comm_init(0, 1, hecdna.comm_unique_id())
    got = ctx.matmul_diag_col_sharded(A, X, rk, gk)
    for g, q, r in zip(got, plain, ref):
        assert np.array_equal(g.download(), r.download()) and g.scale == r.scale
        assert np.array_equal(q.download(), r.download())
    with pytest.raises(hecdna.InvalidArgument, match="already"):
        ctx.comm_init(0, 1, hecdna.comm_unique_id())


def test_cabi_sharded_null_planned_diagonal_rejected(env, hecdna):
    """hecdna.h contract: a rank reads only the diagonals its plan assigns and NULL is allowed for the others; a
    NULL (None) handle for a diagonal the rank must read is an HEC_EINVAL, never a dereference.  At world 1 every
    diagonal is planned, so any None is rejected; bench.py's sharded stage exercises None for other ranks'
    diagonals at world > 1."""
    e = env
    n = 6
    gA = [e.up(e.enc(seed=900 + j)) for j in range(n)]
    gX = [e.up(e.enc(seed=950))]
    for hole in (0, 3, n - 1):
        A = list(gA)
        A[hole] = None
        with pytest.raises(hecdna.InvalidArgument):
            e.ctx.matmul_diag_col_sharded(A, gX, e.rk, e.gk)
    ref = e.ctx.matmul_diag_col(gA, gX, e.rk, e.gk)[0]           # the context is still usable
    got = e.ctx.matmul_diag_col_sharded(gA, gX, e.rk, e.gk)[0]
    assert np.array_equal(got.download(), ref.download())


def _sharded_ops_worker(rank, world, port, q):
    """One rank of hec_matmul_diag_col_sharded over a host communicator (gloo), its context on cuda:0."""
    import os
    import sys
    import torch
    import torch.distributed as dist
    torch.cuda.is_available()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from _helpers import load_hecdna, load_oracle
    hec, orc = load_hecdna(), load_oracle()
    import hecdna.shard as shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        e = Env(orc, hec, 1 << 11, [50, 36, 36, 50], seed=31)
        n, p = 20, 3
        A = [e.enc(seed=700 + j) for j in range(n)]
        X = [e.enc(seed=800 + i) for i in range(p)]
        exp = e.o.matmul_diag_col(A, X, e.rk_h, e.gk_h)
        plan = shard.plan_diagonal_shards(e.N, n, world)
        mine = set(plan[rank])
        gA = [e.up(A[j]) if j in mine else None for j in range(n)]   # other ranks' diagonals: never read
        gX = [e.up(x) for x in X]
        e.ctx.comm_init_ops(rank, world, hec.HostComm())
        res = []

        def call(diags):
            try:
                got = e.ctx.matmul_diag_col_sharded(diags, gX, e.rk, e.gk)
            except hec.InvalidArgument as ex:
                return "EINVAL: " + str(ex)
            return all(np.array_equal(g.download(), c.data) and g.scale == c.scale for g, c in zip(got, exp))
        bad = list(gA)
        if rank == world - 1:
            bad[plan[rank][0]] = None                                  # fails its own checks
        res.append(call(bad))
        res.append(call(gA))                                           # the next call: bit-exact on every rank
        other = list(gA)
        if rank == world - 1:                                          # consistent within the rank, not across
            other = [e.ctx.ciphertext(A[j].data, A[j].scale * (1 + 1e-6)) if j in mine else None for j in range(n)]
        res.append(call(other))
        res.append(call(gA))
        q.put((rank, "ok", res))
    except Exception as ex:  # surface the failure to the parent
        q.put((rank, repr(ex), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_cabi_sharded_matvec_multirank_host_comm(world):
    """hec_matmul_diag_col_sharded at world > 1 (each rank a process with its own context on
    the one GPU, collectives through hec_comm_init_ops over gloo; RCCL refuses two ranks on one device): a rank that
    fails its argument checks makes every rank raise invalid_argument without a hang, the next call is bit-exact
    against the oracle's full matvec on every rank, a cross-rank scale mismatch is an error on every rank."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_ops_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res
    last = world - 1
    for rank, _, (r1, r2, r3, r4) in res:
        assert r1.startswith("EINVAL") and (rank == last or "on rank %d" % last in r1), (rank, r1)
        assert r2 is True and r4 is True, (rank, r2, r4)
        assert r3 == "EINVAL: scale mismatch", (rank, r3)
