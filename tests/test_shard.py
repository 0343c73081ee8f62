"""Multi-GPU sharding logic on CPU: the trie-subtree planner, and the one exchange
step over a world_size-2 gloo process group.  The per-rank partial accumulators come from the
oracle here (the GPU path for the same step is in test_gpu_shard.py); what is under test is the
planner, the u64-as-int64 collective and the owner bookkeeping in hecdna.shard."""
import os
import socket

import numpy as np
import pytest


@pytest.fixture(scope="module")
def shard(hecdna):
    import hecdna.shard as s
    return s


def test_rotation_elts_follow_seal_naf(shard, orc):
    N = 1 << 11
    m = orc.Oracle.create_coeff_modulus(N, [50, 36, 50])
    o = orc.Oracle(N, m)
    assert sorted(shard.default_galois_elts(N)) == sorted(o.default_galois_elts())
    for v in list(range(-40, 41)) + [N // 2 - 1, 1000, -777]:
        assert shard._naf(v) == orc.Oracle.naf(v)
        if 0 < abs(v) < N // 2:
            assert shard.elt_from_step(N, v) == o.elt_from_step(v)


@pytest.mark.parametrize("N,n,total", [(1 << 13, 64, 84), (1 << 15, 4096, 5460), (1 << 16, 1024, 1364)])
def test_trie_cost_known_counts(shard, N, n, total):
    # 5460 = key switches of the cfg3 matvec on the trie (SEAL's per-rotation count is 18204)
    assert shard.trie_cost(N, range(n)) == total


@pytest.mark.parametrize("N,n", [(1 << 13, 64), (1 << 15, 4096), (1 << 16, 1024), (1 << 11, 5)])
@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
def test_plan_partitions_and_balances(shard, N, n, G):
    if G > n:
        with pytest.raises(ValueError):
            shard.plan_diagonal_shards(N, n, G)
        return
    plan = shard.plan_diagonal_shards(N, n, G)
    assert len(plan) == G and all(plan)
    assert sorted(j for p in plan for j in p) == list(range(n))
    costs = [shard.trie_cost(N, p) for p in plan]
    total = shard.trie_cost(N, range(n))
    depth = max(len(shard.rotation_elts(N, j, set(shard.default_galois_elts(N)))) for j in range(n))
    # subtrees stay whole: at most one shared path repeated per cut
    assert sum(costs) <= total + (G - 1) * depth
    if n >= 64:
        assert max(costs) <= -(-total // G) + 2 * depth


def test_owners(shard):
    assert shard.owners(8, 4) == [0, 0, 1, 1, 2, 2, 3, 3]
    assert shard.owners(3, 2) == [0, 1, 0]
    assert shard.owners(1, 1) == [0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, p, q):
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from _helpers import load_hecdna, load_oracle
    load_hecdna()
    import hecdna.shard as shard
    orc = load_oracle()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        N, n = 1 << 11, 8
        m = orc.Oracle.create_coeff_modulus(N, [50, 36, 36, 50])
        o = orc.Oracle(N, m)
        sk = o.secret_key(5)
        rk = o.relin_key(sk, 6)
        gk = o.galois_keys(sk, o.default_galois_elts(), 7)
        rng = np.random.default_rng(11)
        enc = lambda s: o.encrypt(sk, o.encode(rng.uniform(-1, 1, N // 2), 2.0**30, 3), 2.0**30, s)  # noqa
        A = [enc(100 + j) for j in range(n)]
        X = [enc(200 + i) for i in range(p)]
        plan = shard.plan_diagonal_shards(N, n, world)
        mine = plan[rank]
        # this rank's partial = sum over its contiguous runs of oracle range partials (mod q)
        acc = None
        runs, start = [], mine[0]
        for a, b in zip(mine, mine[1:] + [None]):
            if b != a + 1:
                runs.append((start, a + 1))
                start = b
        qs = np.asarray(m[:3], dtype=np.uint64).reshape(1, 3, 1)
        for jb, je in runs:
            part = o.matmul_diag_col(A, X, rk, gk, j_begin=jb, j_end=je, finish=False)
            d = np.stack([c.data for c in part])
            acc = d if acc is None else (acc + d) % qs
        scale = part[0].scale
        buf = torch.from_numpy(acc.reshape(p, -1).view(np.int64).copy())
        rows = shard.exchange_partials(buf, world)
        red = shard.reduce_rows_mod_q(rows.numpy(), m, 3, N)
        owned = [i for i, w in enumerate(shard.owners(p, world)) if w == rank]
        assert len(owned) == red.shape[0]
        full = o.matmul_diag_col(A, X, rk, gk)
        for k, i in enumerate(owned):
            c = orc.Ct(red[k].reshape(3, 3, N).copy(), scale)
            fin = o.rescale(o.relinearize(c, rk))
            assert fin.scale == full[i].scale
            assert np.array_equal(fin.data, full[i].data), (rank, i)
        q.put((rank, "ok", owned))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


# p == world: the reduce-scatter path; otherwise all-reduce + round-robin owners.  World 4 rehearses the exchange
# the driver's multi-GPU runs use over RCCL, on gloo (CPU).
@pytest.mark.parametrize("world,p", [(2, 2), (2, 3), (4, 4), (4, 5)])
def test_gloo_world2_exchange_bit_exact(shard, world, p):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, p, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res
    owned = sorted(i for r in res for i in r[2])
    assert owned == list(range(p))


@pytest.mark.parametrize("N,n,world", [(1 << 15, 4096, 2), (1 << 15, 4096, 8), (1 << 13, 64, 3), (1 << 16, 1024, 4),
                                       (1 << 11, 10, 8)])
def test_cpp_planner_equals_python(hecdna, N, n, world):
    """hec_plan_diagonal_shards (the C-ABI planner a C++ caller of the he_linalg.h drop-in uses) makes the same
    trie-subtree partition as shard.plan_diagonal_shards."""
    import hecdna.shard as shard
    keys = shard.default_galois_elts(N)
    assert hecdna.plan_diagonal_shards(N, n, world, keys) == shard.plan_diagonal_shards(N, n, world, set(keys))


def _agree_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from _helpers import load_hecdna
    hec = load_hecdna()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = hec.HostComm()
        p, s = 3, 2.0**80
        out = []
        # 1. the last rank fails SEAL's checks: every rank returns its status
        st = hec.HEC_EINVAL if rank == world - 1 else 0
        out.append(hec.shard_agree(comm, rank, st, "scale out of bounds" if st else "", [s] * p))
        # 2. all pass with equal scales
        out.append(hec.shard_agree(comm, rank, 0, "", [s] * p))
        # 3. all pass locally, but rank 0's product scale of output 1 differs (SEAL's add_inplace over the whole sum)
        out.append(hec.shard_agree(comm, rank, 0, "", [s, s * (1 + 1e-9) if rank == 0 else s, s]))
        # 4. two failing ranks (world >= 3: rank 1 invalid_argument, rank 2 logic_error): the larger code names it
        st = {1: hec.HEC_EINVAL, 2: hec.HEC_ELOGIC}.get(rank, 0) if world >= 3 else 0
        out.append(hec.shard_agree(comm, rank, st, {1: "bad one", 2: "bad two"}.get(rank, ""), [s] * p))
        # 5. the protocol holds no state: the next agreement passes
        out.append(hec.shard_agree(comm, rank, 0, "", [s] * p))
        q.put((rank, "ok", out))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_cabi_shard_agree_gloo(hecdna, world):
    """hec_matmul_diag_col_sharded's agreement step (hec_shard_agree over a host communicator,
    the same code the RCCL path runs) at world > 1 on the CPU: a rank failing its argument checks makes every rank
    return its status without a hang, a cross-rank scale mismatch is an invalid_argument on every rank, and the
    next call agrees again."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res
    EINVAL, ELOGIC = hecdna.HEC_EINVAL, hecdna.HEC_ELOGIC
    for rank, _, out in res:
        (s1, m1), (s2, _), (s3, m3), (s4, m4), (s5, _) = out
        assert s1 == EINVAL
        assert m1 == ("scale out of bounds" if rank == world - 1 else
                      "matmul_diag_col_sharded: the arguments failed SEAL's checks on rank %d" % (world - 1))
        assert s2 == 0 and s5 == 0
        assert (s3, m3) == (EINVAL, "scale mismatch")
        if world >= 3:  # a failing rank keeps its own error; the others report the larger code (rank 2's)
            assert (s4, m4) == {1: (EINVAL, "bad one"), 2: (ELOGIC, "bad two")}.get(
                rank, (ELOGIC, "matmul_diag_col_sharded: the arguments failed SEAL's checks on rank 2"))
        else:
            assert s4 == 0


def _py_agree_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from _helpers import load_hecdna
    hec = load_hecdna()
    import hecdna.shard as shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, p = 2.0**80, 3
        out = []

        def run(err, scales):
            r = shard.agree(err, scales, rank, world)
            out.append(None if r is None else (type(r).__name__, str(r)))
        run(hec.InvalidArgument(1, "scale out of bounds") if rank == world - 1 else None, [s] * p)
        run(None, [s] * p)
        run(None, [s, s * (1 + 1e-9) if rank == 0 else s, s])
        run(hec.LogicError(2, "bad two") if rank == 1 else None, [s] * p)
        run(None, [s] * p)
        q.put((rank, "ok", out))
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_python_shard_agree_gloo(hecdna, world):
    """shard.sharded_matvec's agreement step (the hec_shard_agree protocol over torch.distributed) at world > 1 on
    the CPU: an argument error on one rank is raised on every rank, a cross-rank scale mismatch too, and the next
    agreement passes."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_py_agree_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for pr in procs:
        pr.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res
    last = world - 1
    for rank, _, (a1, a2, a3, a4, a5) in res:
        assert a1 == ("InvalidArgument", "scale out of bounds" if rank == last else
                      "matmul_diag_col_sharded: the arguments failed SEAL's checks on rank %d" % last)
        assert a2 is None and a5 is None
        assert a3 == ("InvalidArgument", "scale mismatch")
        assert a4 == ("LogicError", "bad two" if rank == 1 else
                      "matmul_diag_col_sharded: the arguments failed SEAL's checks on rank 1")
