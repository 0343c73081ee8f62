"""Multi-GPU sharding of the matvec.  One process per GPU.

Two modes:

* throughput (the BASELINE metric): every rank holds a replica of the encrypted matrix and the keys
  and runs its own input vectors through ``Context.matmul_diag_col``.  No data-path collective.

* single-matvec / row-sharded (cfg4 curve): the diagonal index j of BatchedMatrix::matmul
  (he_linalg.cpp:977-997) is split into disjoint sets, one per rank, balanced by the number of
  key switches the rotation prefix trie spends on each range (ranges are whole trie subtrees, see
  plan_diagonal_shards).  Rank g computes the size-3 partial
  accumulator  sum_{j in J_g} A[j] (x) rot(x, j)  (hec_matmul_diag_col_partial_set), the ranks exchange the
  partials once (RCCL reduce-scatter / all-reduce of the u64 words as int64 — G * q < 2^63 for q < 2^60
  and G <= 8, so the plain integer sum is exact), every coefficient is reduced mod q
  (hec_ciphertext_reduce), and the owner of each output runs the lazy relinearize + rescale
  (hec_matmul_finish, he_linalg.cpp:999-1002).  Modular addition is associative, so the bits equal the
  1-GPU result.

torch is only plumbing here (device tensors for the collective); it is imported lazily so the C-ABI
package itself never depends on it.
"""
from __future__ import annotations

import numpy as np


# ------------------------------------------------------------------ rotation cost model (host logic)
def _naf(v: int) -> list[int]:
    """seal::util::naf — non-adjacent form, least-significant term first."""
    res, sign, v, i = [], v < 0, abs(v), 0
    while v:
        z = (2 - (v & 3)) if v & 1 else 0
        v = (v - z) >> 1
        if z:
            res.append((-z if sign else z) << i)
        i += 1
    return res


def default_galois_elts(N: int) -> list[int]:
    """KeyGenerator::create_galois_keys() default set: 2N-1 and 3^(+-2^i), i <= log2(N)-2."""
    m = 2 * N
    pos, neg, out = 3, pow(3, -1, m), []
    for _ in range(N.bit_length() - 2):
        out += [pos, neg]
        pos, neg = pos * pos % m, neg * neg % m
    return out + [m - 1]


def elt_from_step(N: int, step: int) -> int:
    """GaloisTool::get_elt_from_step (generator 3)."""
    m = 2 * N
    if step == 0:
        return 1
    if step < 0:
        step = N // 2 + step
    return pow(3, step, m)


def rotation_elts(N: int, step: int, keys: set[int]) -> list[int]:
    """The Galois elements rotate_internal applies for `step`, in order."""
    if step == 0:
        return []
    e = elt_from_step(N, step)
    if e in keys:
        return [e]
    seq = []
    for t in _naf(step):
        if abs(t) != N // 2:
            seq += rotation_elts(N, t, keys)
    return seq


def trie_cost(N: int, steps, keys: set[int] | None = None) -> int:
    """Key switches the rotation prefix trie spends on `steps` (= distinct non-empty prefixes)."""
    keys = keys if keys is not None else set(default_galois_elts(N))
    prefixes = set()
    for s in steps:
        seq = tuple(rotation_elts(N, s, keys))
        for k in range(1, len(seq) + 1):
            prefixes.add(seq[:k])
    return len(prefixes)


def _chunk(order, seqs, budget, limit):
    """Greedy split of `order` into chunks whose trie cost is <= budget (a single diagonal may exceed
    it).  Returns the chunks, or None once more than `limit` are needed."""
    chunks, cur, seen, cost = [], [], set(), 0
    for j in order:
        pre = [seqs[j][:k] for k in range(1, len(seqs[j]) + 1)]
        add = sum(1 for x in pre if x not in seen)
        if cur and cost + add > budget:
            chunks.append(cur)
            if len(chunks) >= limit:
                return None
            cur, seen, cost = [], set(), 0
            add = len(pre)
        cur.append(j)
        seen.update(pre)
        cost += add
    chunks.append(cur)
    return chunks


def plan_diagonal_shards(N: int, n: int, world: int, keys: set[int] | None = None) -> list[list[int]]:
    """Split the diagonals j in [0, n) over `world` ranks by subtrees of the rotation prefix trie.

    The diagonals are ordered depth-first over the trie (lexicographic order of their Galois element
    sequences keeps every subtree contiguous), then cut into `world` chunks with the smallest
    per-chunk key-switch budget that fits (binary search).  A cut inside a subtree only repeats
    the shared path above it on both sides, so the total over ranks stays within a few key switches
    of the 1-GPU trie (contiguous j ranges would instead repeat most of the upper trie per rank).
    Every rank gets a non-empty list (requires n >= world)."""
    if world < 1 or n < world:
        raise ValueError("need 1 <= world <= n")
    keys = keys if keys is not None else set(default_galois_elts(N))
    seqs = [tuple(rotation_elts(N, j, keys)) for j in range(n)]
    order = sorted(range(n), key=lambda j: seqs[j])
    total = trie_cost(N, range(n), keys)
    lo, hi = max(1, total // world), total + 1
    best = None
    while lo <= hi:
        mid = (lo + hi) // 2
        ch = _chunk(order, seqs, mid, world)
        if ch is not None:
            best, hi = ch, mid - 1
        else:
            lo = mid + 1
    chunks = best
    # pad to exactly `world` non-empty chunks by splitting the largest ones
    while len(chunks) < world:
        k = max(range(len(chunks)), key=lambda i: len(chunks[i]))
        c = chunks.pop(k)
        chunks[k:k] = [c[: len(c) // 2], c[len(c) // 2:]]
    return [sorted(c) for c in chunks]


# ------------------------------------------------------------------ the one exchange step
def owners(p: int, world: int) -> list[int]:
    """Rank that finishes (relinearize + rescale) output i: contiguous blocks when p % world == 0
    (reduce-scatter), otherwise round robin after an all-reduce."""
    if p % world == 0:
        return [i // (p // world) for i in range(p)]
    return [i % world for i in range(p)]


def exchange_partials(buf, world: int, group=None):
    """Sum the partial accumulators of all ranks.

    buf: int64 tensor [p, words] holding this rank's p size-3 partials (u64 bit patterns, each word
    < 2^60).  Returns the tensor of summed rows this rank owns (see `owners`).  A plain int64 sum
    is exact: world * (2^60 - 1) < 2^63 for world <= 8."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return buf
    if world > 8:
        raise ValueError("u64 partial-sum exchange is exact only for world <= 8")
    p = buf.shape[0]
    if p % world == 0:
        out = torch.empty((p // world,) + tuple(buf.shape[1:]), dtype=buf.dtype, device=buf.device)
        dist.reduce_scatter_tensor(out, buf, op=dist.ReduceOp.SUM, group=group)
        return out
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    rank = dist.get_rank(group)
    mine = [i for i, o in enumerate(owners(p, world)) if o == rank]
    return buf[mine]


def reduce_rows_mod_q(rows: np.ndarray, moduli, level: int, N: int) -> np.ndarray:
    """Host-side restatement of hec_ciphertext_reduce for u64 rows [p, size*level*N] (CPU tests)."""
    r = rows.view(np.uint64).reshape(rows.shape[0], -1, level, N)
    q = np.asarray(moduli[:level], dtype=np.uint64).reshape(1, 1, level, 1)
    return (r % q).reshape(rows.shape[0], -1)


def _are_close(a: float, b: float) -> bool:  # SEAL util::are_close
    return abs(a - b) < np.finfo(np.float64).eps * max(abs(a), abs(b), 1.0)


def agree(err, scales, rank: int, world: int, group=None, device=None):
    """The agreement step before the exchange (the protocol of hec_shard_agree, include/hecdna.h): every rank passes
    its own argument-check result (err: None or the hecdna.HecError it raised) and the product scales of its p
    partial outputs; two all-reduces later a failing rank re-raises its own error, every other rank raises the error
    of the failing rank with the larger (code << 8 | rank + 1), and when no rank failed every rank raises
    invalid_argument "scale mismatch" if the ranks' scales of one output are not SEAL-close (add_inplace over the
    whole sum).  So no rank is left waiting in the exchange.  Returns None when the ranks agree."""
    import torch
    import torch.distributed as dist
    import hecdna
    p = len(scales)
    code = 0
    if err is not None:
        code = ((err.code if isinstance(err, hecdna.HecError) and err.code in (1, 2) else 2) << 8) | (rank + 1)
    inf = float("inf")
    mn = torch.tensor([float(code)] + [inf if code else float(s) for s in scales], dtype=torch.float64, device=device)
    mx = torch.tensor([float(code)] + [-inf if code else float(s) for s in scales], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    mn, mx = mn.cpu().numpy(), mx.cpu().numpy()
    if err is not None:
        return err
    agreed = int(mx[0])
    if agreed:
        cls = hecdna.InvalidArgument if agreed >> 8 == 1 else hecdna.LogicError
        return cls(agreed >> 8, "matmul_diag_col_sharded: the arguments failed SEAL's checks on rank %d"
                   % ((agreed & 0xFF) - 1))
    for i in range(p):
        if not _are_close(float(mn[1 + i]), float(mx[1 + i])):
            return hecdna.InvalidArgument(1, "scale mismatch")
    return None


def sharded_matvec(ctx, diags, cols, rk, gk, rank: int, world: int, plan=None, group=None):
    """Row-sharded diag x col matvec on this rank's GPU (torch.distributed already initialised).

    Returns (owned output indices, their finished Ciphertexts).  The ranks agree on the argument checks before the
    exchange (`agree`), so an error on one rank is raised on every rank instead of leaving the others waiting."""
    import torch
    import hecdna
    if not torch.cuda.is_available():
        raise RuntimeError("torch sees no GPU: initialise torch.cuda before loading hecdna so both use one "
                           "HIP runtime (see INTEGRATION.md)")
    N, n, p = ctx.N, len(diags), len(cols)
    plan = plan or plan_diagonal_shards(N, n, world)
    dev = torch.device("cuda", ctx.device)
    accs, err, scales = None, None, [0.0] * p
    try:
        accs = ctx.matmul_diag_col_partial_set(diags, plan[rank], cols, gk)
        scales = [a.info()[2] for a in accs]
    except Exception as e:  # noqa: BLE001 -- any failure (a HecError, a bad handle or plan, ctypes) must reach
        err = e             # the agreement step, or the other ranks wait in the exchange
        scales = [0.0] * p
    import torch.distributed as dist
    on_dev = world > 1 and dist.get_backend(group) == "nccl"
    err = agree(err, scales, rank, world, group, dev if on_dev else None)
    if err is not None:
        raise err
    size, level, scale = accs[0].info()
    words = size * level * N
    buf = torch.empty((p, words), dtype=torch.int64, device=dev)
    for i, a in enumerate(accs):
        a.export_device(buf[i].data_ptr())
    ctx.synchronize()
    mine_rows = exchange_partials(buf, world, group)
    torch.cuda.synchronize(dev)
    mine = [i for i, o in enumerate(owners(p, world)) if o == rank]
    red = []
    for k, i in enumerate(mine):
        c = hecdna.Ciphertext(ctx)
        c.import_device(mine_rows[k].data_ptr(), size, level, scale)
        ctx.reduce(c)
        red.append(c)
    return mine, (ctx.matmul_finish(red, rk) if red else [])
