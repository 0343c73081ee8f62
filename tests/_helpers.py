"""Shared test helpers.  Tests are the only place (with smoke() and bench's cpu_baseline leg) that
load the oracle, and only as the checker."""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "homomorphic-encryption-algorithms-diploma-thesis_amd")


def load_hecdna():
    if "hecdna" in sys.modules:
        return sys.modules["hecdna"]
    spec = importlib.util.spec_from_file_location("hecdna", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["hecdna"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    return oracle_py


def ks_count(N, n, elts=None):
    """Number of key switches SEAL's rotate_internal performs for rotations j = 1..n-1 with the
    default Galois key set."""
    def elt(step):
        m = 2 * N
        if step < 0:
            step = N // 2 + step
        return pow(3, step, m)
    keys = set()
    m = 2 * N
    pos, neg = 3, pow(3, -1, m)
    keys.add(m - 1)
    for _ in range(N.bit_length() - 2):
        keys.add(pos); keys.add(neg)
        pos = pos * pos % m; neg = neg * neg % m

    def naf(v):
        res, sign, v, i = [], v < 0, abs(v), 0
        while v:
            z = (2 - (v & 3)) if v & 1 else 0
            v = (v - z) >> 1
            if z:
                res.append((-z if sign else z) << i)
            i += 1
        return res

    def count(step):
        if step == 0:
            return 0
        if elt(step) in keys:
            return 1
        return sum(count(s) for s in naf(step) if abs(s) != N // 2)
    return sum(count(j) for j in range(1, n))


def rotation_trie_stats(N, n, min_children=2):
    """The engine's rotation prefix trie for j = 1..n-1 (csrc/hec_engine.hip RotTrie): SEAL's key-switch
    sequence per rotation (one key for +-2^i, else the NAF terms, least significant first).  Returns
    (key switches, hoisted nodes, children of hoisted nodes, children of the other nodes); a node is
    hoisted when it has at least min_children children (HEC_HOIST_MIN)."""
    def naf(v):
        res, i = [], 0
        while v:
            z = (2 - (v & 3)) if v & 1 else 0
            v = (v - z) >> 1
            if z:
                res.append(z << i)
            i += 1
        return res
    kids = {(): 0}
    for j in range(1, n):
        seq = [j] if j & (j - 1) == 0 else [s for s in naf(j) if abs(s) != N // 2]
        p = ()
        for e in seq:
            c = p + (e,)
            if c not in kids:
                kids[c] = 0
                kids[p] += 1
            p = c
    hoisted = [k for k in kids.values() if k >= min_children]
    return len(kids) - 1, len(hoisted), sum(hoisted), sum(k for k in kids.values() if 0 < k < min_children)


def reference_matrix(n):
    """The reference's demo data (src/demos/matrix_operations.cpp:1079-1087): column c, row r ->
    2 + n*c + r.  Returned as M[r][c]."""
    return np.array([[2 + n * c + r for c in range(n)] for r in range(n)], dtype=np.float64)


def diag_vectors(M, slots):
    """Diagonal j of M (slot r = M[r][(r+j) mod n]) replicated cyclically over all slots."""
    n = M.shape[0]
    return [np.array([M[r % n][(r % n + j) % n] for r in range(slots)]) for j in range(n)]


def col_vector(x, slots):
    n = len(x)
    return np.array([x[r % n] for r in range(slots)])


def rotation_seq(N, j):
    """SEAL's key-switch sequence for rot(x, j) under the default Galois keys (rotate_internal: one key
    for j = 2^i, else the NAF terms least significant first, +-N/2 skipped), as step amounts."""
    if j & (j - 1) == 0:
        return [j]
    res, v, i = [], j, 0
    while v:
        z = (2 - (v & 3)) if v & 1 else 0
        v = (v - z) >> 1
        if z and abs(z << i) != N // 2:
            res.append(z << i)
        i += 1
    return res


def trie_subset(N, n, target=64, seed=0):
    """A subset of the diagonals [0, n) whose rotation prefix trie exercises every shape of the full
    one (the engine's RotTrie / walk_trie_hoisted): all children of the root (the largest hoisted node),
    the depth-1 node with the most children (hoisted groups split at HOIST_GROUP below the root too),
    the deepest NAF chains with a terminal at every depth along them, j = 0 (the no-rotation term),
    then random diagonals up to `target`."""
    seqs = {j: tuple(rotation_seq(N, j)) for j in range(1, n)}
    pick = {0}
    first = {}
    for j, s in seqs.items():
        first.setdefault(s[0], j)
    pick |= set(first.values())
    depth = max(len(s) for s in seqs.values())
    deep = [j for j, s in seqs.items() if len(s) == depth]
    for j in (deep[0], deep[len(deep) // 3], deep[2 * len(deep) // 3], deep[-1]):
        pick.add(j)
        s = seqs[j]
        for k in range(1, len(s)):  # terminals along the chain: positive prefix sums whose sequence is the prefix
            v = sum(s[:k])
            if 0 < v < n and seqs[v] == s[:k]:
                pick.add(v)
    kids = {}
    for j, s in seqs.items():
        if len(s) >= 2:
            kids.setdefault(s[:1], {}).setdefault(s[:2], j)
    busiest = max(kids.values(), key=len)
    pick |= set(busiest.values())
    rng = np.random.default_rng(seed)
    rest = [j for j in range(1, n) if j not in pick]
    extra = max(0, target - len(pick))
    pick |= set(int(x) for x in rng.choice(rest, extra, replace=False))
    return sorted(pick)


def subset_trie_shape(N, js):
    """(children of the root, max children of any node, depth, key switches SEAL runs per vector)."""
    kids = {(): set()}
    for j in js:
        s = tuple(rotation_seq(N, j)) if j else ()
        for k in range(len(s)):
            kids.setdefault(s[:k], set()).add(s[:k + 1])
            kids.setdefault(s[:k + 1], set())
    return (len(kids[()]), max(len(v) for v in kids.values()), max(len(k) for k in kids),
            sum(len(rotation_seq(N, j)) for j in js if j))
