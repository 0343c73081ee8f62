"""The CPU oracle reproduces every committed golden fixture (tests/golden/, written by make_golden.py):
the cfg1 demo matvec in both of the reference's forms (COL_OR_DIAG = 1 diag x col, and the compiled default
COL_OR_DIAG = 0 col x col^T, src/demos/matrix_operations.cpp:1123-1132) and the cfg2 batched NTT.  The GPU
tests compare the HIP path with the same hashes, so a change in either side shows here first."""
import json
import os
import sys

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
from make_golden import cfg1_inputs, sha  # noqa: E402

THREADS = min(8, os.cpu_count() or 1)


def test_cfg1_inputs_match_fixture(orc):
    fx = json.load(open(os.path.join(GOLD, "cfg1_matvec.json")))
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    assert m == fx["moduli"]
    assert [sha(c.data, c.scale) for c in cts] == fx["input_sha256"]
    assert sha(rk) == fx["rk_sha256"]
    assert {str(e): sha(k) for e, k in gk.items()} == fx["gk_sha256"]


def test_cfg1_diag_col_golden(orc):
    fx = json.load(open(os.path.join(GOLD, "cfg1_matvec.json")))
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    outs = o.matmul_diag_col(cts, cts, rk, gk, nthreads=THREADS)
    assert [sha(c.data, c.scale) for c in outs] == fx["output_sha256"]
    assert outs[0].level == fx["output_level"] and outs[0].scale == fx["output_scale"]


def test_cfg1_col_colT_golden(orc):
    fx = json.load(open(os.path.join(GOLD, "cfg1_colcolT.json")))
    o, m, sk, rk, gk, cts = cfg1_inputs(orc)
    assert [sha(c.data, c.scale) for c in cts] == fx["input_sha256"]
    outs = o.matmul_col_colT(cts, cts, fx["n"], rk, gk, nthreads=THREADS)
    assert [sha(c.data, c.scale) for c in outs] == fx["output_sha256"]


def test_cfg2_ntt_golden(orc):
    fx = json.load(open(os.path.join(GOLD, "cfg2_ntt.json")))
    N, m = fx["N"], fx["moduli"]
    assert orc.Oracle.create_coeff_modulus(N, fx["bits"]) == m
    o = orc.Oracle(N, m)
    rng = np.random.default_rng(fx["rng_seed"])
    data = np.stack([rng.integers(0, q, N, dtype=np.uint64) for q in m])
    assert sha(data) == fx["input_sha256"]
    assert [sha(o.ntt_fwd(i, data[i])) for i in range(len(m))] == fx["forward_sha256"]
