"""Experiment (development tool): two contexts on one GPU, each on its own HIP stream with its own
workspace, keys and diagonals, running halves of the batch concurrently from two host threads, vs one
context with the whole batch."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
torch.cuda.set_device(0)
import bench  # noqa: E402

hec = bench.load_hecdna()
N, n, B = 1 << 15, int(os.environ.get("EXP_N", "4096")), int(os.environ.get("EXP_B", "64"))
moduli = hec.create_coeff_modulus(N, [60] + [40] * 9 + [60])
L = len(moduli) - 1


def setup(nb, seed):
    ctx = hec.Context(N, moduli, device=0)
    elts = ctx.default_galois_elts()
    rk = ctx.relin_key(seed=11)
    gk = ctx.galois_keys(uniform_elts=elts, seed=1000)
    diags = [ctx.ciphertext().fill_uniform(2, L, 2.0**40, 10_000 + j) for j in range(n)]
    cols = [ctx.ciphertext().fill_uniform(2, L, 2.0**40, seed + i) for i in range(nb)]
    outs = [hec.Ciphertext(ctx) for _ in range(nb)]
    ctx.synchronize()
    return ctx, rk, gk, diags, cols, outs


def run(s):
    ctx, rk, gk, diags, cols, outs = s
    ctx.matmul_diag_col(diags, cols, rk, gk, out=outs)
    ctx.synchronize()


mode = sys.argv[1] if len(sys.argv) > 1 else "one"
if mode == "one":
    s = setup(B, 90_000)
    run(s)
    t0 = time.perf_counter()
    for _ in range(2):
        run(s)
    dt = (time.perf_counter() - t0) / 2
else:
    k = int(mode)
    ss = [setup(B // k, 90_000 + 1000 * i) for i in range(k)]
    ths = [threading.Thread(target=run, args=(x,)) for x in ss]
    [t.start() for t in ths]
    [t.join() for t in ths]
    t0 = time.perf_counter()
    for _ in range(2):
        ths = [threading.Thread(target=run, args=(x,)) for x in ss]
        [t.start() for t in ths]
        [t.join() for t in ths]
    dt = (time.perf_counter() - t0) / 2
print(f"mode={mode} B={B} n={n}: {dt * 1e3:.1f} ms/step, {B / dt:.3f} matvec/s", flush=True)
