#!/usr/bin/env python3
"""Benchmark: CKKS matvec ciphertexts/sec (N=2^15, L=10) on 1..8 MI355X — BASELINE.json metric.

Workload (BASELINE cfg3): the reference's BatchedMatrix::matmul diag x col (he_linalg.cpp:943-1006)
with n = 4096 diagonals at N = 2^15, coeff_modulus {60, 40 x 9, 60} (L = 10 data primes + P),
default Galois key set (29 keys), lazy relinearization + one rescale per output.  One "step" = one
pass of the hot path over one batch: B input vectors (the p columns of `other`) against the same
encrypted matrix and keys, producing B output ciphertexts.  Inputs are resident in HBM before the
timed region.  Multi-GPU: one process per GPU (torch.distributed over RCCL), each rank holds a
replica of the matrix + keys and processes its own B vectors (weak scaling, no data-path
collective — SURVEY §8(e) throughput mode).

Data: synthetic — uniformly random RNS residues for ciphertexts and keys, generated on the device
(RLWE ciphertexts and key-switching keys are pseudo-uniform; every kernel is data-oblivious, so the
timing equals that of real encryptions; bit-exact parity on real encryptions is in tests/).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "homomorphic-encryption-algorithms-diploma-thesis_amd")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
S_CT = lambda N, l: 2 * l * N * 8  # noqa: E731


def load_hecdna():
    import importlib.util
    spec = importlib.util.spec_from_file_location("hecdna", os.path.join(PKG, "__init__.py"),
                                                  submodule_search_locations=[PKG])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["hecdna"] = mod
    spec.loader.exec_module(mod)
    return mod


def ks_total(N, n):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _helpers import ks_count
    return ks_count(N, n)


def algorithmic_bytes_per_matvec(N, l, n, B, ks):
    """bytes(B) = (n*S_ct + KS*S_key + S_key)/B + KS*2*S_ct + n*S_ct + S_ct3 + S_ct."""
    K = l + 1
    s_ct, s_ct3, s_key = 2 * l * N * 8, 3 * l * N * 8, 2 * l * K * N * 8
    return (n * s_ct + ks * s_key + s_key) / B + ks * 2 * s_ct + n * s_ct + s_ct3 + s_ct


def pmc_traffic(kernel, B, logn, level, n, variant="ctct"):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3 PMC passes
    (profiles/r06_pmc_<kernel>_B<B>[_ctpt].json, else the newest earlier round's; written by tools/pmc_summary.py: FETCH_SIZE and
    WRITE_SIZE in separate passes, gfx950 FETCH x2 correction for 16-B/lane reads) when they were taken on this
    configuration and matvec variant; else None."""
    sfx = "" if variant == "ctct" else f"_{variant}"
    for tag in ("r06", "r05", "r04", "r03", "r02", "r01"):  # the newest round's pass for this kernel
        path = os.path.join(ROOT, "profiles", f"{tag}_pmc_{kernel}_B{B}{sfx}.json")
        if os.path.exists(path):
            break
    else:
        return None
    p = json.load(open(path))
    if (p["batch"], p["logN"], p["level"], p.get("n"), p.get("variant", "ctct")) != (B, logn, level, n, variant):
        return None
    return p["traffic_bytes_per_dispatch"]


def pmc_step_traffic(kernels, B, logn, level, n, variant="ctct"):
    """Whole-step HBM traffic per matvec from the committed PMC passes (the files pmc_traffic reads): the newest
    round whose set covers every kernel of the step on this configuration, summed traffic_bytes_per_step / B
    (VERDICT r05's whole-step figure: bytes actually moved, against SURVEY 8(d)'s algorithmic bytes); else None."""
    sfx = "" if variant == "ctct" else f"_{variant}"
    for tag in ("r06", "r05", "r04", "r03", "r02", "r01"):
        per = {}
        for k in kernels:
            path = os.path.join(ROOT, "profiles", f"{tag}_pmc_{k}_B{B}{sfx}.json")
            if not os.path.exists(path):
                break
            p = json.load(open(path))
            if (p["batch"], p["logN"], p["level"], p.get("n"), p.get("variant", "ctct")) != (B, logn, level, n, variant):
                break
            per[k] = p["traffic_bytes_per_step"] / B / 1e9
        else:
            if per:
                return {"GB_per_matvec": round(sum(per.values()), 1), "by_kernel": {k: round(v, 2) for k, v in per.items()},
                        "source": f"profiles/{tag}_pmc_<kernel>_B{B}{sfx}.json (one PMC step each, FETCH_SIZE x 2 + "
                                  f"WRITE_SIZE; the step's setup dispatches included)"}
    return None


def cgroup_cpu_quota():
    """CPUs granted by the cgroup's CPU quota (cgroup v2 cpu.max, else v1 cfs_quota/period), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(-(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, -(-q // p))
    except (OSError, ValueError):
        return None


def cpu_info():
    """(model, host CPUs, affinity CPUs, threads the CPU leg uses, why that many)."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = cgroup_cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if quota is not None and quota < share:
        return model, os.cpu_count(), share, quota, f"cgroup CPU quota ({quota} CPUs)"
    if omp > 0 and omp < share:
        # the GPU pool's per-job CPU share (16 per GPU) is announced through OMP_NUM_THREADS and not enforced by
        # a cgroup quota or the affinity mask, which span the whole host: the leg uses that share
        return model, os.cpu_count(), share, omp, f"the job's CPU share OMP_NUM_THREADS={omp} (affinity {share})"
    return model, os.cpu_count(), share, share, f"affinity mask ({share} CPUs)"


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(ngpus, argv, port):
    """The one-process-per-GPU launch of this script (torch.distributed.run, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ngpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def bench_seeds(rank, sharded):
    """Seeds of the synthetic inputs.  The relinearization key, the Galois keys and the matrix diagonals are the
    state every rank replicates (one keygen shared by every diagonal, matrix_operations.cpp:1057-1068),
    so they never depend on the rank: a sharded step sums partials that ranks computed with their own copies, and
    rank 0's self-check recomputes them with its copy.  Only the input vectors of throughput mode are per rank
    (each replica processes its own batch); sharded mode splits ONE batch, the same on every rank."""
    return {"relin": 11, "galois": 1000, "diag": 10_000, "col": 90_000 + (0 if sharded else 100 * rank)}


def cpu_baseline(N, moduli, n, sample_diags, threads, data=None):
    """The oracle (the C++ restatement of the reference's SEAL path, kind "port"), built here with
    -march=native, timed on this host:
      all cores: ONE FULL matvec (all n diagonals, SEAL's per-rotation key switches, relinearize + rescale)
                 on `threads` threads (parallel over diagonal ranges, bit-identical partial sums);
      1 core:    the first `sample_diags` diagonals, extrapolated by key-switch count (labelled as such:
                 a full 1-core cfg3 matvec takes ~15 minutes).
    data (the GPU run's own inputs, downloaded: {"A": n diagonals, "X": [one input vector], "rk", "gk"}): the full
    matvec runs on them and its output is returned, so the bench checks the bits it timed against the oracle."""
    import subprocess
    import tempfile
    build = tempfile.mkdtemp(prefix="orc_native_")
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", f"OUT={build}"])
    os.environ["HEC_ORACLE_LIB"] = os.path.join(build, "liboracle_native.so")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as orc
    o = orc.Oracle(N, moduli)
    rng = np.random.default_rng(5)
    L, K = len(moduli) - 1, len(moduli)

    def rnd_ct():
        return orc.Ct(np.stack([np.stack([rng.integers(0, moduli[i], N, dtype=np.uint64) for i in range(L)])
                                for _ in range(2)]), 2.0**40)

    def rnd_key():
        k = np.empty((L, 2, K, N), dtype=np.uint64)
        for i in range(K):
            k[:, :, i] = rng.integers(0, moduli[i], (L, 2, N), dtype=np.uint64)
        return k
    if data is not None:
        A = [orc.Ct(a, 2.0**40) for a in data["A"]]
        X = [orc.Ct(x, 2.0**40) for x in data["X"]]
        rk, gk = data["rk"], data["gk"]
    else:
        elts = o.default_galois_elts()
        gk = {e: rnd_key() for e in elts}
        rk = rnd_key()
        A = [rnd_ct() for _ in range(8)]   # n diagonals cycle over 8 distinct ciphertexts (data-oblivious timing)
        X = [rnd_ct()]
    from _helpers import ks_count
    ks_sample = ks_count(N, sample_diags)
    full, outs = o.bench_matvec(A, n, X, rk, gk, nthreads=threads, outputs=True)
    one = o.bench_matvec(A, n, X, rk, gk, nthreads=1, j_end=sample_diags, finish=False)
    return {"full_s": full, "one_core_s": one * ks_total(N, n) / ks_sample, "ks_sample": ks_sample,
            "outputs": [c.data for c in outs]}


def run_cfg2(args, hec, world, rank, local, barrier, max_over_ranks):
    """BASELINE configs[1]: batched forward NTT + dyadic multiply + inverse NTT at N = 2^15 over the 10 data primes of
    the cfg2-4 chain {60, 40 x 9, 60} (the primitives of math_operations.cpp:316-354's per-primitive
    timing).  One step = forward NTT of --batch polynomials x 10 limbs in place, their dyadic product with a second
    NTT-form batch, inverse NTT of the product.  value = limb-NTTs per second (forward + inverse); the roofline uses
    SURVEY §8(d)'s 524,288 B (2 N 8) per limb-NTT (both passes together)."""
    N = 1 << 15
    moduli = hec.create_coeff_modulus(N, [60] + [40] * 9 + [60])
    nl, npolys = 10, args.batch
    ctx = hec.Context(N, moduli, device=local)
    rng = np.random.default_rng(2 + rank)
    words = npolys * nl * N
    bufs = [hec.DeviceBuffer(ctx, words * 8) for _ in range(3)]
    for b in bufs[:2]:
        host = np.stack([rng.integers(0, moduli[i], (npolys, N), dtype=np.uint64) for i in range(nl)], axis=1)
        b.upload(host)
        del host
    ctx.synchronize()

    def step():
        ctx.ntt_device(bufs[0], nl, npolys)
        ctx.dyadic_device(bufs[0], bufs[1], bufs[2], nl, npolys)
        ctx.ntt_device(bufs[2], nl, npolys, inverse=True)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)

    limb_ntts = 2 * nl * npolys * args.steps * world
    kernels, roof = {}, None
    if not args.no_profile:
        ctx.profile(2)
        step()
        ctx.synchronize()
        for cls in ctx.profile_classes():
            if not cls.startswith("k:"):
                continue
            ms, _, nbytes, kl = ctx.profile_read_ex(cls)
            kernels[cls[2:]] = {"ms": round(ms, 4), "launches": kl, "bytes_per_launch": int(nbytes / max(1, kl)),
                                "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1) if ms else None}
        ctx.profile(0)
        ntt = [v for k, v in kernels.items() if k.startswith("k_ntt/")]
        ms = sum(v["ms"] for v in ntt)
        nb_pass = sum(v["bytes_per_launch"] * v["launches"] for v in ntt)
        nlaunch = sum(v["launches"] for v in ntt)
        # SURVEY 8(d)'s unit: one limb-NTT = 2 N 8 = 524,288 B (the limb read once and written once, twiddles
        # amortised), whatever the number of passes the kernel takes; a step runs 2 nl npolys limb-NTTs in nlaunch
        # pass launches, so a launch is credited with its share of those bytes
        nb = 2 * nl * npolys * 2 * N * 8
        gbs = nb / (ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None, "kernel": "k_ntt", "avg_ms": round(ms / nlaunch, 4),
                "algorithmic_bytes_per_launch": int(nb / nlaunch), "launches_per_step": nlaunch,
                "us_per_limb_ntt": round(ms * 1e3 / (2 * nl * npolys), 4),
                "per_pass_GBps": round(nb_pass / (ms * 1e-3) / 1e9, 1),
                "note": "SURVEY 8(d) unit: 524,288 B per limb-NTT (one read and one write of the limb); the transform "
                        "takes two passes, each reading and writing every limb, so the kernels move twice these bytes "
                        "(per_pass_GBps counts both passes' in + out)"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_py as orc
        o = orc.Oracle(N, moduli)
        sample = 200  # limbs per direction, about 0.5 s of scalar CPU work
        data = [rng.integers(0, moduli[i % nl], N, dtype=np.uint64) for i in range(sample)]
        t1 = time.perf_counter()
        for i, a in enumerate(data):
            o.ntt_inv(i % nl, o.ntt_fwd(i % nl, a))
        cs = time.perf_counter() - t1
        cpu = {"value": round(2 * sample / cs, 2), "unit": "limb-NTT/s", "cores": 1, "kind": "port",
               "sample": f"{sample} forward + {sample} inverse limb-NTTs at N=2^15 (the oracle's Harvey NTT, SEAL's "
                         f"ntt_negacyclic_harvey restated, one thread, via ctypes)"}
    if rank == 0:
        print(json.dumps({
            "metric": "batched negacyclic NTT limb-transforms/sec (N=2^15, 10 primes), forward + dyadic + inverse",
            "value": round(limb_ntts / dt, 1), "unit": "limb-NTT/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": f"cfg2: forward NTT + dyadic + inverse NTT of {npolys} polys x {nl} limbs, N=2^15, "
                                   f"primes {{60, 40 x 9}}", "batch_per_gpu": npolys,
                       "parallelism": f"replicas, dp{world}"},
            "roofline": roof, "kernels_one_step": kernels, "cpu_baseline": cpu}))


def any_failed_over(dist, failed, device):
    """One all-reduce (MAX) of (rank + 1 if this rank failed else 0): the highest failing rank, or None."""
    if dist is None:
        return 0 if failed else None
    import torch
    t = torch.tensor([float(dist.get_rank() + 1) if failed else 0.0], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = int(t.item())
    return v - 1 if v else None


def sharded_extra_leg(prepare, run, selfcheck, barrier, max_over_ranks, any_failed, rank, nsh, batch):
    """Control flow of the cfg4 sharded leg that follows the metric's timed steps at N > 1: every
    collective is reached by every rank, whatever fails where.
      prepare() -> state: per-rank setup (plan, the rank-0 batch on every rank); a failure on any rank is agreed by
        any_failed(flag) (one all-reduce) and every rank skips the leg with the same error;
      run(state) -> result: one sharded matvec (shard.sharded_matvec: its own argument agreement before the exchange,
        so an argument error on one rank is raised on every rank); one warmup call, then nsh timed calls between
        barriers, max over ranks;
      selfcheck(result): rank 0 only, local (no collective).
    The metric is complete before this leg runs: an exception here is reported in the line, not raised."""
    try:
        state, err = prepare(), None
    except Exception as e:  # noqa: BLE001 (reported in the line)
        state, err = None, e
    bad = any_failed(err is not None)
    if bad is not None:
        return {"error": f"preparation failed on rank {bad}" + (f": {type(err).__name__}: {err}" if err else "")}
    try:
        res = run(state)  # warmup
        barrier()
        t0 = time.perf_counter()
        for _ in range(nsh):
            res = run(state)
        barrier()
        sdt = max_over_ranks(time.perf_counter() - t0)
        out = {"value": round(batch * nsh / sdt, 6), "unit": "matvec/s", "steps": nsh,
               "ms_per_step": round(sdt / nsh * 1e3, 3), "scaling": "strong", "batch": batch}
    except Exception as e:  # noqa: BLE001 (raised on every rank by the agreement inside run)
        import traceback
        traceback.print_exc(file=sys.stderr)
        return {"error": f"{type(e).__name__}: {e}"}
    if rank == 0:
        try:
            out["self_check"] = selfcheck(res)
        except Exception as e:  # noqa: BLE001
            out["self_check"] = {"error": f"{type(e).__name__}: {e}", "bitexact": None}  # not run, not failed
    return out


def dry_run(args, world, rank):
    """--dry-run: the launcher, the process group, the max-over-ranks timing and the rank-0 line over gloo,
    with no GPU and no engine (tests/test_bench_measurement.py runs it at world size 2 on the CPU)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    for _ in range(args.warmup + args.steps):
        if world > 1:
            dist.barrier()
    dt = time.perf_counter() - t0

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    dt = max_over_ranks(dt)
    # the sharded extra leg's control flow over gloo with stand-in work: --dry-run-fail <where>:<rank> injects an
    # exception on one rank in the preparation, in the sharded call before its agreement, or in rank 0's self-check
    where, _, frank = (args.dry_run_fail or "none:-1").partition(":")
    frank = int(frank)

    def prepare():
        if where == "prepare" and rank == frank:
            raise RuntimeError("injected preparation failure")
        return torch.arange(4, dtype=torch.int64)

    def run_stub(state):
        err = RuntimeError("injected failure before the agreement") if where == "run" and rank == frank else None
        flag = torch.tensor([1.0 if err else 0.0], dtype=torch.float64)
        if world > 1:  # shard.agree's all-reduce, then the exchange
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        if flag.item():
            raise err or RuntimeError("the arguments failed the checks on another rank")
        buf = state.clone()
        if world > 1:
            dist.all_reduce(buf)
        return buf

    def selfcheck(res):
        if where == "selfcheck":
            raise RuntimeError("injected self-check failure")
        return {"outputs_checked": 1, "bitexact": bool(res[1].item() == world)}

    sharded = None
    if world > 1 or args.sharded_steps:
        sharded = sharded_extra_leg(prepare, run_stub, selfcheck, barrier, max_over_ranks,
                                    lambda f: any_failed_over(dist if world > 1 else None, f, torch.device("cpu")),
                                    rank, args.sharded_steps or 1, 4)
    ok = torch.tensor([0.0], dtype=torch.float64)  # the post-leg all_ranks_bitexact all-reduce
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "CKKS matvec ciphertexts/sec (N=2^15, L=10)", "value": 0.0, "unit": "matvec/s",
                          "n_gpus": world, "rccl_world": dist.get_world_size() if world > 1 else 1,
                          "dist_backend": "gloo", "dry_run": True, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(dt / max(1, args.steps) * 1e3, 3), "sharded": sharded}))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128,
                    help="input vectors per GPU per step (p), run as one batch on the context stream.  Round 6 one-lane "
                         "sweep on one box (profiles/r06a_batch_sweep.json): 10.47 / 10.53 / 10.59 / 10.70 matvec/s at "
                         "96 / 128 / 144 / 192.  128 keeps the driver's --steps 20 --warmup 5 run well inside its "
                         "600 s limit (192 took 542 s in BENCH_r05) for 1.6 %% of throughput; 384 does not fit the "
                         "workspaces in 288 GB; HEC_LANES=3 splits it into 3 concurrent lanes (opt-in)")
    ap.add_argument("--n", type=int, default=4096, help="matrix dimension (diagonals)")
    ap.add_argument("--logn", type=int, default=15)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-diags", type=int, default=48)
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--variant", choices=["ctct", "ctpt"], default="ctct",
                    help="ctct: ciphertext diagonals, the reference's BatchedMatrix::matmul (default); ctpt: "
                         "plaintext diagonals (multiply_plain, no relinearization; SURVEY 8(f) rank 1)")
    ap.add_argument("--mode", choices=["throughput", "sharded"], default="throughput",
                    help="throughput: replicas, own vectors per rank (the metric, weak scaling); sharded: one "
                         "batch split over ranks by trie subtrees of the diagonals + one RCCL reduce-scatter "
                         "(cfg4 curve, strong scaling)")
    ap.add_argument("--config", choices=["cfg2", "cfg3", "cfg5"], default="cfg3",
                    help="cfg3: the BASELINE metric (4096x4096 matvec, N=2^15, L=10); cfg2: BASELINE configs[1], "
                         "batched forward NTT + dyadic + inverse NTT over --batch polys x 10 limbs at N=2^15 "
                         "(limb-NTTs per second; default batch 64); cfg5: BASELINE configs[4], "
                         "the 1024x1024x1024 ct x ct matmul at N=2^16, L=16, measured as output columns per second "
                         "(a step = --batch columns of the product, default 64; not the metric)")
    ap.add_argument("--sharded-steps", type=int, default=None,
                    help="throughput mode at N > 1: after the timed steps, also time this many row-sharded steps of "
                         "one batch (the cfg4 strong-scaling figure, reported under 'sharded'; default 1 at N > 1)")
    ap.add_argument("--no-self-check", action="store_true",
                    help="skip the self-check after the timed steps (PMC passes, which must count one step only)")
    ap.add_argument("--dry-run", action="store_true",
                    help="exercise the launcher, the rank-0 line and the sharded extra leg's control flow over gloo "
                         "without touching a GPU (CPU tests)")
    ap.add_argument("--dry-run-fail", default=None,
                    help="dry run only: inject an exception <prepare|run|selfcheck>:<rank> into the sharded leg")
    args = ap.parse_args()
    wall0 = time.perf_counter()
    if args.config == "cfg5":
        args.logn, args.n = 16, 1024
        if args.batch == ap.get_default("batch"):
            args.batch = 64  # round 4, profiles/r04p_*: 9.93 columns/s vs 9.80 at 32, 9.92 at 48
    if args.config == "cfg2" and args.batch == ap.get_default("batch"):
        args.batch = 64  # 168 MB per buffer, inside the Infinity Cache: 3.20 M limb-NTT/s vs 2.94 M at 128 (r04p)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the N ranks as a child launcher before anything touches a GPU, relay its
        # exit status (rank 0 prints the line)
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.stdout.flush()
        sys.exit(subprocess.call(launcher_cmd(args.gpus, sys.argv[1:], free_port()), env=env))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    # torch first, at every N: libhecdna then binds to torch's HIP runtime, so the RCCL buffers and
    # the engine share one runtime and the 1-GPU and N-GPU runs execute the same code
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    hec = load_hecdna()

    def barrier():
        if dist is not None:
            torch.cuda.synchronize(local)
            dist.barrier()

    def max_over_ranks(dt):
        if dist is None:
            return dt
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if args.config == "cfg2":
        run_cfg2(args, hec, world, rank, local, barrier, max_over_ranks)
        if dist is not None:
            dist.destroy_process_group()
        return
    N = 1 << args.logn
    bits = [60] + [40] * (15 if args.config == "cfg5" else 9) + [60]
    moduli = hec.create_coeff_modulus(N, bits)
    L = len(moduli) - 1
    ctx = hec.Context(N, moduli, device=local)
    elts = ctx.default_galois_elts()
    sharded = args.mode == "sharded"
    seeds = bench_seeds(rank, sharded)
    rk = ctx.relin_key(seed=seeds["relin"])
    gk = ctx.galois_keys(uniform_elts=elts, seed=seeds["galois"])
    scale = 2.0**40
    plan = None
    if sharded:
        import hecdna.shard as shard
        plan = shard.plan_diagonal_shards(N, args.n, world)
        held = set(plan[rank])  # a rank only stores the diagonals of its trie subtrees
    else:
        held = range(args.n)
    ctpt = args.variant == "ctpt"
    if ctpt and sharded:
        raise SystemExit("--variant ctpt runs in throughput mode")
    if ctpt:
        # plaintext diagonals: synthetic U[-1,1] slot values encoded on the GPU (hec_encode), untimed setup
        vals = np.random.default_rng(10_000).uniform(-1, 1, (args.n, N // 2))
        diags = ctx.encode(vals, scale, L)
        del vals
    else:
        diags = [ctx.ciphertext().fill_uniform(2, L, scale, seeds["diag"] + j) if j in held else None
                 for j in range(args.n)]
    # sharded: every rank sees the same input batch (same seeds); throughput: own vectors per rank
    cols = [ctx.ciphertext().fill_uniform(2, L, scale, seeds["col"] + i) for i in range(args.batch)]
    outs = [hec.Ciphertext(ctx) for _ in range(args.batch)]
    ctx.synchronize()

    last_sharded = [None]
    wall = {"setup_s": time.perf_counter() - wall0}

    def step():
        if sharded:
            last_sharded[0] = shard.sharded_matvec(ctx, diags, cols, rk, gk, rank, world, plan=plan)
        elif ctpt:
            ctx.matmul_diagpt_col(diags, cols, gk, out=outs)
        else:
            ctx.matmul_diag_col(diags, cols, rk, gk, out=outs)

    # per-phase breakdown and per-kernel table: one untimed step with asynchronous HIP event pairs recorded on the
    # context's stream around every launch (no host synchronisation inside the step).  With two or more warmup steps
    # it is the LAST WARMUP step (warm workspaces, the same batch and inputs as the timed steps), so it costs no extra
    # step; its outputs are kept and the timed steps' outputs must equal them (self_check.profile_step_bitexact).
    # With fewer warmup steps it is an extra step after the timed ones.
    breakdown = {}
    classes = ("ks_intt", "ks_modup", "ks_mac", "ks_modup_a", "ks_bmac", "ks_modup_h", "ks_hmac", "ks_moddown",
               "galois", "tensor", "relin", "rescale")
    prof = {"classes": [], "ex": {}, "where": None}

    def profile_step(where):
        ctx.profile(2)
        step()
        ctx.synchronize()
        for cls in classes:
            ms, cnt = ctx.profile_read(cls)
            if cnt:
                breakdown[cls] = {"ms": round(ms, 3), "launch_groups": cnt}
        prof["classes"] = ctx.profile_classes()
        prof["ex"] = {c: ctx.profile_read_ex(c) for c in prof["classes"]}
        prof["where"] = where
        ctx.profile(0)

    keep = sorted({0, args.batch // 2, args.batch - 1})
    prof_in_warmup = not args.no_profile and args.warmup >= 2 and not sharded
    prof_saved = None
    tw = time.perf_counter()
    for w in range(args.warmup):
        if prof_in_warmup and w == args.warmup - 1:
            profile_step("last warmup step")
            prof_saved = [(outs[i].download(), outs[i].info()) for i in keep]
        else:
            step()
    ctx.synchronize()
    barrier()
    wall["warmup_s"] = time.perf_counter() - tw
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    wall["timed_s"] = dt
    hbm = {"total_GB": None, "in_use_after_timed_GB": None, "in_use_max_GB": None}

    def hbm_probe(key):
        """Device-wide HBM in use (hipMemGetInfo: the engine's own allocations and torch's alike), the max over
        ranks: the 8-GPU run's per-rank footprint is the replicated matrix and keys plus one batch's workspace."""
        free, tot = torch.cuda.mem_get_info(local)
        used = max_over_ranks((tot - free) / 1e9)
        hbm["total_GB"] = round(tot / 1e9, 1)
        hbm[key] = round(used, 2)
        hbm["in_use_max_GB"] = max(hbm["in_use_max_GB"] or 0.0, round(used, 2))

    hbm_probe("in_use_after_timed_GB")
    tc = time.perf_counter()

    # self-check of the timed outputs, after the timer: three outputs of the last timed step (the
    # first, middle and last vector of the batch), recomputed as ONE call with just those three vectors (another batch
    # size, so other grids and tilings) must equal them bit for bit; the profile step below (a rerun of the batch) and,
    # on rank 0 at N = 1, the CPU leg's oracle matvec of input vector 0 on the same inputs are compared with them too
    check = None
    if not sharded and not args.no_self_check:
        saved = [(outs[i].download(), outs[i].info()) for i in keep]
        alone = (ctx.matmul_diagpt_col(diags, [cols[i] for i in keep], gk) if ctpt else
                 ctx.matmul_diag_col(diags, [cols[i] for i in keep], rk, gk))
        same = [bool(np.array_equal(a.download(), d) and a.info() == inf) for a, (d, inf) in zip(alone, saved)]
        del alone
        check = {"outputs_checked": keep, "single_call_bitexact": all(same)}
        if prof_saved is not None:  # the profiled warmup step ran the same batch on the same inputs
            check["profile_step_bitexact"] = all(np.array_equal(a, d) and ia == inf
                                                 for (a, ia), (d, inf) in zip(prof_saved, saved))

    ms_per_step = dt / args.steps * 1e3
    total = args.batch * (1 if sharded else world) * args.steps
    value = total / dt
    ks = ks_total(N, args.n)

    def sharded_selfcheck(res, cols_used):
        """Rank 0: its first finished outputs of a sharded step against a 1-rank matmul_diag_col of the same inputs
        (every diagonal; the ones rank 0 does not hold are regenerated from their seeds).  Local, no collective."""
        mine, fin = res
        k = min(2, len(mine))
        full = [d if d is not None else ctx.ciphertext().fill_uniform(2, L, scale, seeds["diag"] + j)
                for j, d in enumerate(diags)]
        ref = ctx.matmul_diag_col(full, [cols_used[i] for i in mine[:k]], rk, gk)
        ok = all(np.array_equal(a.download(), b.download()) and a.info() == b.info() for a, b in zip(fin[:k], ref))
        return {"outputs_checked": k, "bitexact": bool(ok)}

    # cfg4 (BASELINE configs[3]) beside the metric: one batch split over the ranks by rotation-trie subtrees of the
    # diagonals, one RCCL reduce-scatter of the size-3 partials (strong scaling), timed after the metric's steps
    sharded_extra = None
    nsh = args.sharded_steps if args.sharded_steps is not None else (1 if world > 1 else 0)
    if not sharded and not ctpt and nsh > 0:
        import hecdna.shard as shard
        splan_box = {}

        def prepare():
            splan = shard.plan_diagonal_shards(N, args.n, world)
            s0 = bench_seeds(0, False)["col"]
            scols = cols if rank == 0 else [ctx.ciphertext().fill_uniform(2, L, scale, s0 + i)
                                            for i in range(args.batch)]  # rank 0's batch on every rank
            splan_box["plan"] = splan
            return splan, scols

        def run(state):
            splan, scols = state
            res = shard.sharded_matvec(ctx, diags, scols, rk, gk, rank, world, plan=splan)
            ctx.synchronize()
            return res, scols

        sharded_extra = sharded_extra_leg(
            prepare, run, lambda r: sharded_selfcheck(r[0], r[1]), barrier, max_over_ranks,
            lambda f: any_failed_over(dist, f, torch.device("cuda", local)), rank, nsh, args.batch)
        if "plan" in splan_box and "error" not in sharded_extra:
            sharded_extra["key_switches_per_rank"] = [shard.trie_cost(N, p) for p in splan_box["plan"]]
    if sharded and rank == 0 and last_sharded[0] is not None:
        sharded_extra = {"self_check": sharded_selfcheck(last_sharded[0], cols)}

    wall["self_check_and_sharded_s"] = time.perf_counter() - tc
    hbm_probe("in_use_after_checks_GB")
    if not args.no_profile and prof["where"] is None:
        tp = time.perf_counter()
        profile_step("extra step after the timed steps")
        if check is not None:  # the profile step reran the whole batch into the same outputs
            check["profile_step_bitexact"] = all(np.array_equal(outs[i].download(), d) and outs[i].info() == inf
                                                  for i, (d, inf) in zip(check["outputs_checked"], saved))
        wall["profile_step_s"] = time.perf_counter() - tp
    prof_classes, prof_ex = prof["classes"], prof["ex"]

    # per-kernel table and roofline.  Every kernel launch of the profile step sits in a "k:<kernel>/<role>"
    # scope that carries its algorithmic bytes (compulsory reads + writes of that kernel given the engine's
    # decomposition, SURVEY 8(d) units: limb = N*8 B, B targets, level l, K = l+1 key moduli):
    # achieved GB/s = bytes / event-timed ms.  The roofline line reports the kernel with the most GPU time.
    kernels = {}
    roof = None
    if not args.no_profile:
        for cls in prof_classes:
            if not cls.startswith("k:"):
                continue
            ms, scopes, nbytes, kl = prof_ex[cls]
            kern, _, role = cls[2:].partition("/")
            k = kernels.setdefault(kern, {"ms": 0.0, "launches": 0, "bytes": 0.0, "roles": {}})
            k["ms"] += ms
            k["launches"] += kl
            k["bytes"] += nbytes
            k["roles"][role or kern] = {"ms": round(ms, 3), "launches": kl,
                                        "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1) if ms else None}
        for kern, k in kernels.items():
            k["GBps"] = round(k["bytes"] / (k["ms"] * 1e-3) / 1e9, 1) if k["ms"] else None
            k["frac"] = round(k["GBps"] / HBM_PEAK_GBS, 4) if k["GBps"] else None
            k["ms"] = round(k["ms"], 3)
            k["bytes_per_launch"] = int(k["bytes"] / max(1, k["launches"]))
            del k["bytes"]
        if kernels:
            kern = max(kernels, key=lambda x: kernels[x]["ms"])
            k = kernels[kern]
            per = k["ms"] / k["launches"]
            roof = {"bound": "hbm", "achieved": k["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": k["frac"], "traffic": pmc_traffic(kern, args.batch, args.logn, L, args.n, args.variant),
                    "kernel": kern, "avg_ms": round(per, 4), "algorithmic_bytes_per_launch": k["bytes_per_launch"],
                    "launches_per_step": k["launches"],
                    "share_of_step_gpu_time": round(k["ms"] / sum(v["ms"] for v in kernels.values()), 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not ctpt:
        tcpu = time.perf_counter()
        model, host_cpus, share, threads, why = cpu_info()
        # the GPU run's own inputs: every diagonal, input vector 0, the relinearization and Galois keys
        data = {"A": [d.download() for d in diags], "X": [cols[0].download()], "rk": rk.download(),
                "gk": {e: gk.download(e) for e in elts}}
        res = cpu_baseline(N, moduli, args.n, args.cpu_sample_diags, threads, data=data)
        del data
        if check is not None:
            d0, (size0, level0, scale0) = saved[0]
            check["oracle_outputs_checked"] = [0]
            check["oracle_bitexact"] = bool(np.array_equal(res["outputs"][0], d0))
        cpu = {"value": round(1.0 / res["full_s"], 6), "unit": "matvec/s", "cores": threads, "kind": "port",
               "sample": f"one full n={args.n} N=2^{args.logn} L={L} diag x col matvec ({ks} key switches, SEAL's "
                         f"per-rotation schedule, relinearize + rescale) by the oracle (C++ SEAL-semantics port, "
                         f"-march=native) on {threads} threads, on the GPU run's own diagonals, keys and input "
                         f"vector 0 (its output is compared with the GPU's bit for bit: self_check)",
               "cpu_model": model, "host_cpus": host_cpus, "cpus_available": share, "cores_reason": why,
               "cgroup_cpu_quota": cgroup_cpu_quota(),
               "full_matvec_s": round(res["full_s"], 2),
               "one_core": {"value": round(1.0 / res["one_core_s"], 6), "cores": 1, "extrapolated": True,
                            "sample": f"diagonals j<{args.cpu_sample_diags} ({res['ks_sample']} key switches) "
                                      f"on 1 thread, scaled to {ks} key switches"}}
        wall["cpu_leg_s"] = time.perf_counter() - tcpu

    if check is not None:
        check["bitexact"] = all(v for k, v in check.items() if k.endswith("bitexact"))
        if dist is not None:  # every rank checked its own outputs
            t = torch.tensor([0.0 if check["bitexact"] else 1.0], dtype=torch.float64, device=f"cuda:{local}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            check["all_ranks_bitexact"] = float(t.item()) == 0.0
    algo_mv = algorithmic_bytes_per_matvec(N, L, args.n, args.batch, ks)
    if rank == 0:
        line = {
            "metric": ("CKKS matvec ciphertexts/sec (N=2^15, L=10)" if args.config == "cfg3" else
                       "CKKS matmul output columns/sec (1024x1024x1024, N=2^16, L=16)"),
            "value": round(value, 6), "unit": "matvec/s" if args.config == "cfg3" else "columns/s",
            "n_gpus": world, "rccl_world": dist.get_world_size() if dist is not None else 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": f"he_linalg BatchedMatrix::matmul diag x col, {args.n}x{args.n} "
                                   f"{'ct x pt' if ctpt else 'ct x ct'} matvec, N=2^{args.logn}, L={L}, "
                                   f"default Galois keys",
                       "batch_per_gpu": args.batch, "n": args.n, "key_switches_per_matvec": ks,
                       "parallelism": (f"sharded{world}: diagonals split by rotation-trie subtrees, one RCCL "
                                       f"reduce-scatter of size-3 partials" if sharded else
                                       f"replicated matrix+keys, dp{world} over input vectors"),
                       "batch_global": args.batch * (1 if sharded else world),
                       "precomputed_untimed": "per-Galois-key tables of the hoisted MAC (sign-mask NTTs W and "
                                              "key sums KW, galois_negw / galois_kw) are built once per key "
                                              "and level before the timed steps, like the keys themselves"},
            "roofline": roof,
            "self_check": check,
            "sharded": sharded_extra,
            "kernels_one_step": kernels,
            "cpu_baseline": cpu,
            "whole_step_algorithmic_GBps": round(algo_mv * total / dt / 1e9, 2),
            "whole_step_pmc_traffic": (pmc_step_traffic(list(kernels), args.batch, args.logn, L, args.n, args.variant)
                                       if kernels else None),
            "hbm": hbm,
            "breakdown_ms_one_step": breakdown,
            "profile_schedule": (None if args.no_profile else
                                 f"one untimed step ({prof['where']}), the batch of {args.batch} as one lane on the "
                                 f"context stream (the default schedule; with HEC_LANES > 1 profiling turns the "
                                 f"concurrent lanes off so each launch has the GPU to itself); asynchronous HIP event "
                                 f"pairs per launch"),
            "wall_s": {k: round(v, 2) for k, v in {**wall, "total_s": time.perf_counter() - wall0}.items()},
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()
    if check is not None and not (check["bitexact"] and check.get("all_ranks_bitexact", True)):
        print("bench.py: self-check: the timed outputs are NOT bit-exact (single call / profile step / oracle)",
              file=sys.stderr)
        sys.exit(1)
    if sharded_extra is not None and (sharded_extra.get("self_check") or {}).get("bitexact") is False:
        # a sharded step whose outputs differ from the 1-rank matvec is no valid measurement: fail the run
        print("bench.py: sharded self-check is NOT bit-exact against the 1-rank matvec", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
