"""bench.py's measurement formulas (CPU): the algorithmic bytes per matvec restate SURVEY §8(d), the
key-switch counts are SEAL's NAF schedule and the trie's, and tools/profile_step.py picks the profile
step's dispatches out of a kernel trace."""
import csv
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


@pytest.mark.parametrize("B,gb", [(1, 1283.76), (8, 346.29), (64, 229.11)])
def test_algorithmic_bytes_match_survey(bench, B, gb):
    # cfg3, KS = 18,204 -> 1,283.76 / 346.29 / 229.11 GB per matvec at B = 1 / 8 / 64
    assert round(bench.algorithmic_bytes_per_matvec(1 << 15, 10, 4096, B, 18204) / 1e9, 2) == gb


def test_key_switch_counts(bench):
    from _helpers import rotation_trie_stats
    assert bench.ks_total(1 << 15, 4096) == 18204  # SEAL's schedule, SURVEY §8(a)
    assert bench.ks_total(1 << 13, 64) == 156
    ks, hoisted, children, others = rotation_trie_stats(1 << 15, 4096)
    assert (ks, hoisted, children, others) == (5460, 1024, 4436, 1024)
    assert rotation_trie_stats(1 << 16, 1024)[0] == 1364  # cfg5


def test_launcher_command(bench):
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "3"], 29512)
    assert cmd[1:8] == ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8", "--master-addr=127.0.0.1",
                        "--master-port=29512", os.path.join(ROOT, "bench.py")]
    assert cmd[8:] == ["--gpus", "8", "--steps", "3"]


@pytest.mark.parametrize("gpus", [2, 4])
def test_gpus_n_launches_n_ranks_one_line(gpus):
    """`bench.py --gpus N` with no WORLD_SIZE starts N ranks itself (gloo dry run: no GPU) and exactly one JSON line
    comes out, from rank 0, with the world size the process group saw."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run", "--steps",
                          "2", "--warmup", "1"], capture_output=True, text=True, env=env, timeout=300, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == gpus and r["rccl_world"] == gpus and r["dry_run"] and r["steps"] == 2


def test_whole_step_pmc_traffic(bench):
    """The line's whole-step PMC figure: the committed round-6 passes at the bench shape sum to the per-kernel traffic
    per matvec (399 GB); a kernel without a pass on that shape, or another shape, gives None rather than
    a partial sum."""
    ks = ["k_bmac", "k_fan2", "k_fan2j", "k_hmacm", "k_ntt", "k_tensor_multi2"]
    t = bench.pmc_step_traffic(ks, 128, 15, 10, 4096)
    assert t is not None and 390 < t["GB_per_matvec"] < 410 and set(t["by_kernel"]) == set(ks)
    assert t["source"].startswith("profiles/r06_pmc_")
    assert bench.pmc_step_traffic(ks + ["k_moddown1"], 128, 15, 10, 4096) is None
    assert bench.pmc_step_traffic(ks, 128, 15, 10, 2048) is None


def test_replicated_seeds_do_not_depend_on_rank(bench):
    """The keys and the matrix diagonals are the replicated state of every rank: their seeds must be the
    same on every rank, or a sharded step sums partials computed under different keys.  Throughput mode gives each rank
    its own input vectors; sharded mode splits one batch, the same on every rank."""
    for sharded in (False, True):
        s0 = bench.bench_seeds(0, sharded)
        for r in range(1, 8):
            s = bench.bench_seeds(r, sharded)
            assert (s["relin"], s["galois"], s["diag"]) == (s0["relin"], s0["galois"], s0["diag"])
            assert (s["col"] == s0["col"]) == sharded
    assert bench.bench_seeds(3, True)["col"] == bench.bench_seeds(0, False)["col"]  # the sharded leg's batch = rank 0's


def test_cpu_leg_sizing(bench, monkeypatch):
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: None)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    model, host, share, threads, why = bench.cpu_info()
    assert threads == 1 or share == 1
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 1)
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_info()[3] == 1


def test_profile_step_tool(tmp_path):
    # 3 timed steps x 2 dispatches (lanes) then a 2-dispatch profile step of 10 us each
    trace = tmp_path / "trace.csv"
    with open(trace, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        t = 0
        for d in [30_000] * 6 + [10_000, 10_000]:
            w.writerow(["void hec::k_hmacm<4, 2, 2, 3>(...)", t, t + d])
            w.writerow(["void hec::k_ntt<...>(...)", t + d, t + d + 5])
            t += d + 100
    benchj = tmp_path / "bench.json"
    benchj.write_text(json.dumps({"roofline": {"kernel": "k_hmacm", "launches_per_step": 2, "avg_ms": 0.0101}}))
    out = tmp_path / "out.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "profile_step.py"), str(trace), str(benchj),
                           str(out)], stdout=subprocess.DEVNULL)
    r = json.load(open(out))
    assert r["profile_step_dispatches"] == 2 and r["profile_step_avg_us"] == 10.0
    assert r["all_dispatches"] == 8 and r["event_timed_avg_us"] == 10.1


@pytest.mark.parametrize("fail", [None, "prepare:1", "prepare:0", "run:1", "selfcheck:0"])
def test_dry_run_sharded_leg_never_strands_a_rank(fail):
    """the sharded extra leg after the metric (bench.sharded_extra_leg, the same control flow the
    GPU run uses) reaches every collective on every rank whatever fails where: an exception on one rank in the
    preparation, in the sharded call before its agreement, or in rank 0's self-check.  World 2 over gloo; the run must
    end (timeout) with exactly one line, the metric intact and the failure reported in 'sharded'."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "1"]
    if fail:
        cmd += ["--dry-run-fail", fail]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    sh = json.loads(lines[0])["sharded"]
    if fail is None:
        assert sh["value"] > 0 and sh["self_check"]["bitexact"] is True
    elif fail.startswith("prepare"):
        assert sh["error"].startswith("preparation failed on rank " + fail[-1])
    elif fail.startswith("run"):
        assert "error" in sh and "value" not in sh
    else:
        assert sh["value"] > 0 and "injected" in sh["self_check"]["error"] and sh["self_check"]["bitexact"] is None
