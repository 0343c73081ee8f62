"""Collect the bench lines of one A/B directory (gpurun_out/<tag>/<name>_<rep>.json, one JSON line each) into one
summary file under profiles/ (development tool).
usage: python tools/ab_collect.py gpurun_out/<tag> profiles/<tag>_<what>.json "<what was compared, and how>"
"""
import json
import os
import sys


def main():
    src, out, what = sys.argv[1], sys.argv[2], sys.argv[3]
    runs = []
    for fn in sorted(os.listdir(src)):
        if not fn.endswith(".json"):
            continue
        txt = open(os.path.join(src, fn)).read().strip().splitlines()
        if not txt:
            continue
        try:
            d = json.loads(txt[-1])
        except json.JSONDecodeError:
            continue
        stem = fn[:-5]
        name, _, rep = stem.rpartition("_")
        k = d.get("kernels_one_step") or {}
        run = {"run": name or stem, "rep": int(rep) if rep.isdigit() else rep, "value": d.get("value"),
               "unit": d.get("unit"), "ms_per_step": d.get("ms_per_step"),
               "batch": (d.get("config") or {}).get("batch_per_gpu"),
               "self_check_bitexact": (d.get("self_check") or {}).get("bitexact"),
               "kernel_ms_one_step": {n: v.get("ms") for n, v in k.items()}}
        roles = (k.get("k_ntt") or {}).get("roles")
        if roles:
            run["k_ntt_roles_ms"] = {r: v.get("ms") for r, v in roles.items()}
        if d.get("hbm"):
            run["hbm"] = d["hbm"]
        runs.append(run)
    json.dump({"what": what, "source": src, "runs": runs}, open(out, "w"), indent=1)
    print(out, len(runs), "runs")


if __name__ == "__main__":
    main()
