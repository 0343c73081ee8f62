"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs of the same one-step bench
command) into per-kernel HBM traffic JSON files that bench.py reads (profiles/<tag>_pmc_<kernel>_B<B>.json).
Development tool.

Correction (MI355X_MICROARCH.md, HBM): on gfx950 FETCH_SIZE tallies a wide coalesced streaming read at half its
bytes (calibrated for 16 B/lane); read bytes = 2 x FETCH_SIZE (kB = 1024 B).  WRITE_SIZE is exact for 16-B/lane
stores.  Kernels with 8-B/lane accesses (k_ntt, k_fan, k_tensor_multi) are outside that calibration: their
files also carry the raw counters and the ratio to the kernel's algorithmic bytes (bench.py's per-kernel
table) so the factor can be read off a known byte count.
usage: python tools/pmc_summary.py <fetch.csv> <write.csv> <batch> <logN> <level> <n> <tag> <cmd> <kernel>...
PMC_VARIANT=ctpt in the environment tags the files as the ct x pt matvec's (pmc_<kernel>_B<B>_ctpt.json)."""
import csv
import json
import os
import sys


def per_dispatch(path, kernel, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        base = name[name.find("k_"):].split("<")[0].split("(")[0] if "k_" in name else name
        if base == kernel and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    if os.environ.get("PMC_FIRST_HALF"):  # the run held the measured step, then an equal-length small call (a
        keep = sorted(vals)[: len(vals) // 2]  # bench self-check before round 5's --no-self-check): the step only
        vals = {k: vals[k] for k in keep}
    return vals


fetch_csv, write_csv, B, logN, level, n, tag, cmd = sys.argv[1:9]
variant = os.environ.get("PMC_VARIANT", "ctct")
outdir = os.path.dirname(os.path.abspath(fetch_csv))
for kernel in sys.argv[9:]:
    f = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
    w = per_dispatch(write_csv, kernel, "WRITE_SIZE")
    if not f or not w:
        continue
    fk = sum(f.values()) / len(f)
    wk = sum(w.values()) / len(w)
    res = {
        "kernel": kernel, "batch": int(B), "logN": int(logN), "level": int(level), "n": int(n),
        "variant": variant, "dispatches": len(f),
        "FETCH_SIZE_kB_per_dispatch": round(fk, 1), "WRITE_SIZE_kB_per_dispatch": round(wk, 1),
        "FETCH_SIZE_kB_per_step": round(sum(f.values()), 1), "WRITE_SIZE_kB_per_step": round(sum(w.values()), 1),
        "correction": "read bytes = 2 x FETCH_SIZE (gfx950 tallies coalesced streaming reads at half their bytes); "
                      "write bytes = WRITE_SIZE",
        "traffic_bytes_per_dispatch": int(round((2 * fk + wk) * 1024)),
        "traffic_bytes_per_step": int(round((2 * sum(f.values()) + sum(w.values())) * 1024)),
        "command": cmd,
    }
    path = os.path.join(outdir, f"pmc_{kernel}_B{B}{'' if variant == 'ctct' else '_' + variant}.json")
    json.dump(res, open(path, "w"), indent=1)
    print(json.dumps(res))
