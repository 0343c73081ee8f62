"""Summarise the two SQ-counter passes of tools/gpu_sq.sh into per-kernel totals and fractions (development tool).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* are in quad-cycles; the fractions divide by SQ_WAVE_CYCLES (per wave).
usage: [SQ_BY_INSTANCE=1] python tools/sq_summary.py <p1/run_counter_collection.csv> <p2/...csv> <command text> > out.json
SQ_BY_INSTANCE=1: one entry per template instantiation instead of per kernel."""
import collections
import csv
import json
import os
import sys

BY_INST = os.environ.get("SQ_BY_INSTANCE") == "1"
tot = collections.defaultdict(collections.Counter)
disp = collections.defaultdict(set)
for path in sys.argv[1:3]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        base = name[name.find("k_"):].split("<")[0].split("(")[0] if "k_" in name else name
        if BY_INST:  # one entry per template instantiation (the IO class names the k_ntt role)
            base = name[name.find("k_"):].split("(")[0] if "k_" in name else name
        tot[base][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[base].add((path, r["Dispatch_Id"]))
out = {"command": sys.argv[3], "kernels": {}}
for k, c in sorted(tot.items()):
    d = {n: int(v) for n, v in sorted(c.items())}
    d["dispatches"] = len(disp[k]) // 2
    if c["SQ_WAVE_CYCLES"]:
        d["wait_any_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3)
        d["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 3)
    if c["SQ_INSTS_LDS"]:
        d["lds_bank_conflict_per_lds_inst"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"], 3)
    out["kernels"][k] = d
json.dump(out, sys.stdout, indent=1)
