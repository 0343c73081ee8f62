"""rocprofv3 kernel-trace average of the roofline kernel over bench.py's profile step only (development
tool).  bench.py times its steps (one lane by default since round 5; concurrent lanes with HEC_LANES=3), then runs
one extra step as a single lane with HIP event pairs (the roofline's avg_ms), its last GPU work; that step's
dispatches are the roofline kernel's last `launches_per_step` dispatches in the trace.
usage: python tools/profile_step.py <run_kernel_trace.csv> <bench.json> <out.json>"""
import csv
import json
import sys

trace, bench, out = sys.argv[1:4]
line = json.loads(open(bench).read().strip().splitlines()[-1])
roof = line["roofline"]
kern, nlast = roof["kernel"], roof["launches_per_step"]
by_kernel = {}
for r in csv.DictReader(open(trace)):
    name = r["Kernel_Name"]
    base = name[name.find("k_"):].split("<")[0].split("(")[0] if "k_" in name else name
    by_kernel.setdefault(base, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for v in by_kernel.values():
    v.sort()
durs = by_kernel.get(kern, [])
last = [d for _, d in durs[-nlast:]]
res = {"kernel": kern, "profile_step_dispatches": len(last),
       "profile_step_avg_us": round(sum(last) / len(last) / 1e3, 2),
       "event_timed_avg_us": round(roof["avg_ms"] * 1e3, 2),
       "all_dispatches": len(durs), "all_dispatch_avg_us": round(sum(d for _, d in durs) / len(durs) / 1e3, 2),
       "note": "the profile step runs the batch as one lane, as the event-timed roofline does (the timed steps "
               "too unless HEC_LANES > 1)"}
# every kernel of the bench's per-kernel table over the same profile step (its last `launches` dispatches):
# rocprof's own time shares for the single-lane step, to set beside the whole-run stats CSV, whose shares
# are inflated for kernels that overlap each other in the concurrent lanes
step = {}
for k, v in line.get("kernels_one_step", {}).items():
    d = by_kernel.get(k, [])[-v["launches"]:]
    if d:
        step[k] = {"rocprof_ms": round(sum(x for _, x in d) / 1e6, 3), "event_ms": v["ms"], "dispatches": len(d)}
tot = sum(v["rocprof_ms"] for v in step.values()) or 1.0
for v in step.values():
    v["share"] = round(v["rocprof_ms"] / tot, 3)
res["profile_step_kernels"] = step
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
