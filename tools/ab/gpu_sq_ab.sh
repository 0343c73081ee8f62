#!/bin/bash
# SQ counters of one kernel regex under two engine settings (n = 512 bench, one lane).
# usage: bash tools/gpu_sq_ab.sh <tag> <kernel-regex> "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; RE=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HEC_LANES=1
i=0
for envs in "$@"; do
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64"; do
    p=$((p+1))
    env $envs timeout -k 10 120 rocprofv3 --pmc $pass --kernel-include-regex "$RE" --output-format csv -d $OUT/s${i}_$p -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 512 --no-cpu-baseline --no-profile --steps 1 --warmup 0 > $OUT/s${i}_$p.log 2>&1 || { tail $OUT/s${i}_$p.log; exit 1; }
  done
  python3 - "$envs" $OUT/s${i}_* <<'PY'
import csv, sys, glob, collections
tot = collections.Counter(); disp = set()
for d in sys.argv[2:]:
    for f in glob.glob(d + "/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add((d, r["Dispatch_Id"]))
t = tot
print(sys.argv[1], "dispatches", len(disp) // 2, {k: int(v) for k, v in sorted(t.items())})
if t["SQ_WAVE_CYCLES"]:
    print("  wait_any %.3f valu_active %.3f lds_conflict/lds_inst %.3f busy %d" % (t["SQ_WAIT_ANY"] / t["SQ_WAVE_CYCLES"], t["SQ_ACTIVE_INST_VALU"] / t["SQ_WAVE_CYCLES"], t["SQ_LDS_BANK_CONFLICT"] / max(1, t["SQ_INSTS_LDS"]), t["SQ_BUSY_CYCLES"]))
PY
  i=$((i+1)); p=0
done
