#!/bin/bash
# round 6: bench batch sweep at one lane (B = 128 / 96 / 144 / 192), SQ counters at B = 192 (tools/gpu_sq.sh), cfg2,
# then a second sweep rep
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06a
mkdir -p $OUT
sweep() {
  for B in 128 96 144 192; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-profile --steps 3 --warmup 1 --batch $B \
        > $OUT/b${B}_$1.json 2> $OUT/b${B}_$1.err
    rc=$?
    echo "B=$B rep=$1 rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/b${B}_$1.json'));print(d['value'],d['ms_per_step'],d['self_check']['bitexact'])" 2>&1 | tail -1)"
    if [ $rc -ne 0 ]; then tail -3 $OUT/b${B}_$1.err; exit $rc; fi
  done
}
sweep 1
bash tools/gpu_sq.sh r06a_sq > /dev/null || exit 1
SQ_BY_INSTANCE=1 python tools/sq_summary.py gpurun_out/r06a_sq/p1/run_counter_collection.csv gpurun_out/r06a_sq/p2/run_counter_collection.csv "tools/gpu_sq.sh (bench --n 512 --batch 192, HEC_LANES=1)" > gpurun_out/r06a_sq/sq_by_instance.json || exit 1
python tools/sq_summary.py gpurun_out/r06a_sq/p1/run_counter_collection.csv gpurun_out/r06a_sq/p2/run_counter_collection.csv "tools/gpu_sq.sh (bench --n 512 --batch 192, HEC_LANES=1)" > gpurun_out/r06a_sq/sq.json || exit 1
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --config cfg2 --steps 50 --warmup 5 > $OUT/cfg2_$rep.json 2> $OUT/cfg2_$rep.err || { tail -3 $OUT/cfg2_$rep.err; exit 1; }
  head -c 300 $OUT/cfg2_$rep.json; echo
done
sweep 2
