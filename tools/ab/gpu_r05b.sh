#!/bin/bash
# round 5: batch lanes A/B at the bench default (B = 192), alternating, with the world-1 self-check
set -u
OUT=gpurun_out/r05b
mkdir -p $OUT
for rep in 1 2; do
  for L in 3 1; do
    HEC_LANES=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 \
        > $OUT/lanes${L}_$rep.json 2> $OUT/lanes${L}_$rep.err
    rc=$?
    echo "lanes=$L rep=$rep rc=$rc $(python3 -c "import json,sys;d=json.load(open('$OUT/lanes${L}_$rep.json'));print(d['value'],d['ms_per_step'],d['self_check'])" 2>&1)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
