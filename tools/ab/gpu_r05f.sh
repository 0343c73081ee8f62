#!/bin/bash
# round 5: bench batch sweep at the one-lane default (B = 192 / 256 / 288), alternating
set -u
OUT=gpurun_out/r05f
mkdir -p $OUT
for rep in 1 2; do
  for B in 192 256 288; do
    timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 --batch $B \
        > $OUT/b${B}_$rep.json 2> $OUT/b${B}_$rep.err
    rc=$?
    echo "B=$B rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/b${B}_$rep.json'));print(d['value'],d['ms_per_step'],d['self_check']['bitexact'])" 2>&1 | tail -1)"
    if [ $rc -ne 0 ]; then tail -3 $OUT/b${B}_$rep.err; exit $rc; fi
  done
done
