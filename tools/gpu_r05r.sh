#!/bin/bash
# round 5: deferred tensor batches on a side stream (HEC_TENSOR_SIDE 1 vs 0): parity subset with both, the full-size
# lane test, then the bench alternating
set -u
OUT=gpurun_out/r05r
mkdir -p $OUT
for M in 1 0; do
  HEC_TENSOR_SIDE=$M timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or rescale or matvec or lanes" > $OUT/tests_$M.log 2>&1
  rc=$?
  echo "tests side=$M rc=$rc: $(tail -1 $OUT/tests_$M.log)"
  if [ $rc -ne 0 ]; then tail -30 $OUT/tests_$M.log; exit $rc; fi
done
for rep in 1 2; do
  for M in 0 1; do
    HEC_TENSOR_SIDE=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-profile --steps 2 --warmup 1 \
        > $OUT/s${M}_$rep.json 2> $OUT/s${M}_$rep.err
    rc=$?
    echo "side=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/s${M}_$rep.json'));print(d['value'],d['ms_per_step'],d['self_check'])" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/s${M}_$rep.err; exit $rc; fi
  done
done
