#!/bin/bash
# round 5: shapes of the sibling-group k_hmacm (HEC_HMAC_SHAPE) — parity, then A/B at the bench default
set -u
OUT=gpurun_out/r05j
mkdir -p $OUT
for S in 1 2 3 4; do
  HEC_HMAC_SHAPE=$S timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_parity.py -k "zero or (matvec and not lanes)" > $OUT/parity_$S.log 2>&1
  rc=$?
  echo "shape $S parity rc=$rc $(tail -1 $OUT/parity_$S.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for rep in 1 2; do
  for S in 0 3 4 1 2; do
    if [ $rep = 2 ] && { [ $S = 1 ] || [ $S = 2 ]; }; then continue; fi
    HEC_HMAC_SHAPE=$S timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/s${S}_$rep.json 2> $OUT/s${S}_$rep.err
    rc=$?
    echo "shape=$S rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/s${S}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],'hmacm',k['k_hmacm']['ms'])" 2>&1 | tail -1)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
