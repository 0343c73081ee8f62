#!/bin/bash
# round 5: split-input Shoup butterflies in the fan-out kernels (HEC_SPLIT_BFLY 0 / 1 / 2): the key-switch parity
# subset under modes 1 and 3, then the bench alternating modes 0, 1, 2 (kernel times from the profile step)
set -u
OUT=gpurun_out/r05p
mkdir -p $OUT
for M in 1 3; do
  HEC_SPLIT_BFLY=$M timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or rescale or matvec or ntt" \
      > $OUT/tests_m$M.log 2>&1
  rc=$?
  echo "tests mode $M rc=$rc: $(tail -1 $OUT/tests_m$M.log)"
  if [ $rc -ne 0 ]; then tail -30 $OUT/tests_m$M.log; exit $rc; fi
done
for rep in 1 2; do
  for M in 0 1 2; do
    HEC_SPLIT_BFLY=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/m${M}_$rep.json 2> $OUT/m${M}_$rep.err
    rc=$?
    echo "mode=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/m${M}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],{n:k[n]['ms'] for n in ('k_fan2','k_fan2j','k_ntt')})" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/m${M}_$rep.err; exit $rc; fi
  done
done
