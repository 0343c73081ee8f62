#!/bin/bash
# round 5: k_hmacb (HEC_HMAC=3, the FP64 targets' hoisted digit pass B inside the sibling-group MAC): parity subset
# under HMAC=3, then the bench alternating HMAC 2 / 3
set -u
OUT=gpurun_out/r05q
mkdir -p $OUT
HEC_HMAC=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or rescale or matvec" > $OUT/tests.log 2>&1
rc=$?
echo "tests HMAC=3 rc=$rc: $(tail -1 $OUT/tests.log)"
if [ $rc -ne 0 ]; then tail -30 $OUT/tests.log; exit $rc; fi
for rep in 1 2; do
  for M in 2 3; do
    HEC_HMAC=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/h${M}_$rep.json 2> $OUT/h${M}_$rep.err
    rc=$?
    echo "hmac=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/h${M}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],{n:(k[n]['ms'],k[n]['launches']) for n in k})" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/h${M}_$rep.err; exit $rc; fi
  done
done
