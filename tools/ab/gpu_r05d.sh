#!/bin/bash
# round 5: parity of the group-launch hoisted MAC, then A/B of HEC_HMAC=2 (group) vs 1 (pairs) at the bench default
set -u
OUT=gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "variants or zero or lanes or matvec or rotate" > $OUT/parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -3 $OUT/parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for H in 2 1; do
    HEC_HMAC=$H timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/hmac${H}_$rep.json 2> $OUT/hmac${H}_$rep.err
    rc=$?
    echo "hmac=$H rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/hmac${H}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],'hmacm',k['k_hmacm']['ms'],k['k_hmacm']['GBps'])" 2>&1)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
