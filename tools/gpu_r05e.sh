#!/bin/bash
# round 5: parity of the grouped divide-and-round pass B, then A/B vs the previous commit's library
set -u
OUT=gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "variants or zero or lanes or matvec or rotate" > $OUT/parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -3 $OUT/parity.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for V in new old; do
    if [ $V = old ]; then export HECDNA_LIB=$PWD/tools/variants/prev/libhecdna.so; else unset HECDNA_LIB; fi
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 > $OUT/${V}_$rep.json 2> $OUT/${V}_$rep.err
    rc=$?
    echo "$V rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/${V}_$rep.json'));k=d['kernels_one_step']['k_ntt']['roles']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],'divround_b',k['divround_b'])" 2>&1)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
