#!/bin/bash
# round 5: k_fan2j with split-input butterflies in its scalar-twiddle round only (HEC_SPLIT_BFLY=4) vs the default 1
set -u
OUT=gpurun_out/r05s
mkdir -p $OUT
HEC_SPLIT_BFLY=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or matvec" > $OUT/tests.log 2>&1
rc=$?
echo "tests mode 4 rc=$rc: $(tail -1 $OUT/tests.log)"
if [ $rc -ne 0 ]; then tail -30 $OUT/tests.log; exit $rc; fi
for rep in 1 2; do
  for M in 1 4; do
    HEC_SPLIT_BFLY=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/m${M}_$rep.json 2> $OUT/m${M}_$rep.err
    rc=$?
    echo "mode=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/m${M}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],{n:k[n]['ms'] for n in ('k_fan2','k_fan2j')})" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/m${M}_$rep.err; exit $rc; fi
  done
done
