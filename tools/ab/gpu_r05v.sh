#!/bin/bash
# round 5: split-input butterflies in k_bmac's integer-target pass B (HEC_BMAC_SPLIT 1, 6 VGPRs spilled at 4 waves/SIMD)
# vs plain Shoup (0): parity subset under 1, then the bench alternating
set -u
OUT=gpurun_out/r05v
mkdir -p $OUT
HEC_BMAC_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or matvec or rotate" > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc: $(tail -1 $OUT/tests.log)"
if [ $rc -ne 0 ]; then tail -30 $OUT/tests.log; exit $rc; fi
for rep in 1 2; do
  for M in 0 1; do
    HEC_BMAC_SPLIT=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/b${M}_$rep.json 2> $OUT/b${M}_$rep.err
    rc=$?
    echo "bmac_split=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/b${M}_$rep.json'));k=d['kernels_one_step']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],{n:k[n]['ms'] for n in ('k_bmac','k_fan2j')})" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/b${M}_$rep.err; exit $rc; fi
  done
done
