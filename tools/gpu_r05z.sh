#!/bin/bash
# round 5: chunks per block of the hoisted digits' pass B at N = 2^15 (HEC_MODUP_NB 16 = 129 VGPRs, 3 waves/SIMD;
# 8 = 126 VGPRs, 4 waves; 4 = half-wave blocks), alternating on one box
set -u
OUT=gpurun_out/r05z
mkdir -p $OUT
for rep in 1 2; do
  for M in 16 8 4; do
    HEC_MODUP_NB=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/nb${M}_$rep.json 2> $OUT/nb${M}_$rep.err
    rc=$?
    echo "nb=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/nb${M}_$rep.json'));k=d['kernels_one_step']['k_ntt']['roles']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],k['modup_h_b'])" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/nb${M}_$rep.err; exit $rc; fi
  done
done
