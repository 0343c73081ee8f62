#!/bin/bash
# round 5: the mod-up pass B capped at 128 VGPRs for a fourth wave per SIMD (HEC_PASSB_W4=1, 8 VGPRs spilled) vs its
# 132 VGPRs at 3 waves (0), alternating on one box
set -u
OUT=gpurun_out/r05za
mkdir -p $OUT
for rep in 1 2; do
  for M in 0 1; do
    HEC_PASSB_W4=$M timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 --warmup 1 \
        > $OUT/w${M}_$rep.json 2> $OUT/w${M}_$rep.err
    rc=$?
    echo "w4=$M rep=$rep rc=$rc $(python3 -c "
import json;d=json.load(open('$OUT/w${M}_$rep.json'));k=d['kernels_one_step']['k_ntt']['roles']
print(d['value'],d['ms_per_step'],d['self_check']['bitexact'],k['modup_h_b'],k.get('divround_b'))" 2>&1)"
    if [ $rc -ne 0 ]; then tail -5 $OUT/w${M}_$rep.err; exit $rc; fi
  done
done
