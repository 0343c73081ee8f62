#!/bin/bash
# round 6: the hoisted MAC's 60-bit targets on split sums in their own launch (HEC_HMAC_INT=2, k_hmacm_i) — parity
# (key-switch variants, hoisted zero corrections, cfg3 and cfg5 subsets, the new cfg3 test), then cfg3 B = 128 A/B
# int 1 / int 2, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06z}
mkdir -p gpurun_out/$T
HEC_HMAC_INT=2 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "keyswitch or hoisted or matvec or cfg3 or cfg5 or split_sum" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for hi in 1 2; do
    HEC_HMAC_INT=$hi timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/int${hi}_$i.json 2> gpurun_out/$T/int${hi}_$i.err || { tail gpurun_out/$T/int${hi}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/int${hi}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('int$hi', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()})"
  done
done
echo done
