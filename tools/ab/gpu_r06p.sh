#!/bin/bash
# round 6: the single-pass mod-down (HEC_MODDOWN1, k_moddown1) — parity at cfg3 first, then cfg3 B = 128 A/B against
# the two-pass mod-down, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06p}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "single_pass_moddown or cfg3_rotations" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for md in 0 1; do
    HEC_MODDOWN1=$md timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/md${md}_$i.json 2> gpurun_out/$T/md${md}_$i.err || { tail gpurun_out/$T/md${md}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/md${md}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('md$md', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, {r: v['ms'] for r, v in k['k_ntt']['roles'].items()})"
  done
done
echo done
