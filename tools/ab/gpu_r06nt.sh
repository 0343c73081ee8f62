#!/bin/bash
# round 6: the hoisted digits E stored non-temporally (HEC_NT_E=1) — does the MAC that reads them next run faster
# when the tile's lines are not kept for reuse (the r06u/r06v observation)?  Parity subset with the flag, then cfg3
# B = 128 A/B on one library, alternating, three reps
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06nt}
mkdir -p gpurun_out/$T
HEC_NT_E=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "hoisted or cfg3_matvec" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2 3; do
  for nt in 0 1; do
    HEC_NT_E=$nt timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/nt${nt}_$i.json 2> gpurun_out/$T/nt${nt}_$i.err || { tail gpurun_out/$T/nt${nt}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/nt${nt}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('nt$nt', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, k['k_ntt']['roles']['modup_h_b']['ms'])"
  done
done
echo done
