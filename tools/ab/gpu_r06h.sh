#!/bin/bash
# round 6: the wave-shuffle pass B after the scratch fix (DPP lane moves, fixed register indices): parity of modes
# 1 and 2, then cfg2 with shfl 0 / 1 / 2 and cfg3 at B = 128 with shfl 0 / 2, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06h}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "shuffle or test_ntt_bitexact" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for sh in 0 1 2; do
    HEC_NTTB_SHFL=$sh timeout -k 10 200 python bench.py --config cfg2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/$T/cfg2_s${sh}_$i.json 2> gpurun_out/$T/cfg2_s${sh}_$i.err || { tail -3 gpurun_out/$T/cfg2_s${sh}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/cfg2_s${sh}_$i.json').read().strip().splitlines()[-1])
print('cfg2 s$sh', d['value'], {k: v['ms'] for k, v in d['kernels_one_step'].items()})"
  done
done
for i in 1 2; do
  for sh in 0 2; do
    HEC_NTTB_SHFL=$sh timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/s${sh}_$i.json 2> gpurun_out/$T/s${sh}_$i.err || { tail gpurun_out/$T/s${sh}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/s${sh}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('s$sh', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, k['k_ntt'].get('roles', {}).get('modup_h_b'), d.get('hbm'))"
  done
done
echo done
