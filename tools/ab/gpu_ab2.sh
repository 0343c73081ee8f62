#!/bin/bash
# A/B of the in-tree library against a variant .so, alternating: parity subset on the in-tree build first.
# usage: bash tools/gpu_ab2.sh <tag> <variant .so> [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; V=$(realpath $2); shift 2
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_he_math.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for side in new base; do
    L=""; [ $side = base ] && L=$V
    HECDNA_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/$T/${side}_$i.json 2> gpurun_out/$T/${side}_$i.err || { tail gpurun_out/$T/${side}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${side}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$side', d['value'], {n: (v['ms'], {r: x['ms'] for r, x in v['roles'].items()} if len(v['roles']) > 1 else None) for n, v in k.items()})"
  done
done
