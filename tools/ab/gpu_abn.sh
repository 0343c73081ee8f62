#!/bin/bash
# N-way A/B: the in-tree library ("new") and variant .so files, alternating twice; the parity subset on the in-tree
# build first.  usage: bash tools/gpu_abn.sh <tag> <name>=<variant .so> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_he_math.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "new=" "$@"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], {n: (v['ms'], {r: x['ms'] for r, x in v['roles'].items()} if len(v['roles']) > 1 else None) for n, v in k.items()})"
  done
done
