#!/bin/bash
# round 6: k_hmacm on MAC-form operands — parity (key-switch variants, hoisted zero corrections, matvecs, cfg3 / cfg5
# subsets) on the in-tree build, then the bench A/B against variants/base_r06.so (alternating, two reps)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06b}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "keyswitch or hoisted or matvec or rotate or cfg3_bench_schedule or cfg5_subset" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "new=" "base=variants/base_r06.so"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()})"
  done
done
