#!/bin/bash
# round 6: the swizzled mod-up pass B rows against the padded ones again, on another box (r06u: step +0.5 %, the
# mod-up pass B itself -1.8 %, the following k_hmacm +2.8 %), three alternating reps
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06v}
mkdir -p gpurun_out/$T
for i in 1 2 3; do
  for v in "swz=" "pad=variants/pre_swz.so"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, {r: v['ms'] for r, v in k['k_ntt']['roles'].items()})"
  done
done
echo done
