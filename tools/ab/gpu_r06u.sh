#!/bin/bash
# round 6: the mod-up pass B's XOR-swizzled LDS rows (16-B pair slots, no padding) — parity of the hoisted paths,
# SQ bank conflicts of the new kernel, then cfg3 B = 128 A/B against variants/pre_swz.so (padded rows), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06u}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "keyswitch or hoisted or matvec or cfg3 or cfg5_params" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
KRE=k_ntt SQ_B=128 bash tools/gpu_sq.sh ${T}_sq > gpurun_out/$T/sq.log 2>&1 || { tail gpurun_out/$T/sq.log; exit 1; }
for i in 1 2; do
  for v in "swz=" "pad=variants/pre_swz.so"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, {r: v['ms'] for r, v in k['k_ntt']['roles'].items()})"
  done
done
echo done
