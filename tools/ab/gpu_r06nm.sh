#!/bin/bash
# round 6: non-temporal stores for the other large intermediates (HEC_NT_MASK builds: 1 fan-out target tiles, 2
# divide-and-round output, 4 hoisted MAC accumulators, 7 all), every run with HEC_NT_E=1 (the digits E, r06nt);
# parity with mask 7 first, then cfg3 B = 128 alternating, two reps
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06nm}
mkdir -p gpurun_out/$T
export HEC_NT_E=1
HECDNA_LIB=$(realpath variants/ntm7.so) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "hoisted or cfg3_matvec or keyswitch_variants" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "m0=" "m1=variants/ntm1.so" "m2=variants/ntm2.so" "m4=variants/ntm4.so" "m7=variants/ntm7.so"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()}, {r: v['ms'] for r, v in k['k_ntt']['roles'].items()})"
  done
done
echo done
