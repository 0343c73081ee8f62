#!/bin/bash
# round 6: parity subset on the in-tree k_hmacm (MAC form, double-buffered keys, separate zero-correction kernel),
# the staging fix and the wave-shuffle pass B; then cfg3 A/B new vs base and shuffle on/off, and cfg2 new (shuffle
# off/on) vs the round-4 tree, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06g}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or keyswitch or hoisted or matvec or cfg3 or shuffle" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "new=:0" "shfl=:1" "base=variants/base_r06.so:0"; do
    name=${v%%=*}; rest=${v#*=}; lib=${rest%%:*}; sh=${rest##*:}; [ -n "$lib" ] && lib=$(realpath $lib)
    HEC_NTTB_SHFL=$sh HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()})"
  done
done
for i in 1 2; do
  for sh in 0 1; do
    HEC_NTTB_SHFL=$sh timeout -k 10 200 python bench.py --config cfg2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/$T/cfg2_new${sh}_$i.json 2> gpurun_out/$T/cfg2_new${sh}_$i.err || { tail -3 gpurun_out/$T/cfg2_new${sh}_$i.err; exit 1; }
  done
  (cd variants/r04a_tree && timeout -k 10 200 python bench.py --config cfg2 --steps 50 --warmup 5 --no-cpu-baseline) > gpurun_out/$T/cfg2_r04a_$i.json 2> gpurun_out/$T/cfg2_r04a_$i.err || { tail -3 gpurun_out/$T/cfg2_r04a_$i.err; exit 1; }
  for v in new0 new1 r04a; do python3 -c "
import json; d=json.loads(open('gpurun_out/$T/cfg2_${v}_$i.json').read().strip().splitlines()[-1])
print('cfg2 $v', d['value'], d.get('self_check', {}).get('bitexact'), {k: v['ms'] for k, v in d['kernels_one_step'].items()})"; done
done
echo done
