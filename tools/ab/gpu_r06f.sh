#!/bin/bash
# round 6: k_hmacm variants (in-tree: one key buffer reloaded per child + 2-wide products + separate zero-correction
# kernel; vb: double-buffered keys, sequential products) vs base; then cfg2 with the current tree vs the round-4 tree
# (commit 04c4cc7, variants/r04a_tree) on the same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06f
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "keyswitch or hoisted or matvec or cfg3_bench_schedule" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "new=" "vb=variants/hmac_vb.so" "base=variants/base_r06.so"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()})"
  done
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --config cfg2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/$T/cfg2_new_$i.json 2> gpurun_out/$T/cfg2_new_$i.err || { tail -3 gpurun_out/$T/cfg2_new_$i.err; exit 1; }
  (cd variants/r04a_tree && timeout -k 10 200 python bench.py --config cfg2 --steps 50 --warmup 5 --no-cpu-baseline) > gpurun_out/$T/cfg2_r04a_$i.json 2> gpurun_out/$T/cfg2_r04a_$i.err || { tail -3 gpurun_out/$T/cfg2_r04a_$i.err; exit 1; }
  for v in new r04a; do python3 -c "
import json; d=json.loads(open('gpurun_out/$T/cfg2_${v}_$i.json').read().strip().splitlines()[-1])
print('cfg2 $v', d['value'], {k: v['ms'] for k, v in d['kernels_one_step'].items()})"; done
done
