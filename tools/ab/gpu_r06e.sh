#!/bin/bash
# round 6: k_hmacm FP64 targets on the MAC-form loop + 60-bit targets on the u64 loop (in-tree) vs the all-MAC-form
# BTI=1 variant vs base; parity subset on the in-tree build; SQ counters of k_hmacm for in-tree and base
set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06e
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "keyswitch or hoisted or matvec or cfg3_bench_schedule" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for v in "new=" "base=variants/base_r06.so" "bti1=variants/hmac_bti1.so"; do
    name=${v%%=*}; lib=${v#*=}; [ -n "$lib" ] && lib=$(realpath $lib)
    HECDNA_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/${name}_$i.json 2> gpurun_out/$T/${name}_$i.err || { tail gpurun_out/$T/${name}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${name}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$name', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()})"
  done
done
KRE=k_hmacm SQ_B=128 bash tools/gpu_sq.sh ${T}_sq_new > /dev/null || exit 1
HECDNA_LIB=$(realpath variants/base_r06.so) KRE=k_hmacm SQ_B=128 bash tools/gpu_sq.sh ${T}_sq_base > /dev/null || exit 1
for v in new base; do
  SQ_BY_INSTANCE=1 python tools/sq_summary.py gpurun_out/${T}_sq_$v/p1/run_counter_collection.csv gpurun_out/${T}_sq_$v/p2/run_counter_collection.csv "k_hmacm B=128 ($v)" > gpurun_out/${T}_sq_$v/sq.json || exit 1
done
