#!/bin/bash
# round 6: (1) the shard tests alone with a per-test timeout below the 180 s silence limit (r06k went silent in
# test_sharded_partials_sum_to_full_matvec[5]; pytest-timeout dumps the stack if it recurs); (2) parity of the
# split-product 60-bit MAC (HEC_HMAC_INT=2, also cfg5 at l = 16, the bound of its sums); (3) int 1 / 2 A/B at cfg3
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r06l}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/shard.log 2>&1 || { tail -60 gpurun_out/$T/shard.log; exit 1; }
tail -2 gpurun_out/$T/shard.log
HEC_HMAC_INT=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 --timeout-method thread -k "keyswitch or hoisted or matvec_batched or cfg3_bench_schedule or cfg5_params" > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
for i in 1 2; do
  for hi in 1 2; do
    HEC_HMAC_INT=$hi timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/$T/int${hi}_$i.json 2> gpurun_out/$T/int${hi}_$i.err || { tail gpurun_out/$T/int${hi}_$i.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/$T/int${hi}_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('int$hi', d['value'], d['self_check']['bitexact'], {n: v['ms'] for n, v in k.items()})"
  done
done
echo done
