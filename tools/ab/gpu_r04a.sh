#!/bin/bash
# round-4 box: the new tests first, then the GPU suite, then the bench under the default and each A/B variant
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r04a}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_he_math.py tests/test_gpu_encode.py tests/test_gpu_seal_io.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/new_tests.log 2>&1 || { tail -40 gpurun_out/$T/new_tests.log; exit 1; }
tail -2 gpurun_out/$T/new_tests.log
bash tools/gpu_tests.sh $T || exit 1
i=0
for e in "HEC_X=1" "HEC_FAN_OCC=3" "HEC_PRE_EARLY=0" "HEC_TENSOR_XCD=0" "HEC_X=1" "HEC_FAN_OCC=3"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/$T/bench_$i.json 2> gpurun_out/$T/bench_$i.err || { tail gpurun_out/$T/bench_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/$T/bench_$i.json').read().strip().splitlines()[-1]); k=d['kernels_one_step']
print('$e', d['value'], {n: v['ms'] for n, v in k.items()})"
done
timeout -k 10 300 python bench.py --config cfg2 > gpurun_out/$T/cfg2.json 2> gpurun_out/$T/cfg2.err || { tail gpurun_out/$T/cfg2.err; exit 1; }
head -c 600 gpurun_out/$T/cfg2.json
