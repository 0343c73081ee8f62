#!/bin/bash
# quick A/B: a few parity tests of the hoisted path, then the bench under each env setting given.
# usage: bash tools/gpu_ab.sh <tag> "ENV=1 ENV2=3" "ENV=0" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "keyswitch_variants or hoisted or lane or cfg3_matvec or cfg5_params" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/$T/bench_$i.json 2> gpurun_out/$T/bench_$i.err || { tail gpurun_out/$T/bench_$i.err; exit 1; }
  echo "$e: $(head -c 120 gpurun_out/$T/bench_$i.json)"
done
