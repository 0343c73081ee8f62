#!/bin/bash
# A/B/n: the key-switch parity subset on the in-tree library, then one bench per setting (development tool).
# usage: bash tools/gpu_ab_n.sh <tag> "<env settings or empty>" ...   (HECDNA_LIB=... selects an experiment library)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or cfg5 or rescale or matvec or ntt" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/bench_$i.json 2> gpurun_out/$T/bench_$i.err || { tail gpurun_out/$T/bench_$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/$T/bench_$i.json')); k=d['kernels_one_step']
print('$e'.ljust(40), d['value'], {n: k[n]['ms'] for n in k}, {r: v['ms'] for r, v in k['k_ntt']['roles'].items()})"
done
