#!/bin/bash
# Throughput vs batch size (input vectors per step)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/batch
for b in "$@"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --warmup 1 --steps 2 --batch $b > gpurun_out/batch/b$b.log 2>&1 || { tail gpurun_out/batch/b$b.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/batch/b$b.log').read().strip().splitlines()[-1]); print('B=$b', d['value'], d['ms_per_step'])"
done
