#!/bin/bash
# Experiment: throughput of two concurrent bench processes (B=16 each) vs one process at B=16 / B=32.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/conc
A="--no-cpu-baseline --no-profile --warmup 1"
timeout -k 10 200 python bench.py $A --batch 32 --steps 3 > gpurun_out/conc/s32.log 2>&1 || exit 1
timeout -k 10 200 python bench.py $A --batch 16 --steps 3 > gpurun_out/conc/s16.log 2>&1 || exit 1
timeout -k 10 300 python bench.py $A --batch 16 --steps 8 > gpurun_out/conc/p1.log 2>&1 &
P1=$!
timeout -k 10 300 python bench.py $A --batch 16 --steps 8 > gpurun_out/conc/p2.log 2>&1 &
P2=$!
wait $P1 || exit 1
wait $P2 || exit 1
for f in s32 s16 p1 p2; do python -c "import json,sys; d=json.loads(open('gpurun_out/conc/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'])"; done
