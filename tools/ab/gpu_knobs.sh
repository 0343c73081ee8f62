#!/bin/bash
# Engine-knob sweep of the cfg3 bench (no profile step, no CPU baseline).
# usage: bash tools/gpu_knobs.sh <tag> "<VAR=VAL[,VAR=VAL...]>" ...   ("-" = defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=""
  [ "$spec" != "-" ] && envs=$(echo "$spec" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/$T/k$i.json 2> gpurun_out/$T/k$i.err || { tail gpurun_out/$T/k$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/$T/k$i.json').read().strip().splitlines()[-1]); print('$spec', d['value'], d['ms_per_step'])"
done
