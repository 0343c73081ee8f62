#!/bin/bash
# Batch / lane sweep of the cfg3 bench (no profile step, no CPU baseline).  usage: bash tools/gpu_lanes.sh <tag> "<B>:<lanes>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
for cfg in "$@"; do
  B=${cfg%%:*}; NL=${cfg#*:}
  HEC_LANES=$NL timeout -k 10 300 python bench.py --batch $B --no-cpu-baseline --no-profile > gpurun_out/$T/b${B}_l${NL}.json 2> gpurun_out/$T/b${B}_l${NL}.err || { tail gpurun_out/$T/b${B}_l${NL}.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/$T/b${B}_l${NL}.json').read().strip().splitlines()[-1]); print('B=$B lanes=$NL', d['value'], d['ms_per_step'])"
done
