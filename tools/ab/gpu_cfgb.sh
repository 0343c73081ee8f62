#!/bin/bash
# Batch sweep of the non-metric configurations (cfg2, cfg5).  usage: bash tools/gpu_cfgb.sh <tag> "<cfg>:<batch>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out/$T
for spec in "$@"; do
  C=${spec%%:*}; B=${spec#*:}
  timeout -k 10 400 python bench.py --config $C --batch $B --no-cpu-baseline > gpurun_out/$T/${C}_b$B.json 2> gpurun_out/$T/${C}_b$B.err || { tail gpurun_out/$T/${C}_b$B.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/$T/${C}_b$B.json').read().strip().splitlines()[-1]); print('$spec', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
done
