#!/bin/bash
# N-way A/B (tools/gpu_abn.sh) followed by the two SQ-counter passes on the in-tree build, summarised per
# kernel instantiation.  usage: bash tools/gpu_abq.sh <tag> <name>=<variant .so> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
bash tools/gpu_abn.sh "$@" || exit 1
bash tools/gpu_sq.sh ${T}_sq > /dev/null || exit 1
SQ_BY_INSTANCE=1 python tools/sq_summary.py gpurun_out/${T}_sq/p1/run_counter_collection.csv gpurun_out/${T}_sq/p2/run_counter_collection.csv "tools/gpu_sq.sh (bench --n 512, HEC_LANES=1)" > gpurun_out/${T}_sq/sq_by_instance.json
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_sq/sq_by_instance.json'))
for k, v in d['kernels'].items(): print(k[:90], v.get('dispatches'), v.get('wait_any_frac'), v.get('valu_active_frac'), round(v.get('SQ_WAVE_CYCLES', 0) / max(1, v.get('SQ_WAVES', 1))))"
