#!/bin/bash
# Final round measurement on the in-tree build: full GPU suite + smoke, then the profile set at B = 192.
# usage: bash tools/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
bash tools/gpu_suite.sh $T || exit 1
PMC_DIMS="192 15 10 4096" bash tools/gpu_profile.sh ${T}_prof > /dev/null || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_prof/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline'])"
