#!/bin/bash
# The other bench modes at the default batch: ct x pt diagonals, and the row-sharded (cfg4) leg at world 1.
# usage: bash tools/gpu_modes.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python bench.py --variant ctpt --no-cpu-baseline > gpurun_out/$T/ctpt.json 2> gpurun_out/$T/ctpt.err || { tail gpurun_out/$T/ctpt.err; exit 1; }
tail -1 gpurun_out/$T/ctpt.json | cut -c1-250
timeout -k 10 500 python bench.py --mode sharded --no-cpu-baseline > gpurun_out/$T/sharded1.json 2> gpurun_out/$T/sharded1.err || { tail gpurun_out/$T/sharded1.err; exit 1; }
tail -1 gpurun_out/$T/sharded1.json | cut -c1-250
python3 -c "
import json; d=json.loads(open('gpurun_out/$T/sharded1.json').read().strip().splitlines()[-1]); print(d.get('sharded'), d['roofline']['frac'])"
