#!/bin/bash
# The other bench configurations on the in-tree build: ct x pt diagonals (cfg3') and the cfg5 matmul.
# usage: bash tools/gpu_cfgs.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 400 python bench.py --variant ctpt --no-cpu-baseline > gpurun_out/$T/ctpt.json 2> gpurun_out/$T/ctpt.err || { tail gpurun_out/$T/ctpt.err; exit 1; }
tail -1 gpurun_out/$T/ctpt.json | cut -c1-300
timeout -k 10 700 python bench.py --config cfg5 --no-cpu-baseline > gpurun_out/$T/cfg5.json 2> gpurun_out/$T/cfg5.err || { tail gpurun_out/$T/cfg5.err; exit 1; }
tail -1 gpurun_out/$T/cfg5.json | cut -c1-300
