#!/bin/bash
# A/B of one engine switch: the hoisted/key-switch parity subset under the switch, then the bench without and with it.
# usage: bash tools/gpu_ab_env.sh <tag> "ENV=VALUE"   (development tool)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; E=$2
mkdir -p gpurun_out/$T
env $E timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or cfg5_params or rescale or matvec" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/base.json 2> gpurun_out/$T/base.err || exit 1
env $E timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/var.json 2> gpurun_out/$T/var.err || exit 1
echo "base $(head -c 110 gpurun_out/$T/base.json)"
echo "$E $(head -c 110 gpurun_out/$T/var.json)"
