#!/bin/bash
# GPU parity suite then the round-end measurement (bench + rocprof stats + PMC passes).
# usage: bash tools/gpu_round.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu_profile.sh ${1:-r01}
