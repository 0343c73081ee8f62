#!/bin/bash
# GPU parity: the full-size tests first (long oracle runs), then the rest of the -m gpu suite.
# usage: bash tools/gpu_tests.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
t=${1:-r03}
timeout -k 10 720 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -s --timeout 600 --timeout-method thread > gpurun_out/gpu_full_$t.log 2>&1 || { tail -40 gpurun_out/gpu_full_$t.log; exit 1; }
tail -3 gpurun_out/gpu_full_$t.log
timeout -k 10 450 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --deselect tests/test_gpu_fullsize.py > gpurun_out/gpu_tests_$t.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$t.log; exit 1; }
tail -3 gpurun_out/gpu_tests_$t.log
