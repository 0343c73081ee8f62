#!/bin/bash
# Full GPU test suite (one process) and smoke() on the in-tree build.  usage: bash tools/gpu_suite.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -2 gpurun_out/$T/smoke.log
