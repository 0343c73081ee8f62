#!/bin/bash
# round-4 box: build the demo, the new he_math GPU tests first, then the GPU suite, then one bench line (no CPU leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04a
timeout -k 10 300 python -u -m pytest tests/test_gpu_he_math.py tests/test_gpu_encode.py tests/test_gpu_seal_io.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04a/new_tests.log 2>&1 || { tail -40 gpurun_out/r04a/new_tests.log; exit 1; }
tail -3 gpurun_out/r04a/new_tests.log
bash tools/gpu_tests.sh r04a || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err || { tail gpurun_out/r04a/bench.err; exit 1; }
tail -1 gpurun_out/r04a/bench.json | cut -c1-400
