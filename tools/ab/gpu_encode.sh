#!/bin/bash
# GPU encoder + cfg5-parameter parity, then the whole GPU suite, then a short ct x pt bench (GPU-encoded diagonals)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_parity.py::test_cfg5_params_matvec_bitexact -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_encode.log 2>&1 || { tail -40 gpurun_out/gpu_encode.log; exit 1; }
tail -3 gpurun_out/gpu_encode.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --variant ctpt --no-cpu-baseline --batch 32 > gpurun_out/ctpt.log 2>&1 || { tail -20 gpurun_out/ctpt.log; exit 1; }
tail -1 gpurun_out/ctpt.log | cut -c1-300
