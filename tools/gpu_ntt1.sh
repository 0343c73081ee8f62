#!/bin/bash
# single-pass NTT experiment: parity with HEC_NTT1=1, then NTT micro-benchmark 2-pass vs 1-pass
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
HEC_NTT1=1 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "ntt or cfg3_rotations" -x -q --timeout 120 --timeout-method thread > gpurun_out/ntt1_tests.log 2>&1 || { tail -30 gpurun_out/ntt1_tests.log; exit 1; }
tail -1 gpurun_out/ntt1_tests.log
HEC_NTT1=0 timeout -k 10 120 python tools/ntt_bench.py > gpurun_out/ntt_bench0.log 2>&1 || { tail gpurun_out/ntt_bench0.log; exit 1; }
HEC_NTT1=1 timeout -k 10 120 python tools/ntt_bench.py > gpurun_out/ntt_bench1.log 2>&1 || { tail gpurun_out/ntt_bench1.log; exit 1; }
grep logN gpurun_out/ntt_bench0.log; grep logN gpurun_out/ntt_bench1.log
