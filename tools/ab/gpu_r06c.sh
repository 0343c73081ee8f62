#!/bin/bash
# round 6: SQ counters of k_hmacm, in-tree (MAC-form loop) vs variants/base_r06.so, B = 128
set -o pipefail
cd $GRAFT_REPO_ROOT
KRE=k_hmacm SQ_B=128 bash tools/gpu_sq.sh r06c_new > /dev/null || exit 1
HECDNA_LIB=$(realpath variants/base_r06.so) KRE=k_hmacm SQ_B=128 bash tools/gpu_sq.sh r06c_base > /dev/null || exit 1
for v in new base; do
  SQ_BY_INSTANCE=1 python tools/sq_summary.py gpurun_out/r06c_$v/p1/run_counter_collection.csv gpurun_out/r06c_$v/p2/run_counter_collection.csv "tools/gpu_sq.sh k_hmacm B=128 ($v)" > gpurun_out/r06c_$v/sq.json || exit 1
done
