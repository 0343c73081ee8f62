#!/bin/bash
# Round-4 measurement set on the final kernels: A/B against the pre-pairs build, the profile set (bench with CPU
# baseline, rocprofv3 kernel trace, FETCH/WRITE PMC passes), cfg2, and the world-1 sharded (cfg4) line.
# usage: bash tools/gpu_r04e.sh <tag> <variant .so>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
bash tools/gpu_abn.sh $T head=$2 || exit 1
bash tools/gpu_profile.sh ${T}_prof || exit 1
timeout -k 10 300 python bench.py --config cfg2 > gpurun_out/$T/cfg2.json 2> gpurun_out/$T/cfg2.err || { tail gpurun_out/$T/cfg2.err; exit 1; }
tail -1 gpurun_out/$T/cfg2.json | cut -c1-400
timeout -k 10 400 python bench.py --mode sharded --no-cpu-baseline > gpurun_out/$T/sharded1.json 2> gpurun_out/$T/sharded1.err || { tail gpurun_out/$T/sharded1.err; exit 1; }
tail -1 gpurun_out/$T/sharded1.json | cut -c1-600
