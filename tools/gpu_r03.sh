#!/bin/bash
# Round-3 A/B: the bench with the fused hoisted MAC (default) against the per-pair path and another batch tile,
# then the whole GPU suite.  usage: bash tools/gpu_r03.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r03}
mkdir -p gpurun_out/$T
B="python bench.py --no-cpu-baseline --steps 2 --warmup 1"
timeout -k 10 300 $B --sharded-steps 1 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || { tail gpurun_out/$T/bench.err; exit 1; }
head -c 700 gpurun_out/$T/bench.json; echo
HEC_HFUSE=0 timeout -k 10 300 $B > gpurun_out/$T/bench_nofuse.json 2> gpurun_out/$T/bench_nofuse.err || { tail gpurun_out/$T/bench_nofuse.err; exit 1; }
head -c 300 gpurun_out/$T/bench_nofuse.json; echo
HEC_HFUSE_BG=4 timeout -k 10 300 $B > gpurun_out/$T/bench_bg4.json 2> gpurun_out/$T/bench_bg4.err || { tail gpurun_out/$T/bench_bg4.err; exit 1; }
head -c 300 gpurun_out/$T/bench_bg4.json; echo
bash tools/gpu_tests.sh $T
