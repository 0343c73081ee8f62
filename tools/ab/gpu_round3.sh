#!/bin/bash
# Second half of a round measurement: SQ counters (gpu_sq.sh), the cfg5 bench and a one-rank torchrun of the
# sharded mode (RCCL path).  usage: bash tools/gpu_round3.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r02}
mkdir -p gpurun_out/$T
bash tools/gpu_sq.sh ${T}_sq || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --config cfg5 --no-cpu-baseline > gpurun_out/$T/cfg5_bench.json 2> gpurun_out/$T/cfg5_bench.err || { tail gpurun_out/$T/cfg5_bench.err; exit 1; }
tail -1 gpurun_out/$T/cfg5_bench.json | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --mode sharded --steps 1 --warmup 1 --no-cpu-baseline --batch 32 > gpurun_out/$T/sharded1.json 2> gpurun_out/$T/sharded1.err || { tail gpurun_out/$T/sharded1.err; exit 1; }
tail -1 gpurun_out/$T/sharded1.json | cut -c1-300
