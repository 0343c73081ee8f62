#!/bin/bash
# SQ counters (8-slot passes, each its own run) for the dominant kernels on a short bench run at the bench batch:
# one step, one lane, n = 512 diagonals (every kernel of the full step, fewer launches).  Then tools/sq_summary.py.
# usage: [KRE=<kernel regex>] [SQ_B=<batch>] bash tools/gpu_sq.sh <tag>
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq}
B=${SQ_B:-192}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HEC_LANES=1  # one lane: per-kernel counters of whole-batch launches
RE="${KRE:-k_fan|k_bmac|k_ntt|k_hmacm|k_tensor}"
ARGS="--n 512 --batch $B --no-cpu-baseline --no-profile --no-self-check --steps 1 --warmup 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "$RE" --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p1.log 2>&1 || { tail $OUT/p1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64 --kernel-include-regex "$RE" --output-format csv -d $OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p2.log 2>&1 || { tail $OUT/p2.log; exit 1; }
ls $OUT/p1 $OUT/p2
