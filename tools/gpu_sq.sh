#!/bin/bash
# SQ counters (one pass, 8 slots) for the dominant kernels on a small bench run
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HEC_LANES=1  # one lane: per-kernel counters of whole-batch launches
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "${KRE:-k_fan|k_bmac|k_ntt|k_hmacm|k_tensor}" --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 512 --no-cpu-baseline --no-profile --steps 1 --warmup 0 > $OUT/p1.log 2>&1 || { tail $OUT/p1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MUL_F64 --kernel-include-regex "${KRE:-k_fan|k_bmac|k_ntt|k_hmacm|k_tensor}" --output-format csv -d $OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 512 --no-cpu-baseline --no-profile --steps 1 --warmup 0 > $OUT/p2.log 2>&1 || { tail $OUT/p2.log; exit 1; }
ls $OUT/p1 $OUT/p2
