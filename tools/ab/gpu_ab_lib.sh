#!/bin/bash
# A/B of an experiment library (tools/variant_lib.sh): the key-switch parity subset on the variant, then the bench on
# the in-tree libhecdna.so and on the variant, then SQ LDS counters of one kernel for both (development tool).
# usage: bash tools/gpu_ab_lib.sh <tag> <variant .so> [kernel regex for the SQ pass]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; V=$(realpath $2); K=$3
mkdir -p gpurun_out/$T
HECDNA_LIB=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "keyswitch_variants or hoisted or cfg3 or cfg5 or rescale or matvec or ntt" > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -1 gpurun_out/$T/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/base.json 2> gpurun_out/$T/base.err || exit 1
HECDNA_LIB=$V timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/$T/var.json 2> gpurun_out/$T/var.err || exit 1
echo "base $(head -c 110 gpurun_out/$T/base.json)"
echo "var  $(head -c 110 gpurun_out/$T/var.json)"
if [ -n "$K" ]; then
  cd /tmp && export TMPDIR=/tmp HEC_LANES=1
  for side in base var; do
    L=""; [ $side = var ] && L=$V
    HECDNA_LIB=$L timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "$K" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$T/sq_$side -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 512 --no-cpu-baseline --no-profile --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/gpurun_out/$T/sq_$side.log 2>&1 || { tail $GRAFT_REPO_ROOT/gpurun_out/$T/sq_$side.log; exit 1; }
  done
fi
