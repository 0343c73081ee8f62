#!/bin/bash
# Round-end measurement: bench line (with CPU baseline), rocprofv3 kernel-trace stats of the same
# workload, and FETCH_SIZE / WRITE_SIZE PMC passes (separate passes, gfx950 slot limits) on k_bmac.
# usage: bash tools/gpu_profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_bmac --output-format csv -d $OUT/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 256 --no-cpu-baseline --no-profile --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1 || { tail $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_bmac --output-format csv -d $OUT/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n 256 --no-cpu-baseline --no-profile --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1 || { tail $OUT/pmc_write.log; exit 1; }
find $OUT -name "*.csv" | head -20
